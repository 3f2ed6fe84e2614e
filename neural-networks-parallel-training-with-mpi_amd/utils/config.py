"""Configuration and CLI.

Compatible flags (reference ``ref.py:244-253``): ``--lr`` (0.001), ``--momentum`` (0.9),
``--batch_size`` (reference default 4, never used), ``--nepochs`` (3).  Defects fixed here
(SURVEY.md §2.7):

* D6 — ``--lr``/``--momentum`` are typed floats (the reference passes strings to SGD).
* D7 — ``--batch_size`` defaults to ``None`` = whole shard (the reference's effective
  behaviour, ``ref.py:146``); an explicit value is honoured as a per-rank mini-batch.
* D12 — widths, sample/feature counts, noise, seeds are configurable; defaults equal the
  reference constants (``ref.py:42-44,72``).
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional

REFERENCE_WIDTHS = (2, 3, 1)

# Named model/data presets.  "ref" is the reference config (ref.py:41-45,72); "proxy512" is the
# 512-wide proxy the reference algorithm was measured on; "wide8192" and "mnist"
# are the BASELINE.json north-star configs 4 and 5.
PRESETS = {
    "ref": dict(widths=[2, 3, 1], n_samples=16, n_features=2, activation="relu", loss="mse",
                dtype="fp32"),
    "proxy512": dict(widths=[512, 512, 512, 512, 1], n_samples=8192, n_features=512,
                     activation="relu", loss="mse", dtype="bf16"),
    "mlp512x3": dict(widths=[512, 512, 512, 1], n_samples=8192, n_features=512,
                     activation="relu", loss="mse", dtype="bf16"),
    "wide8192": dict(widths=[8192, 8192, 8192, 8192, 8192, 1], n_samples=4096,
                     n_features=8192, activation="relu", loss="mse", dtype="bf16"),
    "mnist": dict(widths=[784, 1024, 1024, 10], n_samples=8192, n_features=784,
                  activation="relu", loss="xent", dtype="bf16"),
}


@dataclass
class TrainConfig:
    # --- reference flags ---
    lr: float = 0.001
    momentum: float = 0.9
    batch_size: Optional[int] = None  # None = full shard (reference behaviour)
    nepochs: int = 3
    # --- model ---
    widths: List[int] = field(default_factory=lambda: list(REFERENCE_WIDTHS))
    activation: str = "relu"          # relu | tanh
    loss: str = "mse"                 # mse | xent
    dtype: str = "fp32"               # fp32 | bf16 (compute dtype; master weights stay fp32)
    # --- optimizer extras (torch.optim.SGD semantics) ---
    dampening: float = 0.0
    weight_decay: float = 0.0
    nesterov: bool = False
    # --- data ---
    n_samples: int = 16
    n_features: Optional[int] = None  # defaults to widths[0]
    noise: float = 1.0
    data_seed: int = 42
    data_gen: str = "auto"            # auto | sklearn | device
    data_dist: str = "scatter"        # scatter | replicate | local
    scaling: str = "per_shard"        # per_shard (reference, D4) | global | none
    averaging: str = "unweighted"     # unweighted (reference, D5) | weighted
    shuffle: bool = True
    val_fraction: float = 0.0         # held-out tail of every shard, evaluated after each epoch
    grad_accum: int = 1               # micro-batches per optimizer step (gradient accumulation)
    # --- runtime ---
    seed: int = 0                     # init seed (reference: torch.manual_seed(0) on rank 0)
    device: str = "auto"              # auto (cuda when a GPU is visible) | cpu | cuda
    comm: str = "auto"                # auto | native (RCCL) | torch (torch.distributed) |
                                      # gloo (gloo even for device tensors) | none
    sync: str = "allreduce"           # allreduce | root (reference-style reduce+bcast)
    comm_mode: str = "auto"           # auto | overlap (comm stream) | inline (compute stream) |
                                      # overlap_rowband (the row-band step, comm stream)
    bucket_mb: float = 1.0
    overlap: bool = True
    graph: bool = True                # capture the steady-state step in a HIP graph
    fast_epochs: bool = True          # full-batch GPU epochs replayed 64 per graph (same output)
    grad_dtype: str = "fp32"          # fp32 | bf16 | auto (all-reduce payload dtype; fp32 as the
                                      # reference averages fp32 gradients, ref.py:185-208; auto:
                                      # bf16 above 64 MB of fp32 gradient on the GPU, as bench.py)
    shard_optimizer: bool = False     # ZeRO-1: reduce-scatter grads, SGD on own 1/P, all-gather
    deterministic: bool = True
    # --- IO / observability ---
    print_rank: str = "all"           # all | 0 | none
    global_loss: bool = False
    metrics_json: Optional[str] = None
    checkpoint: Optional[str] = None
    checkpoint_every: int = 0
    resume: Optional[str] = None
    timeout_s: float = 300.0
    seqcheck: bool = False
    profile_steps: bool = False
    ref_samples_per_s: Optional[float] = None   # 1-GPU samples/s -> parallel efficiency metric
    nprocs: int = 0                   # >0: self-spawn this many ranks when not under a launcher

    def __post_init__(self):
        if self.n_features is None:
            self.n_features = self.widths[0]

    def replace(self, **kw) -> "TrainConfig":
        return dataclasses.replace(self, **kw)


def _widths(s: str) -> List[int]:
    return [int(x) for x in s.replace("x", ",").split(",") if x.strip()]


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train network across multiple distributed processes.")
    # reference-compatible flags (ref.py:245-252) — same names & defaults, typed (D6, D7)
    p.add_argument("--lr", dest="lr", type=float, default=0.001,
                   help="Learning rate for SGD optimizer. [0.001]")
    p.add_argument("--momentum", dest="momentum", type=float, default=0.9,
                   help="Momentum for SGD optimizer [0.9].")
    p.add_argument("--batch_size", dest="batch_size", type=int, default=None,
                   help="Per-process mini-batch size. Default: the whole shard (reference "
                        "behaviour; the reference parses this flag but never uses it).")
    p.add_argument("--nepochs", dest="nepochs", type=int, default=3,
                   help="Number of epochs (times to loop through the dataset).")
    # extensions
    p.add_argument("--preset", choices=sorted(PRESETS), default=None,
                   help="model/data preset (overrides widths/samples/features/act/loss/dtype)")
    p.add_argument("--widths", type=_widths, default=None, help="layer widths, e.g. 2,3,1")
    p.add_argument("--activation", choices=["relu", "tanh"], default=None)
    p.add_argument("--loss", choices=["mse", "xent"], default=None)
    p.add_argument("--dtype", choices=["fp32", "bf16"], default=None)
    p.add_argument("--dampening", type=float, default=0.0)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--nesterov", action="store_true")
    p.add_argument("--n_samples", type=int, default=None)
    p.add_argument("--n_features", type=int, default=None)
    p.add_argument("--noise", type=float, default=1.0)
    p.add_argument("--data_seed", type=int, default=42)
    p.add_argument("--data_gen", choices=["auto", "sklearn", "device"], default="auto")
    p.add_argument("--data_dist", choices=["scatter", "replicate", "local"], default="scatter")
    p.add_argument("--scaling", choices=["per_shard", "global", "none"], default="per_shard")
    p.add_argument("--averaging", choices=["unweighted", "weighted"], default="unweighted")
    p.add_argument("--no_shuffle", dest="shuffle", action="store_false")
    p.add_argument("--val_fraction", type=float, default=0.0,
                   help="hold out this fraction of every rank's rows and print the global "
                        "validation loss after each epoch (the reference's dead x_val/y_val hook)")
    p.add_argument("--grad_accum", "--accum_steps", dest="grad_accum", type=int, default=1,
                   help="micro-batches whose gradients are summed before one synchronisation + "
                        "optimizer step (with the whole-shard batch the shard is cut into this "
                        "many micro-batches)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto",
                   help="auto: the MI355X (HIP kernels + RCCL) when a GPU is visible, else the "
                        "CPU/gloo path")
    p.add_argument("--comm", choices=["auto", "torch", "native", "gloo", "none"], default="auto",
                   help="gradient transport: native = the C++ RCCL runtime (GPU default), torch = "
                        "torch.distributed (nccl on GPU, gloo on CPU), gloo = gloo also for "
                        "device tensors (several ranks sharing one GPU)")
    p.add_argument("--sync", choices=["allreduce", "root"], default="allreduce")
    p.add_argument("--comm_mode", choices=["auto", "overlap", "inline", "overlap_rowband"],
                   default="auto")
    p.add_argument("--bucket_mb", type=float, default=1.0)
    p.add_argument("--no_overlap", dest="overlap", action="store_false")
    p.add_argument("--no_graph", dest="graph", action="store_false")
    p.add_argument("--no_fast_epochs", dest="fast_epochs", action="store_false",
                   help="one graph replay + loss readback per epoch (default: 64 epochs per "
                        "replay, losses recorded on the device; identical output)")
    p.add_argument("--grad_dtype", choices=["auto", "fp32", "bf16"], default="fp32",
                   help="all-reduce payload (default fp32, the reference's gradients); auto = "
                        "bf16 above 64 MB of fp32 gradient on the GPU (one-rounding reduction, "
                        "see parallel/sync.py) -- the bench's choice")
    p.add_argument("--shard_optimizer", "--zero1", dest="shard_optimizer", action="store_true",
                   help="sharded optimizer state (ZeRO-1): reduce-scatter gradients, SGD on this "
                        "rank's 1/P of the parameters, all-gather the updated parameters")
    p.add_argument("--nondeterministic", dest="deterministic", action="store_false")
    p.add_argument("--print_rank", choices=["all", "0", "none"], default="all")
    p.add_argument("--global_loss", action="store_true")
    p.add_argument("--metrics_json", default=None)
    p.add_argument("--checkpoint", default=None)
    p.add_argument("--checkpoint_every", type=int, default=0)
    p.add_argument("--resume", default=None)
    p.add_argument("--timeout_s", type=float, default=300.0)
    p.add_argument("--seqcheck", action="store_true")
    p.add_argument("--profile_steps", action="store_true")
    p.add_argument("--ref_samples_per_s", type=float, default=None,
                   help="single-GPU samples/s of the same per-rank work: the JSON metrics then "
                        "carry parallel_efficiency = samples_per_s / (world * this)")
    p.add_argument("--nprocs", type=int, default=0,
                   help="self-spawn N ranks (when not launched by mpiexec/torchrun)")
    return p


def config_from_args(args) -> TrainConfig:
    """Build a :class:`TrainConfig` from an argparse namespace (or any attribute object).

    Accepts objects that carry only the reference's four attributes: string-typed ``lr`` /
    ``momentum`` (reference D6) are coerced to float.
    """
    if isinstance(args, TrainConfig):
        return args
    g = lambda k, d=None: getattr(args, k, d)  # noqa: E731
    base = TrainConfig()
    kw = {}
    preset = g("preset")
    if preset:
        kw.update(PRESETS[preset])
    for k in ("widths", "activation", "loss", "dtype", "n_samples", "n_features"):
        v = g(k)
        if v is not None:
            kw[k] = v
    for f in dataclasses.fields(TrainConfig):
        if f.name in kw or f.name in ("widths", "activation", "loss", "dtype", "n_samples",
                                      "n_features"):
            continue
        v = g(f.name, None)
        if v is not None:
            kw[f.name] = v
    kw["lr"] = float(kw.get("lr", base.lr))
    kw["momentum"] = float(kw.get("momentum", base.momentum))
    bs = kw.get("batch_size")
    kw["batch_size"] = None if bs in (None, "", 0) else int(bs)
    kw["nepochs"] = int(kw.get("nepochs", base.nepochs))
    if "widths" in kw and "n_features" not in kw:
        kw["n_features"] = kw["widths"][0]
    cfg = TrainConfig(**kw)
    validate(cfg)
    return cfg


def resolve_device(device: str, local_world: int = 1) -> str:
    """``auto`` -> ``cuda`` when every local rank can have a GPU of its own (RCCL refuses two
    ranks on one device), else ``cpu``: ``mpiexec -n 4`` on a 1-GPU node runs the CPU/gloo path
    as the reference does.  ``device_count()`` does not initialise the HIP runtime, so a
    launcher process may call this before it spawns its ranks."""
    if device != "auto":
        return device
    import torch
    n = torch.cuda.device_count()
    return "cuda" if n > 0 and local_world <= n else "cpu"


def validate(cfg: TrainConfig) -> None:
    """Fail fast before any collective."""
    if cfg.grad_dtype not in ("auto", "fp32", "bf16"):
        raise ValueError(f"grad_dtype must be auto, fp32 or bf16, got {cfg.grad_dtype!r}")
    if cfg.device not in ("auto", "cpu", "cuda"):
        raise ValueError(f"device must be auto, cpu or cuda, got {cfg.device!r}")
    if len(cfg.widths) < 2:
        raise ValueError(f"widths needs >= 2 entries, got {cfg.widths}")
    if cfg.n_features != cfg.widths[0]:
        raise ValueError(f"n_features={cfg.n_features} != widths[0]={cfg.widths[0]}")
    if cfg.activation not in ("relu", "tanh"):
        raise ValueError(cfg.activation)
    if cfg.loss not in ("mse", "xent"):
        raise ValueError(cfg.loss)
    if cfg.loss == "xent" and cfg.widths[-1] < 2:
        raise ValueError("xent needs >= 2 output classes")
    if cfg.dtype not in ("fp32", "bf16"):
        raise ValueError(cfg.dtype)
    if cfg.nesterov and (cfg.momentum <= 0 or cfg.dampening != 0):
        raise ValueError("Nesterov momentum requires a momentum and zero dampening")
    if cfg.lr < 0 or cfg.momentum < 0 or cfg.weight_decay < 0:
        raise ValueError("lr, momentum and weight_decay must be >= 0")
    if cfg.batch_size is not None and cfg.batch_size <= 0:
        raise ValueError("batch_size must be positive")
    if cfg.n_samples <= 0:
        raise ValueError("n_samples must be positive")
    if not 0.0 <= cfg.val_fraction < 1.0:
        raise ValueError("val_fraction must be in [0, 1)")
    if int(cfg.grad_accum) < 1:
        raise ValueError("grad_accum must be >= 1")

"""``dist_train`` — the end-to-end training job (reference ``ref.py:56-236``).

Per rank:
  1. discover rank/world from the launcher environment, rendezvous (gloo control plane);
  2. build the dataset and distribute rows (reference: rank 0 ``make_regression`` +
     ``Scatter``/``Scatterv``, ref.py:66-143) — here with int64 counts, any world size, empty
     shards allowed (D1-D3 fixed); per-shard (reference) or global feature scaling;
  3. initialise the model on rank 0 with ``torch.manual_seed(0)`` (ref.py:69,84) and broadcast it
     (ref.py:87-88) into the flat arena that backs the model's parameters;
  4. run the epoch loop: one optimizer step per batch (full shard by default, ref.py:146),
     gradients synchronised by bucketed all-reduce, fused SGD-momentum; print the reference's
     two log lines (ref.py:152,224);
  5. optionally checkpoint (reference-format state_dict) / resume, emit JSON metrics.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
import sys
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from ..data import synth
from ..data.dataset import RegressionDataset, scale_features
from ..data.partition import partition_rows
from ..models.mlp import MLP, MLPSpec, reference_init
from ..parallel import dist as pdist
from ..parallel.sync import (NativeRcclSync, NoSync, ShardedSync, TorchDistSync, make_shm_sync,
                             shm_sync_ok)
from ..utils import checkpoint as ckpt
from ..utils.config import TrainConfig, config_from_args, resolve_device
from ..utils.metrics import MetricsWriter, comm_bus_gbps, comm_volume, parallel_efficiency
from ..utils.seqcheck import SequenceChecker
from ..utils.watchdog import Watchdog
from .arena import Arena
from .engine import MLPEngine

SKLEARN_MAX_ELEMS = 4_000_000
# Below this gradient volume the all-reduce is latency-bound and is issued inline on the compute
# stream (no cross-HW-queue dependencies; see parallel/sync.py); above it buckets overlap backward.
INLINE_MAX_GRAD_BYTES = 64 << 20
HOST_INIT_MAX_PARAMS = 20_000_000

FAST_EPOCHS = 64   # epochs per replayed graph on the fast full-batch path


@dataclass
class TrainResult:
    rank: int
    world: int
    losses: List[float] = field(default_factory=list)        # local loss per epoch (printed)
    global_losses: List[float] = field(default_factory=list)
    val_losses: List[float] = field(default_factory=list)      # global, per epoch
    final_params: Optional[torch.Tensor] = None               # forward-order flat, fp32 CPU
    state_dict: Optional[dict] = None
    rows: int = 0
    epoch_times: List[float] = field(default_factory=list)
    steps: int = 0
    phase_ms: Optional[dict] = None   # --profile_steps: mean ms per step per phase
    schedule: Optional[dict] = None   # what the engine chose: payload, sync, grouped/deferred


def dist_train(args) -> Optional[TrainResult]:
    cfg = config_from_args(args)
    if cfg.nprocs and cfg.nprocs > 1 and not pdist.under_launcher():
        pdist.spawn(_spawn_worker, cfg.nprocs, cfg)
        return None
    return run_worker(cfg)


def _spawn_worker(cfg: TrainConfig):
    run_worker(cfg)


# --------------------------------------------------------------------------------------------
class Job:
    """Everything a rank needs for the run (built by :func:`setup`)."""

    def __init__(self, cfg: TrainConfig):
        self.cfg = cfg
        self.job = pdist.detect_job()
        self.rank, self.world = self.job.rank, self.job.world
        self.device = torch.device("cpu")
        if resolve_device(cfg.device, self.job.local_world) == "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("--device cuda requested but no GPU is visible")
            ndev = torch.cuda.device_count()
            torch.cuda.set_device(self.job.local_rank % ndev)
            self.device = torch.device("cuda", torch.cuda.current_device())
        comm = cfg.comm
        if comm == "auto":
            comm = "native" if self.device.type == "cuda" else "torch"
        if self.world == 1 and cfg.comm != "native":
            comm = "none"   # (an explicit --comm native keeps a 1-rank RCCL communicator: testing)
        self.comm_kind = comm
        self.pg = pdist.ProcessGroupContext(self.job, cfg.timeout_s,
                                            want_nccl=(comm == "torch" and self.device.type == "cuda"))
        self.native_comm = None
        if comm == "native":
            from .. import native
            lib = native.lib()
            uid = lib.rccl_unique_id() if self.rank == 0 else None
            uid = self.pg.broadcast_object(uid, 0)
            self.native_comm = native.make_comm(uid, self.world, self.rank, self.device.index)

    def close(self):
        self.native_comm = None
        self.pg.destroy()


def _compute_dtype(cfg: TrainConfig):
    return torch.bfloat16 if cfg.dtype == "bf16" else torch.float32


def build_shard(j: Job):
    """Return (X fp32 [rows, in] on device, Y fp32 [rows, out] or labels int64, partition)."""
    cfg, rank, world = j.cfg, j.rank, j.world
    part = partition_rows(cfg.n_samples, world)
    rows = part.rows(rank)
    start = part.start(rank)
    out_f = cfg.widths[-1]
    small = cfg.n_samples * cfg.n_features <= SKLEARN_MAX_ELEMS
    use_sklearn = cfg.loss == "mse" and out_f == 1 and (
        cfg.data_gen == "sklearn" or (cfg.data_gen == "auto" and small))
    labels = None
    if use_sklearn:
        if cfg.data_dist == "scatter" and world > 1:
            XY = None
            if rank == 0:
                X, y = synth.reference_regression(cfg.n_samples, cfg.n_features, cfg.noise, cfg.data_seed)
                XY = synth.as_xy_matrix(X, y)
            shard = _scatter_rows(j, XY, part, cfg.n_features + 1)
        else:
            X, y = synth.reference_regression(cfg.n_samples, cfg.n_features, cfg.noise, cfg.data_seed)
            shard = synth.as_xy_matrix(X, y)[part.slice(rank)]
        Xs, ys = shard[:, :cfg.n_features], shard[:, cfg.n_features]
        # RegressionDataset semantics (ref.py:145): per-shard StandardScaler on float64
        if cfg.scaling == "per_shard":
            ds = RegressionDataset(Xs, ys, scale_data=True)
            Xt = ds.X
        else:
            Xt = scale_features(torch.from_numpy(np.ascontiguousarray(Xs)), cfg.scaling,
                                allreduce=lambda t: j.pg.allreduce_cpu(t))
        Xt = Xt.to(torch.float32)                       # the reference's .float() (ref.py:159)
        Yt = torch.from_numpy(np.ascontiguousarray(ys)).to(torch.float32).reshape(-1, 1)
        return Xt.to(j.device), Yt.to(j.device), None, part
    gen_dev = j.device
    if cfg.loss == "xent":
        X, labels = synth.chunked_classification(start, rows, cfg.n_features, out_f,
                                                 seed=cfg.data_seed, device=gen_dev)
        Y = None
    else:
        X, Y = synth.chunked_regression(start, rows, cfg.n_features, cfg.noise,
                                        seed=cfg.data_seed, out=out_f, device=gen_dev)
    if cfg.scaling != "none":
        def ar(t):
            tc = t.cpu()
            j.pg.allreduce_cpu(tc)
            t.copy_(tc)
        X = scale_features(X, cfg.scaling, allreduce=ar)
    return X, Y, labels, part


def _scatter_rows(j: Job, XY, part, width: int) -> np.ndarray:
    """Reference Scatter/Scatterv (ref.py:108,138): over RCCL (grouped ncclSend/ncclRecv with
    per-rank int64 counts and displacements, device to device) when the native communicator is
    up, else over gloo (padded equal chunks, trimmed)."""
    if j.native_comm is not None:
        return _scatter_rows_native(j, XY, part, width)
    import torch.distributed as dist
    mx = max(1, part.max_rows)
    recv = torch.zeros(mx, width, dtype=torch.float64)
    chunks = None
    if j.rank == 0:
        t = torch.from_numpy(np.ascontiguousarray(XY))
        chunks = []
        for r in range(j.world):
            c = torch.zeros(mx, width, dtype=torch.float64)
            n = part.rows(r)
            if n:
                c[:n] = t[part.slice(r)]
            chunks.append(c)
    dist.scatter(recv, chunks, src=0, group=j.pg.gloo)
    return recv[: part.rows(j.rank)].numpy()


def _scatter_rows_native(j: Job, XY, part, width: int) -> np.ndarray:
    counts = [part.rows(r) * width for r in range(j.world)]
    displs = [part.start(r) * width for r in range(j.world)]
    recv = torch.zeros(max(1, counts[j.rank]), dtype=torch.float64, device=j.device)
    if j.rank == 0:
        send = torch.from_numpy(np.ascontiguousarray(XY)).to(j.device).reshape(-1)
    else:
        send = recv          # not read on non-root ranks
    s = torch.cuda.current_stream()
    j.native_comm.scatterv(send.data_ptr(), counts, displs, recv.data_ptr(), 2, 0,
                           int(s.cuda_stream))
    s.synchronize()
    return recv[:counts[j.rank]].view(-1, width).cpu().numpy()


def init_model(j: Job, spec: MLPSpec) -> MLP:
    cfg = j.cfg
    big = spec.n_params > HOST_INIT_MAX_PARAMS and j.device.type == "cuda"
    model = reference_init(spec.widths, spec.activation, seed=cfg.seed,
                           device=j.device if big else None)
    return model


def broadcast_params(j: Job, arena: Arena):
    """Rank 0's parameters to every rank (reference ref.py:87-88 bcast(state_dict))."""
    if j.world == 1:
        return
    if j.native_comm is not None:
        from .. import native
        s = torch.cuda.current_stream()
        j.native_comm.broadcast(arena.master.data_ptr(), arena.numel, 0, 0, int(s.cuda_stream))
        s.synchronize()
    elif j.device.type == "cuda" and j.pg.nccl is not None:
        import torch.distributed as dist
        dist.broadcast(arena.master, src=0, group=j.pg.nccl)
    else:
        import torch.distributed as dist
        t = arena.master.cpu() if j.device.type != "cpu" else arena.master
        dist.broadcast(t, src=0, group=j.pg.gloo)
        if t is not arena.master:
            arena.master.copy_(t)
    arena.sync_shadow()


def grad_payload(cfg: TrainConfig, device_type: str, numel: int) -> str:
    """The all-reduce payload dtype: ``auto`` is bf16 on the GPU above INLINE_MAX_GRAD_BYTES of
    fp32 gradient (the bandwidth-bound regime; same rule as bench.py), fp32 otherwise."""
    if cfg.grad_dtype != "auto":
        return cfg.grad_dtype
    return "bf16" if (device_type == "cuda" and numel * 4 > INLINE_MAX_GRAD_BYTES
                      and not cfg.shard_optimizer) else "fp32"


def make_sync(j: Job, arena: Arena):
    cfg = j.cfg
    if j.comm_kind == "none":
        return NoSync(arena)
    grad_dtype = grad_payload(cfg, j.device.type, arena.numel)
    if cfg.shard_optimizer:
        if cfg.sync == "root" or grad_dtype != "fp32":
            raise ValueError("--shard_optimizer reduce-scatters fp32 gradients "
                             "(no --sync root / --grad_dtype bf16)")
        if j.comm_kind == "native":
            return ShardedSync(arena, j.world, j.rank, native_comm=j.native_comm)
        group = j.pg.nccl if (j.device.type == "cuda" and j.pg.nccl is not None) else j.pg.gloo
        return ShardedSync(arena, j.world, j.rank, group=group)
    if (j.comm_kind in ("torch", "gloo") and
            shm_sync_ok(j.device.type, j.world, j.job.local_world, grad_dtype, cfg.sync)):
        shm = make_shm_sync(arena, j.pg.gloo, j.world, j.rank, timeout_s=cfg.timeout_s)
        if shm is not None:
            return shm
    if j.comm_kind == "native":
        inline = (cfg.comm_mode == "inline" or
                  (cfg.comm_mode == "auto" and arena.numel * 4 <= INLINE_MAX_GRAD_BYTES))
        return NativeRcclSync(arena, j.native_comm, j.world, inline=inline,
                              grad_dtype=grad_dtype, mode=cfg.sync)
    group = (j.pg.nccl if (j.device.type == "cuda" and j.pg.nccl is not None
                           and j.comm_kind != "gloo") else j.pg.gloo)
    return TorchDistSync(arena, group, j.world, mode=cfg.sync, overlap=cfg.overlap,
                         grad_dtype=grad_dtype)


def make_ops(j: Job):
    if j.device.type == "cuda":
        from ..ops.hip_ops import HipOps
        return HipOps(j.device)
    from ..ops.torch_ops import TorchOps
    return cpu_ops(j.device)


def cpu_ops(device):
    """CPU op set: native host steps for tiny models when the native library loads (HostOps),
    else the plain-PyTorch oracle (TorchOps)."""
    from ..ops.torch_ops import TorchOps
    try:
        from ..ops.host_ops import HostOps, host_ops_enabled
        if host_ops_enabled():
            return HostOps(device)
    except (ImportError, OSError, RuntimeError):
        pass
    return TorchOps(device)


def loss_scales(cfg: TrainConfig, rows_local: int, rows_all: List[int], out_f: int):
    """(inv_count, loss_scale, grad_scale) for one step."""
    per = out_f if cfg.loss == "mse" else 1
    loss_scale = 1.0 / (max(rows_local, 1) * per)
    nonempty = sum(1 for r in rows_all if r > 0) or 1
    if cfg.averaging == "weighted":
        tot = sum(rows_all)
        return 1.0 / (max(tot, 1) * per), loss_scale, 1.0
    return loss_scale, loss_scale, 1.0 / nonempty


def _gather_state(eng, sync):
    """Sharded optimizer: re-assemble the full fp32 master + momentum on every rank (collective)."""
    if getattr(sync, "sharded", False):
        eng.synchronize()
        sync.gather_state()


def _comm_only_ms(j: "Job", sync, reps: int = 10) -> float:
    """Milliseconds per repetition of one step's gradient collectives alone (same buckets,
    dtype and order; max over ranks)."""
    cuda = j.device.type == "cuda"

    def sync_dev():
        if cuda:
            torch.cuda.synchronize()
    sync.comm_only()           # warm-up (RCCL sets up channels lazily)
    sync_dev()
    j.pg.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        sync.comm_only()
    sync_dev()
    el = torch.tensor([(time.perf_counter() - t0) / reps * 1e3], dtype=torch.float64)
    import torch.distributed as dist
    j.pg.allreduce_cpu(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def _fault_injection(rank: int) -> Optional[int]:
    """``NNMPI_FAULT_INJECT=<rank>:<epoch>``: that rank raises at the start of that epoch while
    its peers are blocked in the step's collectives -- the reference's deadlock scenario
    (ref.py:185,203), used by the failure-detection test."""
    spec = os.environ.get("NNMPI_FAULT_INJECT")
    if not spec:
        return None
    r, e = spec.split(":")
    return int(e) if int(r) == rank else None


def _print(cfg: TrainConfig, rank: int, msg: str):
    if cfg.print_rank == "all" or (cfg.print_rank == "0" and rank == 0):
        print(msg, flush=True)


def run_worker(cfg: TrainConfig) -> TrainResult:
    j = Job(cfg)
    try:
        return _run(j)
    finally:
        j.close()


def _warn_ignored_knobs(rank: int):
    """An NNMPI_* experiment knob in the environment without NNMPI_EXPERIMENTS=1 selects
    nothing (utils/knobs.py): say so once (rank 0, stderr) instead of ignoring it silently."""
    from ..utils import knobs
    ignored = sorted(k for k, v in knobs.seen().items() if not v["honoured"])
    if ignored and rank == 0:
        print(f"[nnmpi_amd] warning: {', '.join(ignored)} set but not honoured (experiment knobs "
              f"need {knobs.EXPERIMENTS}=1)", file=sys.stderr, flush=True)
    return ignored


def _run(j: Job) -> TrainResult:
    cfg, rank, world = j.cfg, j.rank, j.world
    _warn_ignored_knobs(rank)
    spec = MLPSpec(tuple(cfg.widths), cfg.activation, cfg.loss)
    X, Y, labels, part = build_shard(j)
    # held-out validation rows: the tail of every shard (same rule on every rank, so the
    # training row counts used for loss scaling are known everywhere)
    n_val = lambda c: int(round(c * cfg.val_fraction))  # noqa: E731
    train_counts = [c - n_val(c) for c in part.counts]
    nv = n_val(X.shape[0])
    if nv:
        cut = X.shape[0] - nv
        Xv, Yv = X[cut:], (Y[cut:] if Y is not None else None)
        Lv = labels[cut:] if labels is not None else None
        X, Y = X[:cut], (Y[:cut] if Y is not None else None)
        labels = labels[:cut] if labels is not None else None
    else:
        Xv = Yv = Lv = None
    rows_local = X.shape[0]
    model = init_model(j, spec)
    dtype = _compute_dtype(cfg)
    sharded = cfg.shard_optimizer and j.comm_kind != "none"
    arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], j.device,
                  shadow_dtype=torch.bfloat16 if dtype == torch.bfloat16 else None,
                  bucket_bytes=cfg.bucket_mb * 2 ** 20, pad_to=64 * world if sharded else 64)
    arena.bind_model(model)
    broadcast_params(j, arena)
    start_epoch, steps_done = 0, 0
    if cfg.resume:
        start_epoch, steps_done = ckpt.load_training_state(cfg.resume, arena)
    sync = make_sync(j, arena)
    ops = make_ops(j)
    bs = cfg.batch_size
    max_rows = max(train_counts)
    K = max(1, int(cfg.grad_accum))
    # micro-batch size (every rank uses the same one, so every rank runs the same number of
    # micro-batches and optimizer steps; a short shard gets empty micro-batches)
    mb = bs if bs else (max(1, math.ceil(max_rows / K)) if K > 1 else None)
    cap = min(mb, max_rows) if mb else max_rows
    eng = MLPEngine(spec, arena, ops, sync, device=j.device, dtype=dtype,
                    rowband_overlap=cfg.comm_mode == "overlap_rowband",
                    rows_capacity=max(cap, 1), lr=cfg.lr, momentum=cfg.momentum,
                    dampening=cfg.dampening, weight_decay=cfg.weight_decay,
                    nesterov=cfg.nesterov, use_graph=cfg.graph, overlap=cfg.overlap)
    eng.steps_done = steps_done
    if cfg.profile_steps:
        from ..utils.metrics import EventTimer
        eng.timer = EventTimer(j.device.type)
    Xc = X.to(dtype)
    metrics = MetricsWriter(cfg.metrics_json if rank == 0 else None)
    cvol = comm_volume(arena.numel, world, grad_payload(cfg, j.device.type, arena.numel),
                       sharded=getattr(sync, "sharded", False),
                       shadow=arena.shadow is not None)
    seqchk = SequenceChecker(j.pg) if cfg.seqcheck else None
    if seqchk is not None:
        seqchk.check_plan(sync)      # before any gradient collective
    wd = Watchdog(cfg.timeout_s, j.native_comm) if world > 1 else None
    res = TrainResult(rank, world, rows=rows_local)
    res.schedule = {"device": j.device.type, "comm": j.comm_kind, "sync": type(sync).__name__,
                    "grad_dtype": grad_payload(cfg, j.device.type, arena.numel),
                    "inline": bool(getattr(sync, "inline", False)),
                    "grouped": bool(eng.grouped), "rowband": eng.uses_rowband(rows_local),
                    "deferred_updates": len(eng._defer_plan),
                    "graph": bool(eng.use_graph)}
    n_micro = max(1, math.ceil(max_rows / mb)) if mb else 1
    steps_per_epoch = math.ceil(n_micro / K) if K > 1 else (1 if not bs else n_micro)

    def micro_rows(c: int, m: int) -> int:
        return max(0, min(mb, c - m * mb))
    gen = torch.Generator(device="cpu")
    full_loaded = False
    fault = _fault_injection(rank)
    # Full-shard epochs with nothing per epoch but the two output lines (the reference's own
    # loop, ref.py:150-224): replay FAST_EPOCHS epochs per graph, each step recording its loss
    # on the device, and print the lines after each replay -- same lines, same order, same
    # values, one host sync per replay instead of per epoch.
    # mini-batch epochs (--batch_size): every epoch one graph replay of all its steps
    mb_graph = (cfg.fast_epochs and j.device.type == "cuda" and eng.use_graph
                and eng.timer is None and bool(bs) and K == 1)
    perm_dev = None
    fast = (cfg.fast_epochs and j.device.type == "cuda" and eng.use_graph and eng.timer is None and not bs and K == 1
            and not (cfg.global_loss and world > 1) and cfg.val_fraction == 0 and seqchk is None
            and not (cfg.checkpoint and cfg.checkpoint_every) and fault is None)
    try:
        if fast:
            eng.load_batch(Xc, Y, labels)
            eng.set_scales(*loss_scales(cfg, eng.rows, list(train_counts), cfg.widths[-1]))
            hist = torch.zeros(FAST_EPOCHS, dtype=torch.float32, device=j.device)
            epoch = start_epoch
            # epochs per replay: the watchdog is kicked once per replay, so with several ranks a
            # replay must stay well inside timeout_s -- start small, then size it (a power of two,
            # so only a few graphs are ever captured) from the measured epoch time
            per_replay = 4 if wd else FAST_EPOCHS
            while epoch < cfg.nepochs:
                c = min(per_replay, cfg.nepochs - epoch)
                t0 = time.perf_counter()
                eng.run_steps(c, c, losses=hist)
                eng.synchronize()            # the losses are written on the engine's stream
                vals = hist[:c].tolist()
                dt = (time.perf_counter() - t0) / c
                if wd:
                    wd.kick()
                    fit = int(0.25 * cfg.timeout_s / max(dt, 1e-9))
                    per_replay = max(1, min(FAST_EPOCHS, 1 << max(0, fit.bit_length() - 1)))
                for k in range(c):
                    _print(cfg, rank, "[ = = = = = Epoch {} = = = = = ]".format(epoch + k))
                    res.losses.append(vals[k])
                    res.epoch_times.append(dt)
                    _print(cfg, rank, f"loss in worker {rank}: {vals[k]}")
                    sps = sum(train_counts) / dt if dt > 0 else None
                    metrics.write(epoch=epoch + k, loss=vals[k], epoch_s=dt, steps=1,
                                  samples_per_s=sps, world=world,
                                  parallel_efficiency=parallel_efficiency(sps, world,
                                                                          cfg.ref_samples_per_s),
                                  **cvol, val_loss=None)
                epoch += c
        for epoch in range(start_epoch, cfg.nepochs if not fast else start_epoch):
            if fault is not None and epoch == fault:
                raise RuntimeError(f"injected fault on rank {rank} at epoch {epoch}")
            _print(cfg, rank, "[ = = = = = Epoch {} = = = = = ]".format(epoch))
            t0 = time.perf_counter()
            if bs and cfg.shuffle:
                gen.manual_seed(cfg.seed * 1000003 + rank * 7919 + epoch)
                perm = torch.randperm(rows_local, generator=gen).to(j.device)
            else:
                perm = None
            for s in range(steps_per_epoch):
                if K > 1:
                    micros = range(s * K, min((s + 1) * K, n_micro))
                    rows_all = [sum(micro_rows(c, m) for m in micros) for c in train_counts]
                    inv, lsc, gsc = loss_scales(cfg, rows_all[rank], rows_all, cfg.widths[-1])
                    eng.set_scales(inv, lsc, gsc)
                    for m in micros:
                        lo, hi = m * mb, m * mb + micro_rows(rows_local, m)
                        idx = (perm[lo:hi] if perm is not None
                               else torch.arange(lo, hi, device=j.device))
                        eng.load_batch_indexed(Xc, Y, labels, idx.contiguous())
                        eng.accumulate()
                    eng.apply_accumulated()
                    step_rows = rows_all[rank]
                    if wd:
                        wd.kick()
                    continue
                if not bs:
                    if not full_loaded:  # full-shard batch: order-irrelevant, uploaded once (D10)
                        eng.load_batch(Xc, Y, labels)
                        full_loaded = True
                    rows_all = list(train_counts)
                else:
                    if mb_graph and s == 0 and eng.steps_done > 0:
                        # the whole epoch's mini-batches as one graph replay (same gathers,
                        # scales and steps as the per-step branch below)
                        if perm_dev is None:
                            perm_dev = torch.empty(rows_local, dtype=torch.int64, device=j.device)
                        with torch.cuda.stream(eng.stream):
                            perm_dev.copy_(perm if perm is not None else
                                           torch.arange(rows_local, device=j.device))
                        plan = []
                        for s2 in range(steps_per_epoch):
                            lo, hi = s2 * bs, min((s2 + 1) * bs, rows_local)
                            ra = [max(0, min(bs, c - s2 * bs)) for c in train_counts]
                            plan.append((lo, max(lo, hi)) + tuple(
                                loss_scales(cfg, max(0, hi - lo), ra, cfg.widths[-1])))
                        eng.run_epoch(Xc, Y, labels, perm_dev, plan)
                        step_rows = eng.rows
                        if wd:
                            wd.kick()
                        break
                    lo, hi = s * bs, min((s + 1) * bs, rows_local)
                    idx = perm[lo:hi] if perm is not None else torch.arange(lo, max(lo, hi), device=j.device)
                    eng.load_batch_indexed(Xc, Y, labels, idx.contiguous())
                    rows_all = [max(0, min(bs, c - s * bs)) for c in train_counts]
                inv, lsc, gsc = loss_scales(cfg, eng.rows, rows_all, cfg.widths[-1])
                eng.set_scales(inv, lsc, gsc)
                eng.step()
                step_rows = eng.rows
                if wd:
                    wd.kick()
            loss = eng.loss()
            dt = time.perf_counter() - t0
            res.losses.append(loss)
            res.epoch_times.append(dt)
            _print(cfg, rank, f"loss in worker {rank}: {loss}")
            if cfg.global_loss and world > 1:
                t = torch.tensor([loss * step_rows, float(step_rows)], dtype=torch.float64)
                j.pg.allreduce_cpu(t)
                gl = float(t[0] / max(t[1], 1.0))
                res.global_losses.append(gl)
                _print(cfg, rank, f"global loss: {gl}") if rank == 0 else None
            if cfg.val_fraction > 0:
                vs, vn = eng.evaluate(Xv.to(dtype), Yv, Lv) if Xv is not None else (0.0, 0)
                full_loaded = False          # evaluation reused the input buffers
                per = cfg.widths[-1] if cfg.loss == "mse" else 1
                t = torch.tensor([vs, float(vn)], dtype=torch.float64)
                if world > 1:
                    j.pg.allreduce_cpu(t)
                vl = float(t[0] / max(float(t[1]) * per, 1.0))
                res.val_losses.append(vl)
                _print(cfg, rank, f"validation loss: {vl}") if rank == 0 else None
            if seqchk:
                seqchk.check(epoch, sync.seq, sync.sig)
            sps = sum(train_counts) / dt if dt > 0 else None
            metrics.write(epoch=epoch, loss=loss, epoch_s=dt, steps=steps_per_epoch,
                          samples_per_s=sps, world=world,
                          parallel_efficiency=parallel_efficiency(sps, world,
                                                                  cfg.ref_samples_per_s),
                          **cvol, val_loss=res.val_losses[-1] if res.val_losses else None)
            if cfg.checkpoint and cfg.checkpoint_every and (epoch + 1) % cfg.checkpoint_every == 0:
                _gather_state(eng, sync)
                if rank == 0:
                    ckpt.save(cfg.checkpoint, arena, epoch + 1, eng.steps_done, cfg)
                j.pg.barrier()
        eng.synchronize()
        res.steps = eng.steps_done
        if eng.timer is not None:
            res.phase_ms = eng.timer.summary_ms()
            _print(cfg, rank, "[profile] mean ms per step: " +
                   ", ".join(f"{k} {v:.4f}" for k, v in res.phase_ms.items()))
            # the phase times come from eagerly launched, event-bracketed steps (a replayed
            # graph has no host-visible phase boundaries); the bus bandwidth is NOT derived from
            # them -- in the overlapped schedule "bwd->comm" is only the join tail -- but from
            # the step's collectives timed alone
            comm_ms = _comm_only_ms(j, sync) if world > 1 else None
            metrics.write(profile_ms_per_step=res.phase_ms, phase_timing="eager", rank=rank,
                          comm_only_ms=comm_ms,
                          comm_bus_GBps=comm_bus_gbps(cvol["wire_bytes_per_rank"], comm_ms))
        _gather_state(eng, sync)
        if cfg.checkpoint and rank == 0:
            ckpt.save(cfg.checkpoint, arena, cfg.nepochs, eng.steps_done, cfg)
        res.final_params = arena.flat_params_forward_order().detach().cpu().clone()
        res.state_dict = {k: v.cpu() for k, v in arena.state_dict().items()}
        j.pg.barrier()
    finally:
        if wd:
            wd.stop()
        metrics.close()
    return res

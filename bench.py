"""Headline benchmark: whole-job training throughput (samples/s) of the MLP regression step.

Config (BASELINE.json / BASELINE.md): the reference algorithm's 512-wide proxy — MLP
512 -> 512 -> 512 -> 512 -> 1 (ReLU, MSE), 8192 rows per GPU, full-shard batch (one optimizer
step per epoch, as the reference's DataLoader does, ref.py:146), SGD momentum 0.9, bf16 compute
with fp32 master weights; synthetic make_regression-style data generated on device, random
init.  Weak scaling: every GPU keeps 8192 rows, except that with N > 1 the global row count is
8192*N - 1, so the split is uneven (BASELINE config 3: the last rank holds one row less).  The
short rank only leaves a partial last tile; a LONG rank (8192 + 1 rows) would add a whole extra
row of GEMM tiles on that rank and, since the step time is the max over ranks, slow every rank
down.  Gradients are all-reduced over RCCL (xGMI) every step.

Launch (the reference: ``mpiexec -n N python ...``, README.md:12, ref.py:61-63):

    python bench.py --gpus N [--steps K] [--warmup W]     # spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Without a launcher, ``--gpus N > 1`` starts N fresh rank processes (before anything touches
the GPU in this one) and exits with the worst of their exit codes.  Under a launcher the
launched world must equal ``--gpus``, and a GPU run needs one visible device per local rank:
anything else exits non-zero instead of measuring a different job.

Gradient-sync schedule (``--comm_mode``, default auto): for latency-bound gradient volumes the
fastest schedule depends on the node's collective latency, so the candidates (one inline
all-reduce; ZeRO-1 reduce-scatter + sharded SGD + bf16 all-gather; per-bucket all-reduce on a
comm stream overlapped with backward) are each timed for ``--tune_steps`` steps BEFORE the timed
region and the fastest (max over ranks, so every rank agrees) is kept; its time per candidate
is reported in ``config.comm_tune_ms_per_step``.  Large gradients (bf16 payload above 64 MB,
``--grad_dtype auto``) are tuned too, overlap first: RCCL's all-reduce kernels hold CUs
(256 threads, ~280 registers per wave, read from the gfx950 code object) that a one-wave
256x256 GEMM launch needs, so on a real node whether the overlapped schedule beats one inline
all-reduce is measured, not assumed.

Rank 0 prints ONE JSON line.  The timed region is exactly K full training steps (forward,
loss, backward, gradient all-reduce, optimizer update), bracketed by barrier + device sync on
both sides; the reported time is the max over ranks.  AFTER the timed region (``--no_extras``
skips it) the same ranks measure, each for min(K, 50) steps: the step with the gradient sync
switched off (= the single-GPU step of the same shard: parallel efficiency, exposed comm), the
step's collectives alone (bus GB/s, overlap %), and the step at a fixed global batch equal to
the 1-GPU dataset (8192 rows for the proxy: strong scaling, the reference's own scaling mode,
BASELINE.md:36-39).

``--device cpu`` runs the same job on the CPU/gloo path (BASELINE config 1 plumbing): the
multi-rank logic of this script is tested that way without a GPU.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Reference numbers (reference algorithm on the 512-wide proxy, CPU, samples/s;
# strong scaling of a fixed 8192-row dataset)
BASELINE_SAMPLES_PER_S = {1: 32190.0, 2: 61546.0, 4: 88657.0, 8: 105377.0}
# below this gradient volume the all-reduce is latency-bound: issue it inline (see parallel/sync.py)
INLINE_MAX_GRAD_BYTES = 64 << 20
EXTRA_STEPS = 50
# untimed warm-up tops up to this much continuous step work on the GPU (DVFS ramp; see warm())
MIN_WARM_MS = 30.0
WARM_CHUNK = 16

CONFIGS = {
    "proxy512": dict(widths=[512, 512, 512, 512, 1], loss="mse", rows=8192,
                     model="mlp_512x4_regression(512-512-512-512-1)"),
    "mlp512x3": dict(widths=[512, 512, 512, 1], loss="mse", rows=8192,
                     model="mlp_512x3_regression(512-512-512-1)"),
    "wide8192": dict(widths=[8192] * 5 + [1], loss="mse", rows=4096,
                     model="mlp_8192x4_regression(8192x4-1)"),
    # mid-size: a bf16 all-reduce payload (> 64 MB of fp32 gradient) on a model small enough
    # for multi-rank rehearsals on one GPU
    "wide2048": dict(widths=[2048] * 5 + [1], loss="mse", rows=2048,
                     model="mlp_2048x4_regression(2048x4-1)"),
    "mnist": dict(widths=[784, 1024, 1024, 10], loss="xent", rows=8192,
                  model="mlp_mnist_shape(784-1024-1024-10,xent)"),
    # the reference config itself: fp32 like the reference (whole step in one tiny-MLP kernel)
    "ref": dict(widths=[2, 3, 1], loss="mse", rows=16, model="mlp_reference(2-3-1)", dtype="fp32"),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); > 1 without a launcher: spawn them")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="proxy512", choices=sorted(CONFIGS))
    p.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto",
                   help="cpu: the CPU/gloo plumbing path (no GPU)")
    p.add_argument("--rows", type=int, default=None, help="rows per GPU (weak scaling)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--comm", choices=["native", "torch"], default="native")
    p.add_argument("--grad_dtype", choices=["auto", "fp32", "bf16"], default="auto",
                   help="all-reduce payload (auto: bf16 above 64 MB of fp32 gradients)")
    p.add_argument("--bucket_mb", type=float, default=1.0)
    p.add_argument("--chunk_tiles", type=int, default=0,
                   help="256x256 weight-gradient tiles per output-row chunk bucket at least "
                        "(0: 256 = 4 chunks per 8192-wide layer; 512: 2 chunks)")
    p.add_argument("--no_graph", action="store_true")
    p.add_argument("--no_overlap", action="store_true")
    p.add_argument("--no_group", action="store_true",
                   help="separate dgrad / wgrad / combine launches instead of the grouped one")
    p.add_argument("--even", action="store_true", help="no uneven extra rows")
    p.add_argument("--graph_chunk", type=int, default=0,
                   help="steps per replayed hipGraph (1 = one graph launch per step; 0 = auto: "
                        "each run of n steps as few graphs as possible, at most 128 steps each)")
    p.add_argument("--lr", type=float, default=1e-5)
    p.add_argument("--comm_mode", choices=["auto", "tune", "overlap", "inline", "zero1",
                                           "overlap_rowband"],
                   default="auto",
                   help="overlap: per-bucket all-reduce on a comm stream + per-bucket SGD; "
                        "inline: one all-reduce on the compute stream; zero1: reduce-scatter + "
                        "sharded SGD + bf16 all-gather; tune: time all three before the timed "
                        "region and keep the fastest (auto: tune for small gradient volumes, "
                        "overlap for large)")
    p.add_argument("--tune_steps", type=int, default=32,
                   help="steps per candidate timing in --comm_mode tune (untimed region)")
    p.add_argument("--force_comm", action="store_true",
                   help="use the RCCL gradient path even with one rank (smoke-tests comm overlap)")
    p.add_argument("--no_extras", action="store_true",
                   help="skip the post-timed-region efficiency / overlap / strong-scaling runs")
    p.add_argument("--shared_gpu_rehearsal", action="store_true",
                   help="TESTING ONLY: let the N ranks share the visible GPU(s) (each rank its own "
                        "NCCL_HOSTID, RCCL over loopback) to rehearse the multi-rank code path on "
                        "a 1-GPU box; the JSON line says so and its numbers are not a measurement")
    p.add_argument("--fwd_variant", type=int, default=-1, help="forward GEMM variant (experiments)")
    p.add_argument("--gemm_variant", type=int, default=0,
                   help="GEMM main-loop variant of every launch (experiments; 19..24 = deep-ring "
                        "256x256, needs an NNMPI_BUILD_EXPERIMENTS=1 build)")
    p.add_argument("--pp_order", default="",
                   help="256x256 GEMM kernel for fwd,dgrad,wgrad (0 GM4, 1 row-major, 2 GM4 + one "
                        "DMA half per phase, 3 row-major + one half per phase; experiments)")
    p.add_argument("--head_xcd_rows", type=int, default=0,
                   help="head kernels take XCD-remapped row blocks (experiments)")
    p.add_argument("--store_policy", type=int, default=0,
                   help="GEMM epilogue output stores: 0 plain, 1 nt, 2 sc1 (experiments)")
    p.add_argument("--group_async", type=int, default=-1,
                   help="grouped-backward LDS read mode (experiments)")
    return p.parse_args(argv)


EXPERIMENT_FLAGS = {"fwd_variant": -1, "gemm_variant": 0, "pp_order": "", "head_xcd_rows": 0,
                    "store_policy": 0, "group_async": -1}


def knobs_report(a) -> dict:
    """What could make this run differ from the default configuration: every NNMPI_* variable in
    the environment and every non-default experiment flag, each with whether it took effect
    (experiment knobs count only with NNMPI_EXPERIMENTS=1, nnmpi_amd/utils/knobs.py)."""
    from nnmpi_amd.utils import knobs
    out = {"experiments": knobs.experiments(), "env": knobs.seen(), "flags": {}}
    for k, d in EXPERIMENT_FLAGS.items():
        v = getattr(a, k)
        if v != d:
            out["flags"][k] = {"value": v, "honoured": knobs.experiments()}
    return out


def _free_port() -> int:
    from nnmpi_amd.parallel.dist import free_port
    return free_port()


def _fail(msg: str, code: int = 2):
    print(f"[bench] error: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


def launch_ranks(a, argv) -> int:
    """Start ``--gpus`` rank processes of this script (nothing in this process has touched the
    GPU: ``device_count()`` does not initialise HIP) and return the worst exit code."""
    n = a.gpus
    if a.device != "cpu":
        import torch
        have = torch.cuda.device_count()
        if have < n and not (a.device == "auto" and have == 0) and not a.shared_gpu_rehearsal:
            _fail(f"--gpus {n} needs {n} visible GPUs, this node shows {have}")
        if a.device == "auto" and have == 0:
            a.device = "cpu"
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   NNMPI_LAUNCHER="bench")
        if a.device == "cpu":
            env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // n)))
        if a.shared_gpu_rehearsal:
            # RCCL refuses two ranks on one device unless they look like different hosts
            env.update(NCCL_HOSTID=f"nnmpi-rehearsal-{r}", NCCL_SOCKET_IFNAME="lo",
                       NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    first_bad = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                rc = p.poll()
                if rc is None:
                    continue
                pending.remove(p)
                if rc != 0 and not first_bad:
                    first_bad = rc if rc > 0 else 1
                    for q in pending:      # one rank failed: its peers cannot finish
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return first_bad


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    import torch  # noqa: F401  (import only: does not initialise HIP)
    import nnmpi_amd  # noqa: F401
    from nnmpi_amd.parallel import dist as pdist

    job = pdist.detect_job()
    if job.launcher == "single" and a.gpus > 1:
        sys.exit(launch_ranks(a, argv))
    if job.world != a.gpus:
        _fail(f"launched with {job.world} rank(s) but --gpus {a.gpus}: refusing to report a "
              "different job")
    if a.device == "auto":
        a.device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    if a.device == "cuda":
        have = torch.cuda.device_count()
        # a launcher may hand every rank exactly one device through a visibility variable
        # (then each rank sees 1 GPU and uses it); otherwise fewer GPUs than local ranks is
        # refused before anything runs
        isolated = have == 1 and any(os.environ.get(v) for v in (
            "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"))
        if have < job.local_world and not isolated and not a.shared_gpu_rehearsal:
            _fail(f"{job.local_world} local ranks need as many GPUs; {have} visible "
                  "(one rank per GPU: RCCL refuses two ranks on one device)")
    from nnmpi_amd.parallel import supervisor as sup
    # (supervise only where the supervisors' rendezvous is shared by every rank: a TCP store at
    # MASTER_ADDR, or -- for a plain mpiexec -- all ranks on this node, which share the
    # launcher's FileStore; a multi-node mpiexec without MASTER_* runs unsupervised)
    if (job.world > 1 and not sup.supervised() and sup.rendezvous_shared(job.world, job.local_world)
            and os.environ.get("NNMPI_BENCH_SUPERVISE", "1") != "0"):
        # this process never touches the GPU: it runs the rank as a child and retries the whole
        # job in fresh processes with a more conservative schedule if any rank dies or hangs
        sys.exit(supervise(a, argv, job))
    run(a, job)


def fallback_ladder(a, argv):
    """The argv of every attempt: as launched, then the origin-stream inline all-reduce (one
    collective on the compute stream, the capture form measured to work at P = 2..8), then the
    same without hipGraphs."""
    ladder = [("as launched", [])]
    if a.comm_mode != "inline":
        ladder.append(("--comm_mode inline", ["--comm_mode", "inline"]))
    if a.device != "cpu" and not a.no_graph:
        ladder.append(("--comm_mode inline --no_graph", ["--comm_mode", "inline", "--no_graph"]))
    n = int(os.environ.get("NNMPI_BENCH_ATTEMPTS", len(ladder)))
    return [(d, [sys.executable, os.path.abspath(__file__)] + list(argv) + extra)
            for d, extra in ladder[:max(1, n)]]


def supervise(a, argv, job) -> int:
    from nnmpi_amd.parallel.supervisor import Supervisor
    ladder = fallback_ladder(a, argv)
    s = Supervisor(job.rank, job.world, stall_s=float(os.environ.get("NNMPI_BENCH_STALL_S", 300)))

    def annotate(line, log):
        first_fail = next((f for e in log for f in (e["failures"] or [])), None)
        # set when the measurement comes from a retry: why the first attempt was abandoned
        line["fallback"] = first_fail if len(log) > 1 else None
        line["attempts"] = log
        line["measured_mode"] = log[-1]["mode"]
        return line
    env = {}
    if a.shared_gpu_rehearsal:
        # (as launch_ranks does for its own ranks: RCCL accepts two ranks on one device only if
        # they look like different hosts)
        env = dict(NCCL_HOSTID=f"nnmpi-rehearsal-{job.rank}", NCCL_SOCKET_IFNAME="lo",
                   NCCL_IB_DISABLE="1")
    return s.run([cmd for _, cmd in ladder], lambda k: ladder[k][0], annotate, env_extra=env)


def run(a, job):
    import torch
    import torch.distributed as dist
    from nnmpi_amd.data import synth
    from nnmpi_amd.data.partition import partition_rows
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.engine.trainer import loss_scales
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.parallel import dist as pdist
    from nnmpi_amd.parallel.sync import (NativeRcclSync, NoSync, ShardedSync, TorchDistSync,
                                         make_shm_sync, shm_sync_ok)
    from nnmpi_amd.parallel.supervisor import supervised, write_result
    from nnmpi_amd.utils.config import TrainConfig
    from nnmpi_amd.utils.metrics import comm_volume, scaling_report

    rank, world = job.rank, job.world
    milestone = _milestones(rank)
    gpu = a.device == "cuda"
    if gpu:
        from nnmpi_amd import native
        # kernel-selection experiment flags: honoured only with NNMPI_EXPERIMENTS=1 (the native
        # knobs ignore them otherwise); the JSON line reports them either way
        native.lib().set_fwd_variant(a.fwd_variant)
        native.lib().set_gemm_variant(a.gemm_variant)
        for epi, idx in enumerate(a.pp_order.split(",") if a.pp_order else []):
            native.lib().set_pp256_order(epi, int(idx))
        native.lib().set_group_async(a.group_async)
        native.lib().set_store_policy(a.store_policy)
        native.lib().set_head_xcd_rows(a.head_xcd_rows)
        torch.cuda.set_device(job.local_rank % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
        from nnmpi_amd.ops.hip_ops import HipOps
        make_ops = lambda: HipOps(dev)  # noqa: E731
    else:
        dev = torch.device("cpu")
        from nnmpi_amd.engine.trainer import cpu_ops
        make_ops = lambda: cpu_ops(dev)  # noqa: E731
        a.comm = "torch"
    pg = pdist.ProcessGroupContext(job, 600.0, want_nccl=(gpu and a.comm == "torch" and world > 1))
    milestone("rendezvous")
    c = CONFIGS[a.config]
    widths = c["widths"]
    spec = MLPSpec(tuple(widths), "relu", c["loss"])
    if "dtype" in c:
        a.dtype = c["dtype"]
    if not gpu:
        a.dtype = "fp32"
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    rows_pg = a.rows or c["rows"]
    grad_bytes = spec.n_params * 4
    grad_dtype = a.grad_dtype
    if grad_dtype == "auto":
        grad_dtype = "bf16" if (gpu and grad_bytes > INLINE_MAX_GRAD_BYTES) else "fp32"
    big = spec.n_params > 20_000_000
    use_comm = (world > 1 or (a.force_comm and gpu))
    native_comm = None
    if use_comm and gpu and a.comm == "native":
        lib = native.lib()
        uid = pg.broadcast_object(lib.rccl_unique_id() if rank == 0 else None, 0)
        native_comm = native.make_comm(uid, world, rank, dev.index)
    milestone("communicator")
    comm_group = pg.nccl if (gpu and pg.nccl is not None) else pg.gloo

    def shard(n_global):
        part = partition_rows(n_global, world)
        rows = part.rows(rank)
        if c["loss"] == "xent":
            X, labels = synth.chunked_classification(part.start(rank), rows, widths[0], widths[-1],
                                                     device=dev)
            Y = None
        else:
            X, Y = synth.chunked_regression(part.start(rank), rows, widths[0], device=dev)
            labels = None
        return part, X.to(dtype), Y, labels

    def build(mode, data, comm=True, bucket_mb=None, chunk_tiles=0, bf16_reduce=None, gdt=None):
        """One arena + gradient-sync strategy + engine over ``data`` (a shard()).
        mode: inline | overlap | overlap_rowband | zero1 | none (no gradient synchronisation);
        chunk_tiles: 256x256 tiles per output-row chunk bucket at least (0: the default);
        bf16_reduce: the all-reduce algorithm, "rccl" for RCCL's own ring / tree (None: the
        default -- acc32 for a bf16 payload, ordered for an fp32 one); gdt: the gradient payload
        dtype of this candidate (None: the job's)."""
        gdt = gdt or grad_dtype
        part, X, Y, labels = data
        rows = part.rows(rank)
        model = reference_init(widths, "relu", seed=0, device=dev if (big and gpu) else None)
        zero1 = mode == "zero1" and comm
        arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev,
                      shadow_dtype=torch.bfloat16 if dtype == torch.bfloat16 else None,
                      bucket_bytes=(bucket_mb or a.bucket_mb) * 2 ** 20,
                      pad_to=64 * world if zero1 else 64, chunk_min_tiles=chunk_tiles)
        arena.bind_model(model)
        del model
        if not comm or not use_comm:
            sync = NoSync(arena)
        elif native_comm is not None:
            s = torch.cuda.current_stream()
            native_comm.broadcast(arena.master.data_ptr(), arena.numel, 0, 0, int(s.cuda_stream))
            s.synchronize()
            arena.sync_shadow()
            if zero1:
                sync = ShardedSync(arena, world, rank, native_comm=native_comm)
            else:
                bf16 = gdt == "bf16"
                sync = NativeRcclSync(arena, native_comm, world, inline=(mode == "inline"),
                                      grad_dtype=gdt,
                                      bf16_reduce=bf16_reduce if bf16 else None,
                                      f32_reduce=None if bf16 else bf16_reduce)
        else:
            dist.broadcast(arena.master, src=0, group=comm_group)
            arena.sync_shadow()
            if zero1:
                sync = ShardedSync(arena, world, rank, group=comm_group)
            else:
                sync = (make_shm_sync(arena, comm_group, world, rank)
                        if shm_sync_ok(dev.type, world, job.local_world, gdt) else None)
                if sync is None:
                    sync = TorchDistSync(arena, comm_group, world, grad_dtype=gdt)
        eng = MLPEngine(spec, arena, make_ops(), sync, device=dev, dtype=dtype,
                        rows_capacity=max(rows, 1), lr=a.lr, momentum=0.9,
                        use_graph=not a.no_graph, overlap=not a.no_overlap,
                        grouped=not a.no_group, rowband_overlap=(mode == "overlap_rowband"))
        eng.load_batch(X, Y, labels)
        cfg = TrainConfig(widths=list(widths), loss=c["loss"], n_features=widths[0], device="cpu")
        eng.set_scales(*loss_scales(cfg, rows, list(part.counts), widths[-1]))
        return eng

    def barrier():
        if gpu:
            torch.cuda.synchronize()
        pg.barrier()
        if gpu:
            torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world > 1:
            t = torch.tensor([x], dtype=torch.float64)
            pg.allreduce_cpu(t, op=dist.ReduceOp.MAX)
            x = float(t.item())
        return x

    def device_ok(eng) -> bool:
        """False (and the reason on stderr) when the engine's sticky device error word is set."""
        try:
            eng.check_device_errors()
            return True
        except RuntimeError as exc:
            print(f"[bench] rank {rank}: {exc}", file=sys.stderr, flush=True)
            return False

    def timed(eng, n, chunk):
        """Wall time of n steps, max over ranks (graphs captured beforehand)."""
        eng.prepare_steps(n, chunk)
        barrier()
        t0 = time.perf_counter()
        eng.run_steps(n, chunk)
        eng.synchronize(check=False)
        if gpu:
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # a column-split step that gave up a hand-off wait produced invalid results: the
        # measurement is void on every rank (inf wins the max below)
        if not device_ok(eng):
            el = float("inf")
        pg.barrier()
        return max_over_ranks(el)

    def chunk_for(n: int) -> int:
        # one replay's fixed cost (launch + drain) per graph: a short timed region (the
        # driver's 20 steps) is one graph launch, not 16 + 4
        return a.graph_chunk if a.graph_chunk > 0 else max(1, min(n, 128))

    chunk = chunk_for(a.steps)
    if a.scaling == "weak":
        n_global = rows_pg * world - (0 if (a.even or world == 1) else 1)
    else:
        n_global = rows_pg
    data = shard(n_global)
    mode = a.comm_mode
    if mode == "auto":
        # the best collective schedule depends on the node (link latency for small gradients,
        # comm kernels competing with the GEMMs for CUs for large ones), so it is measured
        # (untimed, before the timed region) rather than assumed
        mode = "tune"
    if not use_comm:
        mode = "none"
    elif native_comm is None and mode == "tune":
        mode = "inline"
    warm_run = {"steps": 0}

    def warm(e, n):
        """n untimed steps, then (GPU) a top-up to at least MIN_WARM_MS of continuous step work.
        The timed region's graphs are captured FIRST (after the eager first step): capturing is
        host-only work, and a GPU left idle meanwhile drops its clocks.  Measured on MI355X
        (profiles/r2s2_short_region_warmup_ab.txt): after setup + capture the first ~10-20 ms of
        steady work run at lower clocks -- the driver's 20-step region measured 0.1015-0.1017
        ms/step after 5 warm-up steps (0.5 ms of work) and 0.0953-0.0970 after 200, 50 steps
        0.0992-0.0995 vs 0.0938-0.0942 -- so a short region after W = 5 steps times the DVFS ramp,
        not the step, and a 1-GPU run (no tuning phase) would be timed colder than an N-GPU run
        (whose tuning keeps the GPU busy), skewing the scaling efficiency.  The top-up count is
        derived from the slowest rank's warm-up step time, so every rank runs the same steps
        (collectives); the JSON reports it (warmup_steps_run)."""
        milestone("warm-up")
        ran = 0
        if n > 0 and e.steps_done == 0:
            e.run_steps(1, 1)
            n -= 1
            ran += 1
        e.prepare_steps(a.steps, chunk)
        e.prepare_steps(n, chunk_for(n))
        if gpu:
            e.prepare_steps(WARM_CHUNK, WARM_CHUNK)
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.run_steps(n, chunk_for(n))
        ran += n
        if gpu and MIN_WARM_MS > 0 and n > 0:
            e.synchronize()
            per = max_over_ranks((time.perf_counter() - t0) / max(n, 1))
            extra = max(0, math.ceil(MIN_WARM_MS * 1e-3 / max(per, 1e-6)) - n)
            extra = -(-extra // WARM_CHUNK) * WARM_CHUNK
            for _ in range(extra // WARM_CHUNK):
                e.run_steps(WARM_CHUNK, WARM_CHUNK)
            ran += extra
        warm_run["steps"] += ran

    tune = None
    tune_algo = None
    bucket_mb = a.bucket_mb
    chunk_tiles = a.chunk_tiles
    bf16_reduce = None
    best_t = None
    best = None
    if mode == "tune":
        tune = {}
        eng = None
        # overlap candidates: --bucket_mb buckets, and ~two buckets (the first all-reduce
        # larger, the exposed last one smaller than the whole gradient)
        half_mb = round(grad_bytes / 2 ** 20 * 0.6, 3)
        ct0 = a.chunk_tiles
        if grad_bytes > INLINE_MAX_GRAD_BYTES:
            # overlap with 4 chunk buckets per 8192-wide layer (one 256-tile wave each: the
            # earliest collective start) and with 2 (half the launches and cross-queue waits,
            # twice the exposed last collective); measured at one rank: docs/PERF.md
            cands = [("overlap", "overlap", a.bucket_mb, ct0), ("overlap_c2", "overlap", a.bucket_mb, 512),
                     ("inline", "inline", None, ct0), ("zero1", "zero1", None, ct0)]
        else:
            cands = [("inline", "inline", None, ct0), ("zero1", "zero1", None, ct0),
                     ("overlap", "overlap", a.bucket_mb, ct0)]
            if half_mb > a.bucket_mb:
                cands.append((f"overlap_{half_mb}mb", "overlap", half_mb, ct0))
            if gpu and c["loss"] == "mse":
                # the row-band step with its last layer's bucket reduced during the other
                # layers' weight gradients (engine._step_body_rowband_overlap)
                cands.append(("overlap_rowband", "overlap_rowband", a.bucket_mb, ct0))
            if gpu and world > 1 and a.grad_dtype == "auto" and native_comm is not None:
                # the inline all-reduce with half the bytes on the links (bf16 payload, fp32
                # sums on each element's owner: one rounding whatever P is)
                cands.append(("inline_bf16", "inline", None, ct0, "bf16"))
        cands = [x if len(x) == 5 else x + (None,) for x in cands]

        def try_cand(key, m, bmb, ct, gdt=None, red=None):
            nonlocal eng, best_t, mode, bucket_mb, chunk_tiles, bf16_reduce, best
            milestone(f"tune {key}")
            e = build(m, data, bucket_mb=bmb, chunk_tiles=ct, bf16_reduce=red, gdt=gdt)
            e.run_steps(a.warmup, chunk_for(a.warmup))
            tm = min(timed(e, a.tune_steps, chunk_for(a.tune_steps)) for _ in range(2))
            if not math.isfinite(tm):
                # a candidate whose step gave up a device wait is never chosen
                tune[key] = None
                del e
                return
            tune[key] = round(tm / a.tune_steps * 1e3, 5)
            algo = getattr(e.sync, "bf16_reduce" if (gdt or grad_dtype) == "bf16" else "f32_reduce", None)
            if m != "zero1" and algo:
                tune_algo[key] = algo
            # every rank sees the same max-over-ranks times, so every rank keeps the same mode
            if eng is None or tm < best_t:
                eng, best_t, mode, bucket_mb, chunk_tiles = e, tm, key, (bmb or a.bucket_mb), ct
                bf16_reduce, best = red, (key, m, bmb, ct, gdt)
            del e

        tune_algo = {}
        for key, m, bmb, ct, gdt in cands:
            try_cand(key, m, bmb, ct, gdt)
        if native_comm is not None:
            # the all-reduce algorithm is tuned too, under the TWO fastest all-reduce schedules
            # (a slow default algorithm must not decide which schedule wins): each one's default
            # (bf16: acc32, one rounding; fp32: rccl for one bucket, the rank-ordered all-to-all
            # for several) against the other algorithm
            # (the bf16-payload inline candidate keeps its one-rounding acc32 reduction: RCCL's
            # bf16 ring rounds the partial sum at every hop, an error that grows with P)
            ranked = sorted((k for k in tune_algo if tune[k] is not None and
                             next(x for x in cands if x[0] == k)[4] != "bf16"),
                            key=lambda k: tune[k])[:2]
            for key in ranked:
                cand = next(x for x in cands if x[0] == key)
                alt = ("rccl" if tune_algo[key] != "rccl" else
                       ("acc32" if (cand[4] or grad_dtype) == "bf16" else "ordered"))
                try_cand(f"{key}+{alt}", cand[1], cand[2], cand[3], cand[4], red=alt)
        if eng is None:
            raise RuntimeError("every gradient-sync candidate gave up a device wait (invalid steps)")
        if gpu:
            torch.cuda.empty_cache()
        # the chosen engine idled while the other candidates ran: warm it again (untimed, like
        # the tuning runs themselves)
        warm(eng, a.warmup)
    else:
        eng = build(mode, data, chunk_tiles=a.chunk_tiles)
        warm(eng, a.warmup)

    # ---------------- the timed region: exactly K steps -------------------------------------
    # graph mode: steps replayed as hipGraphs of `chunk` complete consecutive steps (one
    # replay's fixed cost per chunk); every graph is captured before the timed region
    eng.prepare_steps(a.steps, chunk)
    # the step schedule the timed engine runs (rowband.hip / grouped backward / sequential)
    step_schedule = eng.schedule_name()
    # the all-reduce algorithm the timed engine uses (recorded before the extras free it)
    sync_algo = {"bf16": getattr(eng.sync, "bf16_reduce", None),
                 "fp32": getattr(eng.sync, "f32_reduce", None)}
    loss0 = eng.loss()
    milestone("timed")
    barrier()
    t0 = time.perf_counter()
    eng.run_steps(a.steps, chunk)
    eng.synchronize(check=False)
    if gpu:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    pg.barrier()
    elapsed = max_over_ranks(t1 - t0)
    # (raises on a timed-out column-split hand-off: no line is printed for an invalid step)
    loss = eng.loss()
    ms = elapsed / a.steps * 1e3
    value = n_global * a.steps / elapsed
    mode_name = mode
    # (the tuner's key names the candidate; best[1] is its schedule)
    mode = best[1] if best is not None else mode
    if best is not None and best[4]:
        grad_dtype = best[4]      # the chosen candidate's payload (wire bytes, the JSON line)
    sharded = mode == "zero1"
    n_buckets = len(eng.arena.buckets)
    wire = comm_volume(eng.arena.numel, world, grad_dtype, sharded=sharded,
                       shadow=eng.arena.shadow is not None)["wire_bytes_per_rank"]
    milestone("measured")
    # every replica must hold the same parameters and optimizer state, bit for bit: a hash of
    # the fp32 master, the momentum and the bf16 shadow on every rank, all-gathered over gloo
    digests = pg.allgather_object(replica_digest(eng, gpu))
    replicas_equal = len(set(digests)) == 1

    # ---------------- after the timed region: what the BASELINE metric derives from it ----------
    extras = {}
    strong = None
    extras_error = None

    def agree(ok: bool) -> bool:
        """Every rank's verdict on an extras phase (MIN over gloo): one rank failing outside a
        collective makes every rank skip the remaining phases together instead of leaving its
        peers blocked in the next collective (a rank stuck INSIDE one is the supervisor's
        stall detector's job)."""
        if world == 1:
            return ok
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
        pg.allreduce_cpu(t, op=dist.ReduceOp.MIN)
        return bool(t.item() > 0.5)

    def phase(name, fn):
        nonlocal extras_error
        milestone(f"extras {name}")
        err = None
        try:
            fn()
        except Exception as exc:   # noqa: BLE001
            err = f"{name}: {type(exc).__name__}: {exc}"[:300]
            print(f"[bench] extras failed on rank {rank}: {err}", file=sys.stderr, flush=True)
        if not agree(err is None):
            extras_error = err or f"{name} failed on another rank"
            return False
        return True

    def run_extras():
        """Efficiency / comm-only / strong-scaling measurements, one agreed phase at a time."""
        nonlocal eng, data, extras, strong
        n_ex = max(1, min(a.steps, EXTRA_STEPS))
        res = {"comm_ms": None, "comp_ms": ms}

        def comm_only():
            # the step's collectives alone (same buckets / dtype / order), replayed like the step
            sync = eng.sync
            with torch.no_grad():
                eng.arena.grad.zero_()
            if gpu:
                torch.cuda.synchronize()
            use_graph = gpu and not a.no_graph and not isinstance(sync, TorchDistSync)
            res["comm_ms"] = _time_comm_only(sync, n_ex, chunk_for(n_ex), use_graph, barrier,
                                             max_over_ranks) * 1e3
            with torch.no_grad():
                eng.arena.grad.zero_()

        def single():
            # the same per-rank work with the gradient sync off: every rank alone (1-GPU step)
            e = build("none", data, comm=False)
            e.run_steps(min(a.warmup, 10) + 1, chunk_for(min(a.warmup, 10)))
            res["comp_ms"] = timed(e, n_ex, chunk_for(n_ex)) / n_ex * 1e3
            if not math.isfinite(res["comp_ms"]):
                res["comp_ms"] = None
                raise RuntimeError("a column-split hand-off wait timed out: single-GPU step invalid")

        def strong_scaling():
            # strong scaling: the reference's fixed dataset (the 1-GPU shard, 8192 rows for the
            # proxy) split over the N ranks
            nonlocal strong
            sdata = shard(rows_pg)
            e = build(mode if mode != "none" else "inline", sdata, bucket_mb=bucket_mb,
                      chunk_tiles=chunk_tiles, bf16_reduce=bf16_reduce,
                      gdt=best[4] if best is not None else None)
            e.run_steps(min(a.warmup, 10) + 1, chunk_for(min(a.warmup, 10)))
            s_ms = timed(e, n_ex, chunk_for(n_ex)) / n_ex * 1e3
            if not math.isfinite(s_ms):
                raise RuntimeError("a column-split hand-off wait timed out: strong-scaling step invalid")
            comp_ms = res["comp_ms"]
            # S(1): the single-GPU step of the whole dataset = the compute-only step above
            # (weak scaling gives every rank rows_pg rows, the last one rows_pg - 1)
            st = {"global_batch": rows_pg, "ms_per_step": round(s_ms, 5),
                  "samples_per_s": round(rows_pg / (s_ms * 1e-3), 1),
                  "parallel_efficiency": round(comp_ms / (world * s_ms), 4),
                  "schedule": e.schedule_name(),
                  "rowband_split": bool(getattr(e, "uses_rowband_split", lambda: False)())}
            base = BASELINE_SAMPLES_PER_S.get(world) if a.config == "proxy512" else None
            st["vs_baseline"] = round(st["samples_per_s"] / base, 2) if base else None
            strong = st

        ok = True
        if use_comm:
            ok = phase("comm_only", comm_only)
        eng = None
        if gpu:
            torch.cuda.empty_cache()
        if ok and use_comm:
            ok = phase("single_gpu", single)
        if ok and (res["comp_ms"] is not None):
            extras = scaling_report(world, max(data[0].counts), n_global, ms, res["comp_ms"],
                                    res["comm_ms"], wire)
            extras["single_gpu_ms_per_step"] = res["comp_ms"]
        data = None
        if gpu:
            torch.cuda.empty_cache()
        if ok and world > 1 and a.scaling == "weak":
            phase("strong_scaling", strong_scaling)
        if gpu:
            torch.cuda.empty_cache()

    base = BASELINE_SAMPLES_PER_S.get(world) if a.config == "proxy512" else None
    tflops = spec.flops_per_sample() * n_global / (ms * 1e-3) / 1e12

    def rnd(x, k=4):
        return None if x is None else round(float(x), k)

    def line():
        return {
            "metric": "samples_per_sec_whole_node",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_run": warm_run["steps"],
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": (round(value / base, 2) if base else None),
            "dtype": a.dtype,
            "data": "synthetic (device-generated make_regression-style rows), random init",
            "config": {"model": c["model"], "global_batch": n_global, "seq_len": None,
                       "parallelism": f"dp{world}", "rows_per_gpu": rows_pg,
                       "uneven_split": (not a.even and world > 1 and a.scaling == "weak"),
                       "device": a.device,
                       "comm": (("rccl" if native_comm is not None else
                                 ("nccl" if pg.nccl is not None else "gloo"))
                                if use_comm else "none"),
                       "graph": gpu and not a.no_graph, "graph_chunk": chunk,
                       "overlap": not a.no_overlap, "grouped": not a.no_group,
                       "schedule": step_schedule,
                       "comm_mode": mode_name if use_comm else None,
                       "comm_tune_ms_per_step": tune,
                       "comm_tune_algorithm": (tune_algo if tune is not None else None),
                       "grad_dtype": grad_dtype if use_comm else None,
                       "bf16_reduce": (sync_algo["bf16"] if use_comm and grad_dtype == "bf16"
                                       else None),
                       "f32_reduce": (sync_algo["fp32"] if use_comm and grad_dtype != "bf16"
                                      else None),
                       "grad_wire_bytes_per_rank": wire,
                       "bucket_mb": bucket_mb,
                       "n_buckets": n_buckets},
            "rccl_ranks": (native_comm.size if native_comm is not None else None),
            "replicas_bitwise_equal": replicas_equal,
            "replica_hash": digests[0],
            "shared_gpu_rehearsal": bool(a.shared_gpu_rehearsal),
            "model_tflops_per_s": round(tflops, 2),
            "parallel_efficiency": rnd(extras.get("parallel_efficiency")),
            "single_gpu_samples_per_s": rnd(extras.get("single_gpu_samples_per_s"), 1),
            "single_gpu_ms_per_step": rnd(extras.get("single_gpu_ms_per_step"), 5),
            "exposed_comm_ms": rnd(extras.get("exposed_comm_ms"), 5),
            "comm_only_ms": rnd(extras.get("comm_only_ms"), 5),
            "overlap_pct": rnd(extras.get("overlap_pct"), 1),
            "comm_bus_gbps": rnd(extras.get("comm_bus_gbps"), 2),
            "strong_scaling": strong,
            "extras_error": extras_error,
            "loss_after_warmup": loss0,
            "final_loss": loss,
            "knobs": knobs_report(a),
        }

    if rank == 0 and supervised():
        # the measurement so far, in case the extras never come back (the supervisor prints it)
        write_result(dict(line(), extras_error="extras did not finish", complete=False))
    if not a.no_extras:
        run_extras()
    milestone("done")
    if rank == 0:
        if supervised():
            write_result(dict(line(), complete=True))
        else:
            print(json.dumps(line()), flush=True)
    # Teardown, in order, each step timed on stderr (NNMPI_TEARDOWN_TRACE=1): the graphs (which
    # hold captured RCCL kernels) and engines first, then the communicator, then the process
    # group.  The result is already out: a teardown that stalls (a communicator destroy
    # waiting on a peer that has gone) must not keep the job alive, so a watchdog ends the
    # process after TEARDOWN_S seconds -- with a non-zero code, since a stall is still a defect.
    _exit_watchdog(TEARDOWN_S)
    if gpu:
        torch.cuda.synchronize()
    _trace("teardown: engines and graphs")
    eng = None
    import gc
    gc.collect()
    _trace("teardown: communicator")
    native_comm = None
    gc.collect()
    _trace("teardown: process group")
    pg.destroy()
    _trace("teardown: done")


TEARDOWN_S = 60.0
RC_TEARDOWN_STALL = 4     # = parallel.supervisor.RC_TEARDOWN_STALL (3: the step watchdog)


def _milestones(rank: int):
    """progress(phase) for the supervisor's stall detector, plus TESTING-only fault hooks:
    NNMPI_BENCH_CRASH / NNMPI_BENCH_HANG = "rank:attempt[:phase]" make that rank die by SIGSEGV
    / stop making progress when it reaches the phase (default: "timed") in that attempt ("*":
    every attempt)."""
    from nnmpi_amd.parallel.supervisor import progress

    def hook(var):
        spec = os.environ.get(var, "")
        if not spec:
            return None
        parts = spec.split(":")
        if int(parts[0]) != rank or parts[1] not in ("*", os.environ.get("NNMPI_ATTEMPT", "0")):
            return None
        return parts[2] if len(parts) > 2 else "timed"
    crash_at, hang_at = hook("NNMPI_BENCH_CRASH"), hook("NNMPI_BENCH_HANG")

    def milestone(phase: str):
        progress(phase)
        if crash_at == phase:
            import signal
            print(f"[bench] rank {rank}: injected SIGSEGV at '{phase}'", file=sys.stderr, flush=True)
            os.kill(os.getpid(), signal.SIGSEGV)
        if hang_at == phase:
            print(f"[bench] rank {rank}: injected hang at '{phase}'", file=sys.stderr, flush=True)
            while True:
                time.sleep(60)
    return milestone


def replica_digest(eng, gpu: bool) -> str:
    """Bitwise hash of this rank's replica: fp32 master, momentum and bf16 shadow (HIP kernel
    hash_u32 on the GPU; sha256 of the bytes on the CPU).  A sharded optimizer (ZeRO-1) first
    re-assembles the full master and momentum (a collective: every rank calls this)."""
    import torch
    ar = eng.arena
    eng.synchronize()
    if getattr(eng.sync, "sharded", False):
        eng.sync.gather_state()
    bufs = [ar.master, ar.momentum] + ([ar.shadow] if ar.shadow is not None else [])
    if gpu:
        from nnmpi_amd import native
        torch.cuda.synchronize()
        out = torch.zeros(len(bufs), 1025, dtype=torch.int64, device=ar.master.device)
        s = torch.cuda.current_stream()
        for k, b in enumerate(bufs):
            nbytes = b.numel() * b.element_size()
            native.lib().hash_u32(b.data_ptr(), nbytes // 4, out[k].data_ptr(), int(s.cuda_stream))
        vals = out[:, 1024].cpu().tolist()
        return "-".join(f"{v & 0xFFFFFFFFFFFFFFFF:016x}" for v in vals)
    import hashlib
    h = hashlib.sha256()
    for b in bufs:
        h.update(b.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes())
    return h.hexdigest()[:48]


def _trace(msg: str):
    if os.environ.get("NNMPI_TEARDOWN_TRACE") == "1":
        print(f"[bench rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}",
              file=sys.stderr, flush=True)


def _exit_watchdog(seconds: float):
    import threading

    def fire():
        print(f"[bench] teardown did not finish in {seconds:.0f} s: exiting with code "
              f"{RC_TEARDOWN_STALL} (result already out)", file=sys.stderr, flush=True)
        os._exit(RC_TEARDOWN_STALL)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def _time_comm_only(sync, n, chunk, use_graph, barrier, max_over_ranks) -> float:
    """Seconds per repetition of the step's collectives alone (max over ranks)."""
    import torch
    if use_graph:
        from nnmpi_amd import native
        s = torch.cuda.Stream()
        graphs = []
        reps = min(chunk, n)
        with torch.cuda.stream(s):
            sync.comm_only()           # warm (RCCL lazily sets up its channels on first use)
            s.synchronize()
            g = native.lib().GraphRunner()
            g.begin(int(s.cuda_stream))
            try:
                for _ in range(reps):
                    sync.comm_only()
            except Exception:
                g.cancel()
                raise
            g.end()
            graphs.append(g)
        n_launch = max(1, n // reps)
        barrier()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(n_launch):
                g.launch(int(s.cuda_stream))
        s.synchronize()
        el = time.perf_counter() - t0
        return max_over_ranks(el) / (n_launch * reps)
    sync.comm_only()
    if torch.cuda.is_available() and getattr(sync.arena.grad, "is_cuda", False):
        torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        sync.comm_only()
    if getattr(sync.arena.grad, "is_cuda", False):
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return max_over_ranks(el) / n


if __name__ == "__main__":
    main()

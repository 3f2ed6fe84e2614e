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

Gradient-sync schedule (``--comm_mode``, default auto): for latency-bound gradient volumes the
fastest schedule depends on the node's collective latency, so the three candidates (one inline
all-reduce; ZeRO-1 reduce-scatter + sharded SGD + bf16 all-gather; per-bucket all-reduce on a
comm stream overlapped with backward) are each timed for ``--tune_steps`` steps BEFORE the timed
region and the fastest (max over ranks, so every rank agrees) is kept; its time per candidate
is reported in ``config.comm_tune_ms_per_step``.  Large gradients always overlap.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  The timed region is exactly K full training steps (forward,
loss, backward, gradient all-reduce, optimizer update), bracketed by barrier + device sync on
both sides; the reported time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference numbers (reference algorithm on the 512-wide proxy, CPU, samples/s)
BASELINE_SAMPLES_PER_S = {1: 32190.0, 2: 61546.0, 4: 88657.0, 8: 105377.0}
# below this gradient volume the all-reduce is latency-bound: issue it inline (see parallel/sync.py)
INLINE_MAX_GRAD_BYTES = 64 << 20

CONFIGS = {
    "proxy512": dict(widths=[512, 512, 512, 512, 1], loss="mse", rows=8192,
                     model="mlp_512x4_regression(512-512-512-512-1)"),
    "mlp512x3": dict(widths=[512, 512, 512, 1], loss="mse", rows=8192,
                     model="mlp_512x3_regression(512-512-512-1)"),
    "wide8192": dict(widths=[8192] * 5 + [1], loss="mse", rows=4096,
                     model="mlp_8192x4_regression(8192x4-1)"),
    "mnist": dict(widths=[784, 1024, 1024, 10], loss="xent", rows=8192,
                  model="mlp_mnist_shape(784-1024-1024-10,xent)"),
    # the reference config itself: fp32 like the reference (whole step in one tiny-MLP kernel)
    "ref": dict(widths=[2, 3, 1], loss="mse", rows=16, model="mlp_reference(2-3-1)", dtype="fp32"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="proxy512", choices=sorted(CONFIGS))
    p.add_argument("--rows", type=int, default=None, help="rows per GPU (weak scaling)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--comm", choices=["native", "torch"], default="native")
    p.add_argument("--bucket_mb", type=float, default=1.0)
    p.add_argument("--no_graph", action="store_true")
    p.add_argument("--no_overlap", action="store_true")
    p.add_argument("--no_group", action="store_true",
                   help="separate dgrad / wgrad / combine launches instead of the grouped one")
    p.add_argument("--even", action="store_true", help="no uneven extra rows")
    p.add_argument("--graph_chunk", type=int, default=16,
                   help="steps per replayed hipGraph (1 = one graph launch per step)")
    p.add_argument("--lr", type=float, default=1e-5)
    p.add_argument("--comm_mode", choices=["auto", "tune", "overlap", "inline", "zero1"],
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
    p.add_argument("--fwd_variant", type=int, default=-1, help="forward GEMM variant (experiments)")
    p.add_argument("--group_async", type=int, default=-1,
                   help="grouped-backward LDS read mode (experiments)")
    return p.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    import nnmpi_amd  # noqa: F401
    from nnmpi_amd.data import synth
    from nnmpi_amd.data.partition import partition_rows
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.engine.trainer import loss_scales
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.parallel import dist as pdist
    from nnmpi_amd.parallel.sync import NativeRcclSync, NoSync, ShardedSync, TorchDistSync
    from nnmpi_amd.utils.config import TrainConfig
    from nnmpi_amd.utils.metrics import comm_volume
    from nnmpi_amd import native

    job = pdist.detect_job()
    rank, world = job.rank, job.world
    native.lib().set_fwd_variant(a.fwd_variant)
    native.lib().set_group_async(a.group_async)
    torch.cuda.set_device(job.local_rank % torch.cuda.device_count())
    dev = torch.device("cuda", torch.cuda.current_device())
    pg = pdist.ProcessGroupContext(job, 600.0, want_nccl=(a.comm == "torch" and world > 1))
    c = CONFIGS[a.config]
    widths = c["widths"]
    spec = MLPSpec(tuple(widths), "relu", c["loss"])
    rows_pg = a.rows or c["rows"]
    if a.scaling == "weak":
        n_global = rows_pg * world - (0 if (a.even or world == 1) else 1)
    else:
        n_global = rows_pg
    part = partition_rows(n_global, world)
    rows = part.rows(rank)
    if "dtype" in c:
        a.dtype = c["dtype"]
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32

    # data (device-generated, partition-independent rows)
    if c["loss"] == "xent":
        X, labels = synth.chunked_classification(part.start(rank), rows, widths[0], widths[-1],
                                                 device=dev)
        Y = None
    else:
        X, Y = synth.chunked_regression(part.start(rank), rows, widths[0], device=dev)
        labels = None
    # model: same seed everywhere + broadcast from rank 0 (reference ref.py:87)
    big = spec.n_params > 20_000_000
    use_comm = (world > 1 or a.force_comm)
    cfg = TrainConfig(widths=list(widths), loss=c["loss"], n_features=widths[0])
    inv, lsc, gsc = loss_scales(cfg, rows, list(part.counts), widths[-1])
    native_comm = None
    if use_comm and a.comm == "native":
        lib = native.lib()
        uid = pg.broadcast_object(lib.rccl_unique_id() if rank == 0 else None, 0)
        native_comm = native.make_comm(uid, world, rank, dev.index)

    def build(mode):
        """One arena + gradient-sync strategy + engine.  mode: inline | overlap | zero1."""
        model = reference_init(widths, "relu", seed=0, device=dev if big else None)
        arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev,
                      shadow_dtype=torch.bfloat16 if dtype == torch.bfloat16 else None,
                      bucket_bytes=a.bucket_mb * 2 ** 20,
                      pad_to=64 * world if mode == "zero1" else 64)
        arena.bind_model(model)
        del model
        if native_comm is not None:
            s = torch.cuda.current_stream()
            native_comm.broadcast(arena.master.data_ptr(), arena.numel, 0, 0, int(s.cuda_stream))
            s.synchronize()
            arena.sync_shadow()
            if mode == "zero1":
                sync = ShardedSync(arena, world, rank, native_comm=native_comm)
            else:
                sync = NativeRcclSync(arena, native_comm, world, inline=(mode == "inline"))
        elif world > 1:
            dist.broadcast(arena.master, src=0, group=pg.nccl)
            arena.sync_shadow()
            sync = TorchDistSync(arena, pg.nccl, world)
        else:
            sync = NoSync(arena)
        eng = MLPEngine(spec, arena, HipOps(dev), sync, device=dev, dtype=dtype,
                        rows_capacity=rows, lr=a.lr, momentum=0.9, use_graph=not a.no_graph,
                        overlap=not a.no_overlap, grouped=not a.no_group)
        eng.load_batch(Xc, Y, labels)
        eng.set_scales(inv, lsc, gsc)
        return eng

    def barrier():
        torch.cuda.synchronize()
        pg.barrier()
        torch.cuda.synchronize()

    def timed(eng, n, chunk):
        """Wall time of n steps, max over ranks (graphs captured beforehand)."""
        eng.prepare_steps(n, chunk)
        barrier()
        t0 = time.perf_counter()
        eng.run_steps(n, chunk)
        eng.synchronize()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        pg.barrier()
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64)
            pg.allreduce_cpu(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    Xc = X.to(dtype)
    del X
    chunk = max(1, a.graph_chunk)
    grad_bytes = spec.n_params * 4
    mode = a.comm_mode
    if mode == "auto":
        # small (latency-bound) gradients: the best collective schedule depends on the link
        # latency of the node, so it is measured (untimed, before the timed region) rather than
        # assumed; large gradients always overlap per-bucket all-reduces with the backward.
        mode = "tune" if grad_bytes <= INLINE_MAX_GRAD_BYTES else "overlap"
    if native_comm is None:
        mode = "inline" if use_comm else "none"
    tune = None
    if mode == "tune":
        tune = {}
        eng = None
        for m in ("inline", "zero1", "overlap"):
            e = build(m)
            e.run_steps(a.warmup, chunk)
            tm = min(timed(e, a.tune_steps, chunk) for _ in range(2))
            tune[m] = round(tm / a.tune_steps * 1e3, 5)
            # every rank sees the same max-over-ranks times, so every rank keeps the same mode
            if eng is None or tm < best_t:
                eng, best_t, mode = e, tm, m
            del e
        torch.cuda.empty_cache()
    else:
        eng = build(mode)
        eng.run_steps(a.warmup, chunk)
    sync = eng.sync
    del Xc

    # graph mode: steps replayed as hipGraphs of `chunk` complete consecutive steps (one
    # replay's fixed cost per chunk); every graph is captured before the timed region
    eng.prepare_steps(a.steps, chunk)
    loss0 = eng.loss()
    barrier()
    t0 = time.perf_counter()
    eng.run_steps(a.steps, chunk)
    eng.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pg.barrier()
    elapsed = t1 - t0
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64)
        pg.allreduce_cpu(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
    loss = eng.loss()
    ms = elapsed / a.steps * 1e3
    samples = n_global
    value = samples * a.steps / elapsed
    base = BASELINE_SAMPLES_PER_S.get(world) if a.config == "proxy512" else None
    tflops = spec.flops_per_sample() * samples / (ms * 1e-3) / 1e12
    if rank == 0:
        out = {
            "metric": "samples_per_sec_whole_node",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": (round(value / base, 2) if base else None),
            "dtype": a.dtype,
            "data": "synthetic (device-generated make_regression-style rows), random init",
            "config": {"model": c["model"], "global_batch": samples, "seq_len": None,
                       "parallelism": f"dp{world}", "rows_per_gpu": rows_pg,
                       "uneven_split": (not a.even and world > 1),
                       "comm": a.comm if (world > 1 or a.force_comm) else "none",
                       "graph": not a.no_graph, "graph_chunk": a.graph_chunk, "overlap": not a.no_overlap,
                       "grouped": not a.no_group,
                       "comm_mode": mode if use_comm else None,
                       "comm_tune_ms_per_step": tune,
                       "grad_wire_bytes_per_rank": comm_volume(
                           eng.arena.numel, world, sharded=(mode == "zero1"),
                           shadow=eng.arena.shadow is not None)["wire_bytes_per_rank"],
                       "bucket_mb": a.bucket_mb},
            "model_tflops_per_s": round(tflops, 2),
            "loss_after_warmup": loss0,
            "final_loss": loss,
        }
        print(json.dumps(out), flush=True)
    native_comm = None
    pg.destroy()


if __name__ == "__main__":
    main()

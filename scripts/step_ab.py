"""Whole-step A/B of kernel-selection knobs on the bench step, interleaved in ONE process
(cdna_hip_programming.md §5.4 rule 24: perf deltas come from interleaved rounds, never from
separate invocations).

Every config restores the same parameter/momentum snapshot, re-captures the step graphs (kernel
choices are baked into captured launches), warms one chunk, and times ``--steps`` steps replayed
as multi-step graphs exactly like bench.py's timed region.  Knobs that only change tiling or LDS
read scheduling must leave the result bitwise unchanged: each JSON line reports whether the
config's final parameters equal the first config's (the split-K knob legitimately changes the
summation order and is expected to differ).

    python scripts/step_ab.py [--config proxy512] [--rounds 5] [--steps 64]
    python scripts/step_ab.py --configs '[{}, {"fwd": 2, "gasync": 2}]'
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

DEFAULT_CONFIGS = [
    {},
    {"fwd": 1}, {"fwd": 2}, {"fwd": 5}, {"fwd": 6}, {"fwd": 7}, {"fwd": 8},
    {"gasync": 0}, {"gasync": 2},
    {"wsplit": 8},
]


def apply(lib, knobs):
    lib.set_fwd_variant(int(knobs.get("fwd", -1)))
    lib.set_group_async(int(knobs.get("gasync", -1)))
    lib.set_wgrad_splits(int(knobs.get("wsplit", 0)))
    lib.set_slab_store_policy(int(knobs.get("slab", -1)))     # split-K slab stores (2 = sc1)
    for epi, idx in enumerate(str(knobs.get("pp", "0,0,1")).split(",")):
        lib.set_pp256_order(epi, int(idx))                    # 256x256 kernel per epilogue


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="proxy512", choices=sorted(bench.CONFIGS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--chunk", type=int, default=16)
    ap.add_argument("--configs", default=None, help="JSON list of knob dicts")
    a = ap.parse_args()
    configs = json.loads(a.configs) if a.configs else DEFAULT_CONFIGS
    lib = native.lib()
    c = bench.CONFIGS[a.config]
    widths, rows = c["widths"], c["rows"]
    dev = torch.device("cuda", 0)
    spec = MLPSpec(tuple(widths), "relu", c["loss"])
    arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev,
                  shadow_dtype=torch.bfloat16)
    big = spec.n_params > 20_000_000
    arena.bind_model(reference_init(widths, "relu", seed=0, device=dev if big else None))
    eng = MLPEngine(spec, arena, HipOps(dev), NoSync(arena), device=dev, dtype=torch.bfloat16,
                    rows_capacity=rows, lr=1e-5, momentum=0.9)
    if c["loss"] == "xent":
        X, lab = synth.chunked_classification(0, rows, widths[0], widths[-1], device=dev)
        Y = None
    else:
        X, Y = synth.chunked_regression(0, rows, widths[0], device=dev)
        lab = None
    eng.load_batch(X.to(torch.bfloat16), Y, lab)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    eng.run_steps(2, a.chunk)            # eager first step (momentum init) + one replayed step
    eng.synchronize()
    state = (arena.master, arena.momentum, arena.shadow)
    snap = [t.clone() for t in state]
    times = [[] for _ in configs]
    finals = [None] * len(configs)
    for r in range(a.rounds):
        for i, knobs in enumerate(configs):
            apply(lib, knobs)
            for t, s in zip(state, snap):
                t.copy_(s)
            # (the weights changed outside an optimizer step: the row-band v2 weight images are
            # rebuilt before the next step -- without this, every config after the first started
            # from the previous config's images and no rowband config compared bitwise)
            arena.version += 1
            eng._graphs.clear()
            eng.run_steps(a.chunk, a.chunk)          # capture + warm the new kernels
            eng.prepare_steps(a.steps, a.chunk)
            eng.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run_steps(a.steps, a.chunk)
            eng.synchronize()
            times[i].append((time.perf_counter() - t0) / a.steps * 1e6)
            if r == 0:
                finals[i] = arena.master.clone()
        print(f"[step_ab] round {r + 1}/{a.rounds} done", file=sys.stderr, flush=True)
    apply(lib, {})
    loss = eng.loss()
    for i, knobs in enumerate(configs):
        v = times[i]
        print(json.dumps({"config": a.config, "knobs": knobs,
                          "median_us_per_step": round(statistics.median(v), 2),
                          "min_us_per_step": round(min(v), 2),
                          "bitwise_equal_to_first": bool(torch.equal(finals[i], finals[0])),
                          "loss_finite": loss == loss}), flush=True)


if __name__ == "__main__":
    main()

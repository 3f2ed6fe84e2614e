"""Interleaved A/B timing of the MLP GEMM kernels in ONE process (guide §5.4 rule 24).

Times forward / dgrad / wgrad for a layer shape with both main loops (register-staged v1 and
LDS-DMA ring v2), random operands, median of N interleaved rounds; prints JSON lines."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--inf", type=int, default=512)
    ap.add_argument("--outf", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--impls", default="1,2")
    ap.add_argument("--tiles", default="0,64,128")
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--variants", default="0")
    a = ap.parse_args()
    lib = native.lib()
    ops = HipOps()
    dev = "cuda"
    R, K, N = a.rows, a.inf, a.outf
    x = (torch.rand(R, K, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.rand(N, device=dev)
    y = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
    dz = (torch.rand(R, N, device=dev) * 2 - 1).to(torch.bfloat16)
    dx = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
    gW = torch.empty(N, K, device=dev)
    gb = torch.empty(N, device=dev)
    ws = torch.empty(ops.wgrad_workspace_bytes(R, N, K, torch.bfloat16) // 4 + 64, device=dev)
    jobs = {
        "fwd": lambda: ops.linear_act(x, W, b, "relu", y),
        "dgrad": lambda: ops.linear_dgrad(dz, W, x, "relu", dx),
        "wgrad": lambda: ops.linear_wgrad(dz, x, gW, gb, ws=ws),
    }
    tjobs = {
        "fwd": lambda: torch.mm(x, W.t(), out=y),
        "dgrad": lambda: torch.mm(dz, W, out=dx),
        "wgrad": lambda: torch.mm(dz.t(), x, out=gWb),
    }
    gWb = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    jobs = {k: v for k, v in jobs.items() if k in a.only.split(",")}
    impls = [(int(i), int(t), int(v)) for i in a.impls.split(",") for t in a.tiles.split(",")
             for v in (a.variants.split(",") if i == "2" else ["0"])]
    res = {(j, i): [] for j in jobs for i in impls}
    first_out, same = {}, {}
    for r in range(a.rounds):
        for name in jobs:
            for impl in impls:
                if impl[0] == 0:   # vendor reference point: torch.mm (hipBLASLt), bf16 out
                    fn = tjobs[name]
                else:
                    fn = jobs[name]
                lib.set_gemm_impl(max(impl[0], 1))
                lib.set_gemm_tile(impl[1])
                lib.set_gemm_variant(impl[2])
                # the split-K workspace depends on the (forced) tile: size it for THIS config
                need = ops.wgrad_workspace_bytes(R, N, K, torch.bfloat16) // 4 + 64
                if ws.numel() < need:
                    ws = torch.empty(need, device=dev)
                fn()
                if r == 0 and impl[0] != 0:
                    # bitwise check of every own-kernel variant against the first one (same
                    # MFMA order per output element -> identical results expected)
                    out = {"fwd": y, "dgrad": dx, "wgrad": gW}[name].clone()
                    ref = first_out.setdefault(name, out)
                    same[(name, impl)] = bool(torch.equal(ref, out))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                e.synchronize()
                res[(name, impl)].append(s.elapsed_time(e) * 1e3 / a.iters)
    flops = 2.0 * R * K * N
    for (name, impl), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"kernel": name, "impl": impl[0], "tile": impl[1], "variant": impl[2], "rows": R, "in": K, "out": N,
                          "median_us": round(med, 2), "min_us": round(min(v), 2),
                          "tflops": round(flops / (med * 1e-6) / 1e12, 1),
                          "bitwise_equal_first_variant": same.get((name, impl))}))
    lib.set_gemm_impl(2)
    lib.set_gemm_tile(0)
    lib.set_gemm_variant(0)


if __name__ == "__main__":
    main()

"""Wide weight gradient: how much of its gap to the forward GEMM is the operand layout?

Times, interleaved in one process, the 8192 x 8192 x 4096 product (M = out, N = in, K = rows) on
the production 256x256 tile through gemm_bf16_generic_tile with every operand-layout pair (XMAJ
= the row-major activations the wide wgrad reads today, KMAJ = transposed copies), fp32 output,
and the production forward / weight-gradient launches for reference.  Prints one JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402

KMAJ, XMAJ = 0, 1


def main():
    lib, ops, dev = native.lib(), HipOps(), "cuda"
    R, H = 4096, 8192
    x = (torch.rand(R, H, device=dev) * 2 - 1).to(torch.bfloat16)      # a_{l-1} [rows][in]
    dz = (torch.rand(R, H, device=dev) * 2 - 1).to(torch.bfloat16)     # dZ_l   [rows][out]
    xt, dzt = x.t().contiguous(), dz.t().contiguous()                  # [in][rows], [out][rows]
    W = ((torch.rand(H, H, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.rand(H, device=dev)
    y = torch.empty(R, H, device=dev, dtype=torch.bfloat16)
    C = torch.empty(H, H, device=dev)
    gb = torch.empty(H, device=dev)
    s = native.stream_handle()
    p = native.ptr
    jobs = {
        # A = dZ (x = out, k = rows), B = X (x = in, k = rows)
        "xx": lambda: lib.gemm_bf16_tile(p(dz), H, XMAJ, p(x), H, XMAJ, H, H, R, p(C), H, 256, s),
        "kk": lambda: lib.gemm_bf16_tile(p(dzt), R, KMAJ, p(xt), R, KMAJ, H, H, R, p(C), H, 256, s),
        "kx": lambda: lib.gemm_bf16_tile(p(dzt), R, KMAJ, p(x), H, XMAJ, H, H, R, p(C), H, 256, s),
        "xk": lambda: lib.gemm_bf16_tile(p(dz), H, XMAJ, p(xt), R, KMAJ, H, H, R, p(C), H, 256, s),
        "wgrad": lambda: ops.linear_wgrad(dz, x, C, gb, ws=None),
        "fwd": lambda: ops.linear_act(x, W, b, "relu", y),
    }
    res = {k: [] for k in jobs}
    for _ in range(3):
        for f in jobs.values():
            f()
    torch.cuda.synchronize()
    for _ in range(5):
        for k, f in jobs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000 / 5)
    ref = None
    for k in ("xx", "kk", "kx", "xk"):
        jobs[k]()
        torch.cuda.synchronize()
        if ref is None:
            ref = C.clone()
        else:
            assert torch.equal(C, ref), k   # same k order, same tile: bitwise equal
    print(json.dumps({k: round(statistics.median(v), 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()

"""Operand layout vs speed of the 256x256 ping-pong GEMM at the 8192-wide weight-gradient shape
(M = N = 8192 outputs, K = 4096 rows): KMAJ operands are read with ds_read_b128, XMAJ operands
with ds_read_b64_tr_b16 (twice the LDS read instructions).  The wgrad today is XMAJ x XMAJ;
this times all four layout pairs on the same values (and checks they agree)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--N", type=int, default=8192)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tiles", default="256")
    ap.add_argument("--variants", default="0",
                    help="256-tile kernel variants: 0 default, 15 GM4, 16 early reads GM1, 17 GM1, 18 GM8")
    ap.add_argument("--pairs", default="XX,KK,KX,XK")
    ap.add_argument("--fwd", action="store_true",
                    help="also time the production forward (bias + ReLU, bf16 out) at M x N x K")
    a = ap.parse_args()
    lib = native.lib()
    M, N, K = a.M, a.N, a.K
    g = torch.Generator(device="cuda").manual_seed(0)
    dz = (torch.randn(K, M, device="cuda", generator=g) * 0.05).to(torch.bfloat16)   # XMAJ A
    x = torch.randn(K, N, device="cuda", generator=g).relu().to(torch.bfloat16)      # XMAJ B
    dzt, xt = dz.t().contiguous(), x.t().contiguous()                                # KMAJ
    C = torch.empty(M, N, device="cuda")
    ref = None
    st = torch.cuda.current_stream().cuda_stream
    pairs = [(int(p[0] == "X"), int(p[1] == "X")) for p in a.pairs.split(",")]
    for tile, var in [(int(t), int(v)) for t in a.tiles.split(",") for v in a.variants.split(",")]:
        lib.set_gemm_variant(var)
        for la, lb in pairs:
            A = dz if la else dzt
            B = x if lb else xt
            lda = A.stride(0)
            ldb = B.stride(0)

            def run():
                lib.gemm_bf16_tile(A.data_ptr(), lda, la, B.data_ptr(), ldb, lb, M, N, K,
                                   C.data_ptr(), N, tile, st)
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            same = bool(torch.equal(C, ref))
            maxdiff = float((C - ref).abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            print(json.dumps({"tile": tile, "variant": var, "A": "XMAJ" if la else "KMAJ",
                              "B": "XMAJ" if lb else "KMAJ", "us": round(us, 1),
                              "pflops": round(2 * M * N * K / us / 1e9, 3),
                              "bitwise_equal_to_first": same, "max_abs_diff": maxdiff}),
                  flush=True)
    lib.set_gemm_variant(0)
    if a.fwd:
        # production forward: Y[M][N] = relu(X[M][K] . W[N][K]^T + b), bf16 out
        X = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.rand(N, device="cuda", generator=g)
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def fwd():
            lib.linear_fwd_bf16(X.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), Y.data_ptr(), N,
                                M, N, K, 1, st)
        fwd()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fwd()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps({"kernel": "linear_fwd_bf16 (bias+relu, bf16 out)", "us": round(us, 1),
                          "pflops": round(2 * M * N * K / us / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()

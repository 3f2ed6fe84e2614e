"""Can a memory-bound SGD pass run BESIDE a compute-bound 256x256 GEMM on MI355X?

The 8192-wide layer's GEMM blocks take 2 waves per SIMD x 224 VGPRs (dgrad/forward) or x 248
(weight gradient), one 512-thread block per CU.  An SGD block (30 VGPRs) fits beside a
224-VGPR GEMM block (64 VGPRs per SIMD left) but not beside a 248-VGPR one.  This times, with
events, on one GPU:
  * each kernel alone (dgrad, wgrad without / with the fused SGD epilogue, SGD at several
    grid sizes);
  * dgrad on stream 1 and the SGD on stream 2 concurrently, in both issue orders;
  * the two backward orders of one layer pair: [wgrad+fused SGD ; dgrad] versus
    [wgrad ; (SGD || dgrad)].
Prints one JSON line per measurement (microseconds per repetition).
"""
import argparse
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--width", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops, lib = HipOps(), native.lib()
    R, H = a.rows, a.width
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    W = (torch.randn(H, H, device=dev, generator=g) * 0.01).to(bf)
    dz = (torch.randn(R, H, device=dev, generator=g) * 0.01).to(bf)
    ap_ = torch.randn(R, H, device=dev, generator=g).relu().to(bf)
    dx = torch.empty(R, H, device=dev, dtype=bf)
    n = H * H + H
    ar = types.SimpleNamespace(numel=n, master=torch.randn(n, device=dev) * 0.01,
                               grad=torch.randn(n, device=dev) * 1e-3,
                               momentum=torch.zeros(n, device=dev),
                               shadow=torch.empty(n, device=dev, dtype=bf))
    gW, gb = ar.grad[:H * H].view(H, H), ar.grad[H * H:]
    hp = torch.tensor([0.01, 0.9, 0.0, 0.0, 1.0, 0, 0, 0], device=dev, dtype=torch.float32)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    _p = native.ptr

    def dgrad():
        ops.linear_dgrad(dz, W, ap_, "relu", dx)

    def wgrad(fuse):
        sg = ops.sgd_fusion(ar, hp, False, False) if fuse else None
        assert ops.wgrad_workspace_bytes(R, H, H, bf) == 0
        ops.linear_wgrad(dz, ap_, gW, gb, None, sg)

    def sgd(blocks):
        st = native.stream_handle()
        if blocks == 0:
            lib.sgd_momentum(_p(ar.master), _p(ar.grad), _p(ar.momentum), _p(ar.shadow), n,
                             _p(hp), 0, 0, 0, st)
        else:
            lib.sgd_momentum_bg(_p(ar.master), _p(ar.grad), _p(ar.momentum), _p(ar.shadow), n,
                                _p(hp), 0, 0, 0, blocks, st)

    def timeit(name, body):
        with torch.cuda.stream(s1):
            body()      # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s1):
            e0.record()
            for _ in range(a.reps):
                body()
            e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps({"case": name, "us": round(us, 1)}), flush=True)
        return us

    def conc(first, second):
        """first on s1 (the timed stream), second on s2, both after s1's previous work."""
        def body():
            s2.wait_stream(s1)
            first()
            with torch.cuda.stream(s2):
                second()
            s1.wait_stream(s2)
        return body

    def conc_rev(gemm, side):
        def body():
            s2.wait_stream(s1)
            with torch.cuda.stream(s2):
                side()
            gemm()
            s1.wait_stream(s2)
        return body

    timeit("dgrad", dgrad)
    timeit("wgrad_plain", lambda: wgrad(False))
    timeit("wgrad_fused_sgd", lambda: wgrad(True))
    for b in (0, 256, 512, 1024):
        timeit(f"sgd_grid{b or 'default'}", lambda b=b: sgd(b))
    for b in (0, 256, 512):
        timeit(f"dgrad_then_sgd{b or 'default'}_concurrent", conc(dgrad, lambda b=b: sgd(b)))
        timeit(f"sgd{b or 'default'}_then_dgrad_concurrent", conc_rev(dgrad, lambda b=b: sgd(b)))
    timeit("pair_fused: wgrad+sgd epilogue ; dgrad", lambda: (wgrad(True), dgrad()))

    for b in (256, 512):
        def pair(b=b):
            wgrad(False)
            s2.wait_stream(s1)
            dgrad()
            with torch.cuda.stream(s2):
                sgd(b)
            s1.wait_stream(s2)
        timeit(f"pair_split: wgrad ; (dgrad || sgd{b})", pair)


if __name__ == "__main__":
    main()

"""Weight-gradient tile probe (round 6): the proxy step's three 512 x 512 weight gradients stacked
as one M = 1,536 x N = 512, K = 8,192 weight gradient (same operand bytes and FLOPs as the grouped
launch), through linear_wgrad_bf16 with the 128 x 128 DMA tile or the 256 x 256 ping-pong tile and
split-K caps: GEMM + split-K combine per call (CUDA events, 200 calls).  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split.  Usage: r6_wgrad_tile_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NNMPI_EXPERIMENTS", "1")
import torch  # noqa: E402
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402

lib = native.lib()
dev = torch.device("cuda", 0)
M, N, K = 1536, 512, 8192
g = torch.Generator(device=dev).manual_seed(1)
dZ = (torch.randn(K, M, device=dev, generator=g) * 0.1).to(torch.bfloat16)
X = (torch.randn(K, N, device=dev, generator=g)).to(torch.bfloat16)
ref = (dZ.float().t() @ X.float())
s = torch.cuda.current_stream().cuda_stream
for tile, cap in [(128, 0), (128, 4), (256, 0), (256, 8), (256, 4), (128, 0)]:
    assert lib.set_gemm_tile(tile)
    assert lib.set_wgrad_splits(cap)
    S = lib.wgrad_splits(M, N, K)
    ws = torch.empty(max(1, lib.wgrad_workspace_bytes(M, N, K)) // 4 + 16, device=dev)
    dW = torch.empty(M, N, device=dev)
    db = torch.empty(M, device=dev)
    call = lambda: lib.linear_wgrad_bf16(dZ.data_ptr(), M, X.data_ptr(), N, dW.data_ptr(), db.data_ptr(),
                                         M, N, K, ws.data_ptr(), s)
    for _ in range(20):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        call()
    e1.record()
    torch.cuda.synchronize()
    err = float((dW - ref).norm() / ref.norm())
    print(f"tile {tile} cap {cap}: splits {S}  {e0.elapsed_time(e1) / 200 * 1e3:7.2f} us per call  rel err {err:.2e}",
          flush=True)
lib.set_gemm_tile(0)
lib.set_wgrad_splits(0)

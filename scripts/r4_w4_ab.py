"""4-wave 256x256 forward tile (gemm_w4.hip) vs the production 8-wave ping-pong kernel on the
8192-wide forward (X [4096 x 8192] . W^T [8192 x 8192] + b, relu, bf16): interleaved timing
(hip events, median of 5 rounds x 10 launches) and bitwise comparison of the outputs."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402

lib = native.lib()
M, N, K = 4096, 8192, 8192
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
X = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
W = (torch.randn(N, K, generator=g) * 0.02).to(dev, torch.bfloat16)
b = torch.randn(N, generator=g).to(dev)
Y0 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
Y1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
RELU = 1


def pp():
    lib.linear_fwd_bf16(X.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), Y0.data_ptr(), N, M, N, K, RELU, s)


def w4():
    lib.gemm_w4_fwd(X.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), Y1.data_ptr(), N, M, N, K, RELU, s)


pp(); w4(); torch.cuda.synchronize()
print("bitwise equal:", torch.equal(Y0, Y1), " max |diff|:", float((Y0.float() - Y1.float()).abs().max()))
res = {"pp256": [], "w4": []}
for r in range(5):
    for name, f in (("pp256", pp), ("w4", w4)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
for k, v in res.items():
    print(f"{k}: median {statistics.median(v):.1f} us  min {min(v):.1f} us  "
          f"({2 * M * N * K / statistics.median(v) / 1e6:.0f} TFLOP/s)")

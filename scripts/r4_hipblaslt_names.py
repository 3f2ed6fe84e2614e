"""Which hipBLASLt kernels torch runs for the 8192-wide layer GEMMs (ISA
tabulation against gemm_bf16_pp256_kernel).  Run under rocprofv3 --kernel-trace --stats; the
kernel names land in the stats CSV.  Shapes as profiles/gemm_ab_wide8192_mnist_vs_hipblaslt.json:
forward X[4096x8192] . W^T, dgrad dZ . W, wgrad dZ^T . X (bf16 in / out, fp32 accumulate)."""
import torch

rows, n = 4096, 8192
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(rows, n, device=dev, dtype=torch.bfloat16, generator=g)
W = torch.randn(n, n, device=dev, dtype=torch.bfloat16, generator=g)
dZ = torch.randn(rows, n, device=dev, dtype=torch.bfloat16, generator=g)
for _ in range(3):
    torch.nn.functional.linear(X, W)      # forward
    dZ @ W                                # dgrad
    dZ.t() @ X                            # wgrad
torch.cuda.synchronize()
print("done")

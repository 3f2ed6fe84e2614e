"""Does the 8192-wide weight gradient pay for its operand layout?  The 256x256 ping-pong kernel
(gemm_bf16_tile, plain fp32 output, no SGD) on the weight-gradient shape M = N = 8192, K = 4096 in
all four operand layouts (KMAJ = K contiguous, as the forward's operands; XMAJ = M / N contiguous,
as the weight gradient's dZ and activations are stored), beside the forward shape (M 4096, N 8192,
K 8192, KMAJ x KMAJ) with the same fp32 output, and hipBLASLt (torch.mm) on the same
products.  Interleaved rounds, one process; median of 20 launches per cell."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402

lib = native.lib()
dev = "cuda"
KMAJ, XMAJ = 0, 1
torch.manual_seed(0)


def t_ms(fn, n=20):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def case(M, N, K, la, lb):
    # A is M x K (KMAJ: [M][K], XMAJ: [K][M]); B is N x K likewise; C = A B^T (M x N fp32)
    A = torch.randn((M, K) if la == KMAJ else (K, M), device=dev).to(torch.bfloat16)
    B = torch.randn((N, K) if lb == KMAJ else (K, N), device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def ours():
        lib.gemm_bf16_tile(A.data_ptr(), A.shape[1], la, B.data_ptr(), B.shape[1], lb, M, N, K,
                           C.data_ptr(), N, 256, s)

    Am = A if la == KMAJ else A.t()
    Bm = B.t() if lb == KMAJ else B

    def blas():
        torch.mm(Am, Bm, out=None)

    ours()
    torch.cuda.synchronize()
    ref = (Am.float() @ Bm.float())
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    return ours, blas, err


cases = {
    "wgrad XMAJ x XMAJ (production layout)": (8192, 8192, 4096, XMAJ, XMAJ),
    "wgrad KMAJ x KMAJ (pre-transposed)": (8192, 8192, 4096, KMAJ, KMAJ),
    "wgrad KMAJ x XMAJ": (8192, 8192, 4096, KMAJ, XMAJ),
    "wgrad XMAJ x KMAJ": (8192, 8192, 4096, XMAJ, KMAJ),
    "forward shape KMAJ x KMAJ (fp32 out)": (4096, 8192, 8192, KMAJ, KMAJ),
}
fns = {}
for name, (M, N, K, la, lb) in cases.items():
    o, b, err = case(M, N, K, la, lb)
    fns[name] = (o, b, 2.0 * M * N * K)
    print(f"{name}: rel max err vs fp32 {err:.2e}", flush=True)
res = {n: ([], []) for n in fns}
for rnd in range(3):
    for n, (o, b, fl) in fns.items():
        res[n][0].append(t_ms(o))
        res[n][1].append(t_ms(b))
    print(f"round {rnd} done", flush=True)
for n, (o, b, fl) in fns.items():
    mo, mb = statistics.median(res[n][0]), statistics.median(res[n][1])
    print(f"{n:42s} ours {mo * 1e3:7.1f} us ({fl / mo / 1e9:6.0f} TF)   hipBLASLt {mb * 1e3:7.1f} us "
          f"({fl / mb / 1e9:6.0f} TF)   rounds ours {[round(x * 1e3, 1) for x in res[n][0]]}")

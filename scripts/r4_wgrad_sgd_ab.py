"""Where does the 8192-wide weight gradient + fused SGD spend its time, and does a 2-blocks-per-CU
tile hide the update?  linear_wgrad_bf16 on the wide shape (out = in = 8192, 4096 rows), one
process, interleaved rounds, median of 10 launches per cell:
  sgd/256   production: 256x256 ping-pong tile (1 block per CU), SGD-momentum in the epilogue
  plain/256 the same GEMM storing the fp32 gradient (no update)
  sgd/128   128x128 DMA tile (2 blocks per CU: one block's epilogue beside the other's main loop)
  plain/128
The sgd/128 update must equal sgd/256 bit for bit (same per-element accumulation order).
Then the epilogue's bound: sgd - plain per tile round at out = in = 8192 / 4096 / 2048 (1024 /
256 / 64 tiles, i.e. 4 rounds on 256 CUs / 1 round on 256 / 1 round on 64 CUs): the same per-tile
cost at 64 CUs means the update is bound per CU; a 4x smaller cost means it is bound by HBM
(all CUs updating at once).  Needs NNMPI_EXPERIMENTS=1 (set_gemm_tile)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402

lib = native.lib()
dev = "cuda"
rows, M, N = 4096, 8192, 8192
torch.manual_seed(0)
dz = (torch.randn(rows, M, device=dev) * 0.1).to(torch.bfloat16)
x = torch.relu(torch.randn(rows, N, device=dev)).to(torch.bfloat16)
P = M * N + M
G = torch.zeros(P, device=dev)
W0 = torch.randn(P, device=dev) * 0.01
Mo0 = torch.randn(P, device=dev) * 0.001
W, Mo = W0.clone(), Mo0.clone()
S = torch.zeros(P, device=dev, dtype=torch.bfloat16)
hp = torch.tensor([0.01, 0.9, 0.0, 0.0, 1.0], device=dev)
ws = torch.zeros(max(int(lib.wgrad_workspace_bytes(M, N, rows)), 16) // 4, device=dev)
s = torch.cuda.current_stream().cuda_stream
sgd = (G.data_ptr(), W.data_ptr(), Mo.data_ptr(), S.data_ptr(), hp.data_ptr(), 0, 0)
assert lib.experiments_on(), "run with NNMPI_EXPERIMENTS=1"


def run(tile, fused):
    lib.set_gemm_tile(tile)
    lib.linear_wgrad_bf16(dz.data_ptr(), M, x.data_ptr(), N, G.data_ptr(), G[M * N:].data_ptr(),
                          M, N, rows, ws.data_ptr(), s, sgd if fused else None)
    lib.set_gemm_tile(0)


def t_ms(fn, n=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


# bitwise: one update from the same state through each tile
out = {}
for tile in (0, 128):
    W.copy_(W0)
    Mo.copy_(Mo0)
    run(tile, True)
    torch.cuda.synchronize()
    out[tile] = (W.clone(), Mo.clone(), S.clone())
eq = all(torch.equal(a, b) for a, b in zip(out[0], out[128]))
print(f"sgd/128 update bitwise equal to sgd/256: {eq}", flush=True)
cells = {"sgd/256": (0, True), "plain/256": (0, False), "sgd/128": (128, True), "plain/128": (128, False)}
res = {k: [] for k in cells}
for rnd in range(3):
    for k, (tile, fused) in cells.items():
        res[k].append(t_ms(lambda: run(tile, fused)))
    print(f"round {rnd} done", flush=True)
for k in cells:
    print(f"{k:10s} {statistics.median(res[k]) * 1e3:7.1f} us   rounds {[round(v * 1e3, 1) for v in res[k]]}")

for n in (8192, 4096, 2048):
    d = dz[:, :n].contiguous()
    xx = x[:, :n].contiguous()
    sg = (G.data_ptr(), W.data_ptr(), Mo.data_ptr(), S.data_ptr(), hp.data_ptr(), 0, 0)

    def go(fused):
        lib.linear_wgrad_bf16(d.data_ptr(), n, xx.data_ptr(), n, G.data_ptr(), G[n * n:].data_ptr(),
                              n, n, rows, ws.data_ptr(), s, sg if fused else None)

    a = statistics.median([t_ms(lambda: go(True)) for _ in range(3)]) * 1e3
    b = statistics.median([t_ms(lambda: go(False)) for _ in range(3)]) * 1e3
    tiles = (n // 256) ** 2
    rounds = max(1, tiles // 256)
    print(f"out=in={n}: {tiles} tiles, sgd {a:7.1f} us, plain {b:7.1f} us, update exposed "
          f"{a - b:6.1f} us = {(a - b) / rounds:5.1f} us per tile round", flush=True)

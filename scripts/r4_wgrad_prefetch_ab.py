"""The 8192-wide weight gradient + fused SGD with the in-loop operand prefetch (set_pp_prefetch
0 off / 1 default policy / 2 nt), one process, interleaved rounds, median of 10 launches per
cell; every variant's update bit for bit against no prefetch.  (A one-round-trip-per-half
epilogue form was measured with this script as cell "form 3" and removed again:
profiles/r4_wgrad_sgd_epilogue_bound.txt.)  Needs NNMPI_EXPERIMENTS=1."""
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


def run(pf, fused=True, form=0):
    assert lib.set_pp_prefetch(pf)
    assert lib.set_sgd_epilogue(form)
    lib.linear_wgrad_bf16(dz.data_ptr(), M, x.data_ptr(), N, G.data_ptr(), G[M * N:].data_ptr(),
                          M, N, rows, ws.data_ptr(), s, sgd if fused else None)


def t_ms(fn, n=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


cells = {"form 0, PF 0 (default)": (0, 0), "form 0, PF 1 (default policy)": (1, 0),
         "form 0, PF 2 (nt)": (2, 0)}
out = {}
for k, (pf, form) in cells.items():
    W.copy_(W0)
    Mo.copy_(Mo0)
    run(pf, True, form)
    torch.cuda.synchronize()
    out[k] = (W.clone(), Mo.clone(), S.clone(), G[M * N:].clone())
k0 = next(iter(cells))
for k in cells:
    eq = all(torch.equal(a, b) for a, b in zip(out[k0], out[k]))
    print(f"{k}: update (master, momentum, bf16 shadow, bias grad) bitwise equal to {k0}: {eq}",
          flush=True)
res = {k: [] for k in cells}
plain = []
for rnd in range(4):
    for k, (pf, form) in cells.items():
        res[k].append(t_ms(lambda: run(pf, True, form)))
    plain.append(t_ms(lambda: run(0, False)))
    print(f"round {rnd} done", flush=True)
for k in cells:
    print(f"{k:32s} {statistics.median(res[k]) * 1e3:7.1f} us   rounds {[round(v * 1e3, 1) for v in res[k]]}")
print(f"{'plain (no update)':32s} {statistics.median(plain) * 1e3:7.1f} us   rounds {[round(v * 1e3, 1) for v in plain]}")
lib.set_pp_prefetch(-1)
lib.set_sgd_epilogue(-1)

"""CU-partitioned concurrency for the 8192-wide backward: the weight gradient + fused SGD of layer
l (whose update epilogue is HBM-bound when all 256 CUs reach it at once: profiles/
r4_wgrad_sgd_epilogue_bound.txt) runs on one CU-masked stream while the independent dgrad of
layer l-1 (compute-bound, reads W_{l-1}) runs on another, vs the two back to back on the whole
chip.  Masks: k of 256 CUs to the wgrad, by even / odd bit split and by a contiguous split.
Outputs compared bit for bit against the sequential run.  One process, median of 5 per cell."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402

lib = native.lib()
dev = "cuda"
rows, H = 4096, 8192
torch.manual_seed(0)
dz = (torch.randn(rows, H, device=dev) * 0.1).to(torch.bfloat16)       # dZ_l
a_prev = torch.relu(torch.randn(rows, H, device=dev)).to(torch.bfloat16)  # a_{l-1} (= pre-act for dgrad)
dz2 = (torch.randn(rows, H, device=dev) * 0.1).to(torch.bfloat16)      # dZ_{l-1}
W2 = (torch.randn(H, H, device=dev) * 0.01).to(torch.bfloat16)          # W_{l-1}
dX = torch.empty(rows, H, device=dev, dtype=torch.bfloat16)
P = H * H + H
G = torch.zeros(P, device=dev)
W0 = torch.randn(P, device=dev) * 0.01
Mo0 = torch.randn(P, device=dev) * 0.001
W, Mo = W0.clone(), Mo0.clone()
S = torch.zeros(P, device=dev, dtype=torch.bfloat16)
hp = torch.tensor([0.01, 0.9, 0.0, 0.0, 1.0], device=dev)
ws = torch.zeros(max(int(lib.wgrad_workspace_bytes(H, H, rows)), 16) // 4, device=dev)
sgd = (G.data_ptr(), W.data_ptr(), Mo.data_ptr(), S.data_ptr(), hp.data_ptr(), 0, 0)
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
print(f"CUs: {n_cu}", flush=True)


def wgrad(st):
    lib.linear_wgrad_bf16(dz.data_ptr(), H, a_prev.data_ptr(), H, G.data_ptr(), G[H * H:].data_ptr(),
                          H, H, rows, ws.data_ptr(), st, sgd)


def dgrad(st):
    lib.linear_dgrad_bf16(dz2.data_ptr(), H, W2.data_ptr(), H, a_prev.data_ptr(), H, dX.data_ptr(), H,
                          rows, H, H, 1, st)


def mask_of(bits):
    m = [0] * ((n_cu + 31) // 32)
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    return m


def timed(fn, n=5):
    out = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return statistics.median(out)


main = torch.cuda.current_stream()


def seq():
    dgrad(main.cuda_stream)
    wgrad(main.cuda_stream)


def make_conc(sa, sb):
    ea, eb = torch.cuda.ExternalStream(sa), torch.cuda.ExternalStream(sb)

    def conc():
        ev0 = torch.cuda.Event()
        ev0.record(main)
        ea.wait_event(ev0)
        eb.wait_event(ev0)
        wgrad(sa)
        dgrad(sb)
        e1, e2 = torch.cuda.Event(), torch.cuda.Event()
        e1.record(ea)
        e2.record(eb)
        main.wait_event(e1)
        main.wait_event(e2)
    return conc


def reset():
    W.copy_(W0)
    Mo.copy_(Mo0)


reset()
seq()
torch.cuda.synchronize()
ref = (W.clone(), Mo.clone(), S.clone(), dX.clone())
splits = {}
for k in (128, 144, 160):
    splits[f"even/odd-ish k={k}"] = ([i for i in range(n_cu) if (i % 16) < k * 16 // n_cu],
                                     [i for i in range(n_cu) if (i % 16) >= k * 16 // n_cu])
    splits[f"contiguous k={k}"] = (list(range(k)), list(range(k, n_cu)))
streams = {}
for name, (ba, bb) in splits.items():
    streams[name] = (lib.cu_mask_stream(mask_of(ba)), lib.cu_mask_stream(mask_of(bb)))
res = {"sequential (whole chip)": []}
for name in splits:
    res[name] = []
    res[name + " wgrad alone"] = []
    res[name + " dgrad alone"] = []
for rnd in range(3):
    reset()
    res["sequential (whole chip)"].append(timed(seq))
    for name, (sa, sb) in streams.items():
        conc = make_conc(sa, sb)
        reset()
        conc()
        torch.cuda.synchronize()
        if rnd == 0:
            got = (W.clone(), Mo.clone(), S.clone(), dX.clone())
            print(f"{name}: outputs bitwise equal to sequential: "
                  f"{all(torch.equal(x, y) for x, y in zip(ref, got))}", flush=True)
        res[name].append(timed(conc))
        res[name + " wgrad alone"].append(timed(lambda: (wgrad(sa), torch.cuda.ExternalStream(sa).synchronize())))
        res[name + " dgrad alone"].append(timed(lambda: (dgrad(sb), torch.cuda.ExternalStream(sb).synchronize())))
    print(f"round {rnd} done", flush=True)
for k, v in res.items():
    print(f"{k:40s} {statistics.median(v):8.1f} us   rounds {[round(x, 1) for x in v]}")
for sa, sb in streams.values():
    lib.stream_destroy(sa)
    lib.stream_destroy(sb)

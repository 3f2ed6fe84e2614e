"""Per-block stamps of the proxy step's grouped weight-gradient launch (wgrad_multi_kernel) and
the XCD / CU each row band and each weight-gradient block ran on: block start skew, block
durations, blocks per CU, and whether split s of the weight gradients ran on the XCD that wrote
its rows (row-band band -> XCC id).  Usage: r5_wg_stamps.py [iters]"""
import collections
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rows = 8192
dev = torch.device("cuda", 0)
widths = [512, 512, 512, 512, 1]
spec = MLPSpec(tuple(widths), "relu", "mse")
arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev, shadow_dtype=torch.bfloat16)
arena.bind_model(reference_init(widths))
graph = os.environ.get("R5_GRAPH", "1") == "1"
eng = MLPEngine(spec, arena, HipOps(dev), NoSync(arena), device=dev, dtype=torch.bfloat16,
                rows_capacity=rows, lr=1e-5, momentum=0.9, use_graph=graph)
X, Y = synth.chunked_regression(0, rows, widths[0], device=dev)
eng.load_batch(X.to(torch.bfloat16), Y)
eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
lib = native.lib()
NB = 512
wst = torch.zeros(1024 * 4 + NB * 128, dtype=torch.int64, device=dev)
nbands = lib.rowband_blocks(rows)
slots = lib.rowband_stamp_slots()
NST = slots // 8
rst = torch.zeros(nbands * slots, dtype=torch.int64, device=dev)
lib.set_wgrad_multi_stamps(wst.data_ptr())
if os.environ.get("R5_RBSTAMPS", "0") == "1":
    lib.set_rowband_stamps(rst.data_ptr())
# (graph mode: the stamp buffers are baked into the captured launches)
eng.run_steps(1, 1)
eng.prepare_steps(16, 16)
for _ in range(20):
    eng.run_steps(16, 16)
torch.cuda.synchronize()
durs, skews, spans, percu, aligned = [], [], [], [], []
for it in range(iters):
    wst.zero_()
    eng.run_steps(16, 16)
    torch.cuda.synchronize()
    if it < 3:
        continue
    w = wst[:NB * 4].view(NB, 4).cpu().tolist()
    w = [r for r in w if r[0] != 0]
    t0 = min(r[0] for r in w)
    spans.append((max(r[1] for r in w) - t0) / 100.0)
    skews.append((max(r[0] for r in w) - t0) / 100.0)
    durs += [(r[1] - r[0]) / 100.0 for r in w]
    cu = collections.Counter((r[2] & 15, r[3] >> 8 & 0xFFFF) for r in w)
    percu.append(max(cu.values()))
    # row band -> XCC (stamp slots NST-4: XCC id written by the ST kernel)
    rb = rst.view(nbands, 8, NST)[:, 0, NST - 4].cpu().tolist()
    if it == iters - 1:
        print("blocks", len(w), "launch span median", f"{statistics.median(spans):.2f} us",
              "start skew", f"{statistics.median(skews):.2f} us")
        d = sorted(durs)
        print(f"block duration: min {d[0]:.2f} p10 {d[len(d)//10]:.2f} median {statistics.median(d):.2f} "
              f"p90 {d[9*len(d)//10]:.2f} max {d[-1]:.2f} us")
        print("max blocks on one CU:", collections.Counter(percu))
        xcc_of_block = [r[2] & 15 for r in wst[:NB * 4].view(NB, 4).cpu().tolist()[:len(w)]]
        # per k-step phases (wave 0 of each block): ring wait, barrier, DMA issue, reads + MFMAs
        k = wst[1024 * 4:].view(NB, 128)[:len(w), :128].view(len(w), 32, 4).double()
        nt = int((k[0, :, 0] > 0).sum())
        kk = k[:, :nt]
        bar = kk[:, :, 1] - kk[:, :, 0]
        dma = kk[:, :, 2] - kk[:, :, 1]
        comp = kk[:, :, 3] - kk[:, :, 2]
        wait = kk[:, 1:, 0] - kk[:, :-1, 3]
        print(f"k-steps {nt}: per k-step median cycles: wait {wait.median():.0f}  barrier "
              f"{bar.median():.0f}  DMA issue {dma.median():.0f}  reads+MFMA {comp.median():.0f};  "
              f"wave-0 main loop {(kk[:, -1, 3] - kk[:, 0, 0]).median():.0f} cycles")
        print("wgrad block -> XCC (first 32):", xcc_of_block[:32])
        print("row band -> XCC (first 40):", [int(x) & 15 for x in rb[:40]])
lib.set_wgrad_multi_stamps(0)
lib.set_rowband_stamps(0)

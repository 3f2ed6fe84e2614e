"""Phase stamps of the column-split row-band kernel (rowband.hip rowband_split_kernel, ST build) on
the proxy shape (512-wide, 3 hidden layers, relu, MSE) at a small batch: wave 0's shader clock at
every phase boundary -- main loops, epilogue + copy-out, the hand-offs' store drain + barrier, the
poll, the gather -- median over blocks.  Usage: r5_split_stamps.py [rows] [iters]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NNMPI_EXPERIMENTS", "1")
os.environ.setdefault("NNMPI_ROWBAND_MIN_ROWS", "6144")
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda", 0)
widths = [512, 512, 512, 512, 1]
spec = MLPSpec(tuple(widths), "relu", "mse")
arena = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev, shadow_dtype=torch.bfloat16)
arena.bind_model(reference_init(widths))
eng = MLPEngine(spec, arena, HipOps(dev), NoSync(arena), device=dev, dtype=torch.bfloat16,
                rows_capacity=rows, lr=1e-5, momentum=0.9, use_graph=False)
X, Y = synth.chunked_regression(0, rows, widths[0], device=dev)
eng.load_batch(X.to(torch.bfloat16), Y)
eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
assert eng.uses_rowband_split(rows), "the split kernel does not take this batch"
lib = native.lib()
NST = lib.rowband_split_stamp_slots()
st = torch.zeros(256 * NST, dtype=torch.int64, device=dev)
for _ in range(200):
    eng.step()
torch.cuda.synchronize()
names = ["startup", "f0 main", "f0 epi+put", "f0 drain+bar", "f0 wait", "f0 gather",
         "f1 main", "f1 epi+put", "f1 drain+bar", "f1 wait", "f1 gather", "f2 main",
         "hd epi+dot", "hd drain+bar", "hd wait", "hd part+dz", "dz drain+bar", "dz wait",
         "dz gather", "d2 main", "d2 epi+put", "d2 drain+bar", "d2 wait", "d2 gather",
         "d1 main", "d1 epi+end"]
per = {n: [] for n in names}
spread = {n: [] for n in names}
tot = []
lib.set_rowband_stamps(st.data_ptr())
try:
    for it in range(iters):
        st.zero_()
        eng.step()
        torch.cuda.synchronize()
        if it < 4:
            continue
        t = st.view(256, NST).cpu()
        nb = int((t[:, 0] != 0).sum())
        t = t[:nb]
        tot.append(float((t[:, len(names)] - t[:, 0]).double().median()))
        for i, n in enumerate(names):
            d = (t[:, i + 1] - t[:, i]).double()
            per[n].append(float(d.median()))
            spread[n].append(float((t[:, i + 1].max() - t[:, i + 1].min())))
finally:
    lib.set_rowband_stamps(0)
clk = 2.0e3   # cycles per us at ~2.0 GHz (s_memtime counts the shader clock)
print(f"rows {rows}, blocks {nb}; median block span {statistics.median(tot):.0f} cyc "
      f"(~{statistics.median(tot) / clk:.2f} us at 2.0 GHz)")
for n in names:
    c = statistics.median(per[n])
    print(f"  {n:14s} {c:8.0f} cyc {c / clk:6.2f} us   end spread over blocks {statistics.median(spread[n]):8.0f} cyc")

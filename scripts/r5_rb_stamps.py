"""Phase stamps of the v2 row-band kernel (rowband.hip rowband2_kernel, ST build) on the proxy
step (8192 x 512, 3 hidden layers, relu, MSE): per wave the shader clock at every phase boundary
(main loop done, epilogue stores issued, barrier passed, copy-out issued; head; dgrads).  Prints the
median over blocks of each phase (cycles and us at the measured in-kernel clock), the spread
between the 8 waves of a block, and the kernel span.  Usage: r5_rb_stamps.py [rows] [iters]"""
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

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
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
print("schedule", eng.schedule_name())
lib = native.lib()
nb = lib.rowband_blocks(rows)
slots = lib.rowband_stamp_slots()
NST = slots // 8
st = torch.zeros(nb * slots, dtype=torch.int64, device=dev)
for _ in range(200):     # DVFS warm-up, unstamped
    eng.step()
torch.cuda.synchronize()
lib.set_rowband_stamps(st.data_ptr())
nh = len(widths) - 2
names = ["st issue", "st ring", "st wait", "st lds", "st bar"]
for l in range(nh):
    names += [f"fwd{l} main", f"fwd{l} epi", f"fwd{l} copy", f"fwd{l} bar"]
names += ["hd dot+copy", "hd bar1", "hd part", "hd bar2", "hd dz", "head bar"]
for l in range(nh - 1, 0, -1):
    names += [f"dg{l} main", f"dg{l} epi", f"dg{l} copy", f"dg{l} bar"]
names += ["last copy"]
per = {n: [] for n in names}
wave_skew = {n: [] for n in names}
spans, clocks, starts = [], [], []
for it in range(iters):
    st.zero_()
    eng.step()
    torch.cuda.synchronize()
    if it < 4:
        continue
    t = st.view(nb, 8, NST).cpu()
    rt0 = t[:, 0, NST - 2]
    rt1 = t[:, 0, NST - 1]
    spans.append((int(rt1.max()) - int(rt0.min())) / 100.0)
    starts.append((int(rt0.max()) - int(rt0.min())) / 100.0)
    cyc_total = (t[:, 0, len(names)] - t[:, 0, 0]).double()
    rt_total = (rt1 - rt0).double() / 100.0
    clocks.append(float((cyc_total / rt_total).median()))   # cycles per us
    for i, n in enumerate(names):
        d = (t[:, :, i + 1] - t[:, :, i]).double()   # [blocks, waves]
        per[n].append(float(d.median()))
        wave_skew[n].append(float((t[:, :, i + 1].max(1).values - t[:, :, i + 1].min(1).values).double().median()))
lib.set_rowband_stamps(0)
clk = statistics.median(clocks)
print(f"blocks {nb}; kernel span {statistics.median(spans):.2f} us (block start spread "
      f"{statistics.median(starts):.2f} us); in-kernel clock {clk / 1e3:.3f} GHz")
tot = 0.0
for n in names:
    c = statistics.median(per[n])
    tot += c
    print(f"  {n:12s} {c:9.0f} cyc {c / clk:7.2f} us   wave spread at end {statistics.median(wave_skew[n]):7.0f} cyc")
print(f"  {'sum':12s} {tot:9.0f} cyc {tot / clk:7.2f} us")

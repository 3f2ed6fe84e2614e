"""Per-block real-time stamps of the small-batch weight-gradient launch (gemm_bf16.hip
wgrad_small_kernel: entry, GEMM done, exit; set_wgrad_multi_stamps) on the proxy shape at a small
batch: kernel span, block start spread, GEMM / epilogue / whole-block durations of the GEMM blocks
and of the head-combine blocks.  Usage: r5_wgs_stamps.py [rows] [iters]"""
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
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
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
assert eng.uses_rowband_split(rows)
lib = native.lib()
st = torch.zeros(1024 * 4, dtype=torch.int64, device=dev)
for _ in range(200):
    eng.step()
torch.cuda.synchronize()
span, spread, gemm, epi, blk, tail = [], [], [], [], [], []
lib.set_wgrad_multi_stamps(st.data_ptr())
try:
    for it in range(iters):
        st.zero_()
        eng.step()
        torch.cuda.synchronize()
        if it < 4:
            continue
        t = st.view(1024, 4).cpu()
        used = t[:, 0] != 0
        t = t[used].double() / 100.0   # us
        g = t[:, 1] != 0 * t[:, 1]
        isg = t[:, 1] > 0
        span.append(float(t[:, 2].max() - t[:, 0].min()))
        spread.append(float(t[:, 0].max() - t[:, 0].min()))
        gemm.append(float((t[isg, 1] - t[isg, 0]).median()))
        epi.append(float((t[isg, 2] - t[isg, 1]).median()))
        blk.append(float((t[isg, 2] - t[isg, 0]).median()))
        if (~isg).any():
            tail.append(float((t[~isg, 2] - t[~isg, 0]).max()))
finally:
    lib.set_wgrad_multi_stamps(0)
m = statistics.median
print(f"rows {rows}: blocks {int(used.sum())} (gemm {int(isg.sum())}); kernel span {m(span):.2f} us, "
      f"block start spread {m(spread):.2f} us")
print(f"  gemm blocks: main loop {m(gemm):.2f} us, epilogue {m(epi):.2f} us, whole {m(blk):.2f} us")
if tail:
    print(f"  head-combine blocks: longest {m(tail):.2f} us")

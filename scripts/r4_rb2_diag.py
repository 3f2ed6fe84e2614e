"""Row-band v2 multi-step diagnostics: the fused combine's image writes vs a fresh pack, and the
v1 / v2 trajectories over a few eager steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402


def make(v, widths, rows, graph=False):
    os.environ["NNMPI_RB_V2"] = "1" if v == 2 else "0"
    os.environ["NNMPI_ROWBAND"] = "1"
    spec = MLPSpec(tuple(widths), "relu", "mse")
    ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda", shadow_dtype=torch.bfloat16)
    ar.bind_model(reference_init(widths, "relu", seed=3))
    eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                    rows_capacity=rows, lr=1e-3, momentum=0.9, use_graph=graph)
    X, Y = synth.chunked_regression(0, rows, widths[0], out=1, device="cuda")
    eng.load_batch(X.to(torch.bfloat16), Y)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    return spec, ar, eng


widths, rows = [512, 512, 512, 512, 1], 8192
spec, ar, eng = make(2, widths, rows)
print("rb_version", eng.rb_version, "fuse_sgd", eng.fuse_sgd)
eng.step()
eng.synchronize()
img = eng._rb_buf.clone()
print("fresh after step", eng._rb_current())
with torch.cuda.stream(eng.stream):
    eng._rb_pack()
eng.synchronize()
d = (img.float() - eng._rb_buf.float()).abs()
print("combine images vs fresh pack: max abs diff", float(d.max()), "n diff", int((d > 0).sum()),
      "of", d.numel())
for l, (pf, pd) in enumerate(eng.rb_packed):
    o = pf.data_ptr() - eng._rb_buf.data_ptr()
    o //= 2
    dd = d[o:o + pf.numel()]
    print(" layer", l, "fwd image diffs", int((dd > 0).sum()))
    if pd is not None:
        o2 = (pd.data_ptr() - eng._rb_buf.data_ptr()) // 2
        dd = d[o2:o2 + pd.numel()]
        print(" layer", l, "dgrad image diffs", int((dd > 0).sum()))
res = {}
for v in (1, 2):
    for graph in (False, True):
        _, ar, eng = make(v, widths, rows, graph)
        losses = []
        for _ in range(6):
            eng.step()
            losses.append(eng.loss())
        res[(v, graph)] = (losses, ar.master.double().cpu())
        print("v", v, "graph", graph, ["%.5f" % x for x in losses])
p1 = res[(1, False)][1]
for k, (l, p) in res.items():
    print(k, "rel param diff vs v1 eager", float((p - p1).norm() / p1.norm()))

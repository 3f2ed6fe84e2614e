"""(experiment check) three fused-update proxy steps with the full-batch image path
(set_rb_wkimg(1)) against the row-major path: relative parameter difference and losses."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNMPI_EXPERIMENTS"] = "1"
import torch  # noqa: E402
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

lib = native.lib()
for widths, rows in [([512, 512, 512, 512, 1], 8192), ([512, 512, 512, 512, 1], 6000),
                     ([256, 512, 512, 512, 1], 8191)]:
    X, Y = synth.chunked_regression(0, rows, widths[0], device="cuda")
    X = X.to(torch.bfloat16)
    res = []
    for wk in (1, 0):
        assert lib.set_rb_wkimg(wk)
        spec = MLPSpec(tuple(widths), "relu", "mse")
        ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda", shadow_dtype=torch.bfloat16)
        ar.bind_model(reference_init(widths, "relu", seed=3))
        eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                        rows_capacity=rows, lr=1e-3, momentum=0.9, use_graph=False)
        assert eng.uses_rowband(rows) and not eng.uses_rowband_split(rows)
        eng.load_batch(X, Y)
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        losses = []
        for _ in range(3):
            eng.step()
            losses.append(eng.loss())
        res.append((ar.master.double().cpu(), losses))
    lib.set_rb_wkimg(-1)
    (p1, l1), (p2, l2) = res
    rel = float((p1 - p2).norm() / p2.norm())
    print(widths, rows, "param rel diff", rel, "losses", l1, l2, "OK" if rel < 1e-5 else "FAIL", flush=True)
    assert rel < 1e-5

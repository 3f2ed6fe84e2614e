"""Column-split kernel debug: layer-0 activations vs torch for forced blocks-per-band, listing
mismatches (band row, column, got, want)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNMPI_EXPERIMENTS"] = "1"
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

lib = native.lib()
for rows, C, nh in [(1024, 2, 3), (1024, 4, 3), (1024, 8, 3), (2048, 2, 3), (4096, 2, 1), (4096, 2, 2)]:
    lib.set_rb_split(C)
    widths = [512] * (nh + 1) + [1]
    spec = MLPSpec(tuple(widths), "relu", "mse")
    ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda", shadow_dtype=torch.bfloat16)
    ar.bind_model(reference_init(widths, "relu", seed=3))
    eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                    rows_capacity=rows, lr=0.0, momentum=0.0, use_graph=False)
    X, Y = synth.chunked_regression(0, rows, widths[0], out=1, device="cuda")
    Xb = X.to(torch.bfloat16)
    eng.load_batch(Xb, Y)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    eng.rb_keep_last = True
    eng.step()
    torch.cuda.synchronize()
    W0 = ar.compute_weight(0).float()
    ref = torch.relu(Xb.float() @ W0.t() + ar.bias(0).float())
    got = eng.acts[0][:rows].float()
    bad = ((got - ref).abs() > 0.05 * ref.abs() + 0.05).nonzero()
    print(f"rows {rows} C {C} nh {nh} split {eng.uses_rowband_split(rows)} a0 bad {len(bad)}", flush=True)
    for r, c in bad[:12].tolist():
        print(f"   row {r} (band {r // 32} r {r % 32}) col {c}: got {float(got[r, c]):.4g} want {float(ref[r, c]):.4g}")
    if len(bad):
        rr = bad[:, 0] % 32
        print("   band rows:", sorted(set(rr.tolist()))[:10], "cols:", sorted(set(bad[:, 1].tolist()))[:40])
lib.set_rb_split(-1)

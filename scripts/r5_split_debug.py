"""Column-split row-band kernel debug: one step at the given shapes, reports the device error
word and which outputs hold non-finite values.  Usage: r5_split_debug.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNMPI_EXPERIMENTS"] = "1"
import torch  # noqa: E402

from nnmpi_amd.data import synth  # noqa: E402
from nnmpi_amd.engine.arena import Arena  # noqa: E402
from nnmpi_amd.engine.engine import MLPEngine  # noqa: E402
from nnmpi_amd.models.mlp import MLPSpec, reference_init  # noqa: E402
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402
from nnmpi_amd.parallel.sync import NoSync  # noqa: E402

for widths, rows, act, keep in [([512] * 4 + [1], 3001, "tanh", True), ([512] * 4 + [1], 3001, "tanh", False),
                                ([512] * 2 + [1], 3001, "tanh", True), ([512] * 3 + [1], 2047, "tanh", True),
                                ([512] * 4 + [1], 2999, "relu", True), ([512] * 4 + [1], 1024, "tanh", True)]:
    spec = MLPSpec(tuple(widths), act, "mse")
    ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda", shadow_dtype=torch.bfloat16)
    ar.bind_model(reference_init(widths, act, seed=3))
    eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                    rows_capacity=rows, lr=0.0, momentum=0.0, use_graph=False)
    X, Y = synth.chunked_regression(0, rows, widths[0], out=1, device="cuda")
    eng.load_batch(X.to(torch.bfloat16), Y)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    eng.keep = True
    eng.rb_keep_last = keep
    eng.step()
    torch.cuda.synchronize()
    err = int(eng.ws_rb[:1].view(torch.int32).item())
    bad = []
    for i in range(spec.n_layers - 1):
        for nm, t in (("a", eng.acts[i][:rows]), ("dz", eng._dzl(i, rows))):
            f = ~torch.isfinite(t.float())
            if f.any():
                rr = f.any(1).nonzero().flatten()
                bad.append(f"{nm}{i}: {int(f.sum())} bad, rows {int(rr.min())}..{int(rr.max())} "
                           f"({len(rr)} rows) cols {int(f.any(0).nonzero().min())}..{int(f.any(0).nonzero().max())}")
    a0 = eng.acts[0][:rows].float()
    f = (~torch.isfinite(a0)).nonzero()
    vals = [(int(r), int(c), float(a0[r, c])) for r, c in f[:4].tolist()]
    print(widths, rows, act, "keep", keep, "split", eng.uses_rowband_split(rows), "err", err,
          "loss", float(eng.loss_out[0]), bad, vals, flush=True)

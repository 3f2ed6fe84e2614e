"""Stage-by-stage check of the matrix-core general head against torch on the same inputs:
dlogits with and without the dZ GEMM, dZ against its bf16 bound, guard words after dZ."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402

ops = HipOps()
GUARD = 1 << 20
for rows, in_f, out_f, loss in [(64, 8192, 3, "mse"), (64, 8192, 37, "mse"), (64, 2048, 10, "xent"),
                                (256, 8192, 10, "xent"), (64, 4096, 16, "mse"), (64, 4096, 17, "mse")]:
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.relu(torch.randn(rows, in_f, device="cuda", generator=g)).to(torch.bfloat16)
    W = torch.randn(out_f, in_f, device="cuda", generator=g) * 0.05
    b = torch.randn(out_f, device="cuda", generator=g)
    y = torch.randn(rows, out_f, device="cuda", generator=g) if loss == "mse" else None
    lab = (torch.arange(rows, device="cuda") * 7 % out_f) if loss == "xent" else None
    z = a.double() @ W.double().t() + b.double()
    if loss == "mse":
        rdl = 2 * (z - y.double()) / rows
    else:
        p = torch.softmax(z, 1)
        rdl = p.clone()
        rdl[torch.arange(rows), lab] -= 1
        rdl /= rows
    rdz = (rdl @ W.double()) * (a.double() > 0)
    for with_dz in (False, True):
        gW = torch.zeros(out_f, in_f, device="cuda")
        gb = torch.zeros(out_f, device="cuda")
        big = torch.full((rows * in_f + GUARD,), 3.0, device="cuda", dtype=torch.bfloat16)
        dz = big[:rows * in_f].view(rows, in_f) if with_dz else None
        dl = torch.zeros(rows, out_f, device="cuda")
        lo = torch.zeros(4, device="cuda")
        ws = torch.zeros(ops.head_workspace_bytes(rows, in_f, out_f) // 4 + 16, device="cuda")
        ops.head(a, W, b, y, lab, loss, 1.0 / rows, "relu", dz, gW, gb, dl, lo, 1.0 / rows, ws=ws)
        torch.cuda.synchronize()
        dz_err = float((dz.double() - rdz).abs().max()) if with_dz else -1
        guard_bad = int((big[rows * in_f:] != 3.0).sum()) if with_dz else -1
        print(rows, in_f, out_f, loss, "dz" if with_dz else "no dz",
              "dl err", float((dl.double() - rdl).abs().max()), "dl max", float(rdl.abs().max()),
              "dz err", dz_err, "dz max", float(rdz.abs().max()), "guard words changed", guard_bad,
              flush=True)

"""Time the output layer (head) kernels: logits + loss + dlogits + dZ of the last hidden layer +
weight / bias gradient, in one process, median of interleaved rounds, random operands.

Shapes: the general head (head_general.hip: out > 16 or an fp32 weight image over 64 KiB) at
4096 x 8192 -> 10 and 8192 x 1024 -> 100 (softmax cross-entropy) and 8192 x 512 -> 37 (MSE),
next to the skinny MFMA head of the MNIST shape (8192 x 1024 -> 10) and a torch (hipBLASLt +
ATen) rendition of the same math as the vendor reference point.  Prints one JSON line per shape.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd.ops.hip_ops import HipOps  # noqa: E402

SHAPES = [(4096, 8192, 10, "xent"), (8192, 1024, 100, "xent"), (8192, 512, 37, "mse"),
          (8192, 1024, 10, "xent")]


def main(rounds=7, iters=20):
    ops = HipOps()
    dev = "cuda"
    for rows, in_f, out_f, loss in SHAPES:
        a = torch.rand(rows, in_f, device=dev).to(torch.bfloat16)
        W = ((torch.rand(out_f, in_f, device=dev) * 2 - 1) / in_f ** 0.5).contiguous()
        b = torch.rand(out_f, device=dev)
        y = torch.randn(rows, out_f, device=dev) if loss == "mse" else None
        labels = torch.randint(0, out_f, (rows,), device=dev) if loss == "xent" else None
        dz = torch.empty(rows, in_f, device=dev, dtype=torch.bfloat16)
        gW, gb = torch.empty_like(W), torch.empty_like(b)
        dlog = torch.empty(rows, out_f, device=dev)
        lo = torch.zeros(4, device=dev)
        ws = torch.empty(ops.head_workspace_bytes(rows, in_f, out_f, loss) // 4 + 64, device=dev)

        def ours():
            ops.head(a, W, b, y, labels, loss, 1.0 / rows, "relu", dz, gW, gb, dlog, lo,
                     1.0 / rows, ws=ws)

        af = a.float()

        def vendor():
            z = torch.addmm(b, af, W.t())
            if loss == "xent":
                g = torch.softmax(z, 1)
                g[torch.arange(rows, device=dev), labels] -= 1.0
            else:
                g = 2.0 * (z - y)
            g = g / rows
            torch.mm(g.t(), af, out=gW)
            torch.sum(g, 0, out=gb)
            dz.copy_((g @ W) * (af > 0))

        res = {"ours": [], "torch": []}
        for r in range(rounds):
            for name, fn in (("ours", ours), ("torch", vendor)):
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    fn()
                e.record()
                e.synchronize()
                res[name].append(s.elapsed_time(e) * 1e3 / iters)
        # bytes the head must move at least: activations read (bf16) + dZ written (bf16)
        min_bytes = rows * in_f * 2 * 2
        med = statistics.median(res["ours"])
        print(json.dumps({"rows": rows, "in": in_f, "out": out_f, "loss": loss,
                          "path": "general" if ops.head_is_general(out_f, in_f) else "skinny",
                          "median_us": round(med, 2),
                          "torch_median_us": round(statistics.median(res["torch"]), 2),
                          "min_traffic_gbps": round(min_bytes / (med * 1e-6) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()

"""Is the split step reproducible run-to-run inside ONE process (no other process on the GPU)?
Two fresh engines, 20 fused-update steps each, compared per step (loss) and at the end."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import nnmpi_amd  # noqa: E402,F401
from test_split_contention_gpu import _run  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
a = _run(rows, steps)
b = _run(rows, steps)
k = next((i for i, (x, y) in enumerate(zip(a[4], b[4])) if x != y), None)
print(f"rows {rows}: first differing loss step {k}; tensors differing:",
      [n for n, x, y in zip(("master", "momentum", "shadow", "images"), a[:4], b[:4]) if not torch.equal(x, y)])
if k is not None:
    print("losses a", a[4][max(0, k - 2):k + 2], "b", b[4][max(0, k - 2):k + 2])

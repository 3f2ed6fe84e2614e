"""Phase stamps of the fused multi-output head (head_mo.hip, MNIST shape 8192 x 1024 -> 10,
cross-entropy, relu): per block the 100 MHz real-time counter at kernel entry, after the W image
build, after the logits, after the dlogits barrier, after dZ, after each weight-gradient phase
and at exit.  Prints the median per-phase time over blocks and the spread of block starts / ends
(what the kernel's 17 us is made of)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.ops.hip_ops import ACT_CODES, LOSS_CODES, HipOps  # noqa: E402

rows, in_f, out_f = 8192, 1024, 10
dev = "cuda"
lib = native.lib()
ops = HipOps()
g = torch.Generator(device="cpu").manual_seed(0)
a = torch.relu(torch.randn(rows, in_f, generator=g)).to(dev, torch.bfloat16)
W = (torch.randn(out_f, in_f, generator=g) * 0.05).to(dev)
b = torch.randn(out_f, generator=g).to(dev)
lab = (torch.arange(rows) * 7 % out_f).to(dev)
dz = torch.empty(rows, in_f, device=dev, dtype=torch.bfloat16)
gW = torch.empty(out_f, in_f, device=dev)
gb = torch.empty(out_f, device=dev)
lo = torch.zeros(4, device=dev)
ws = torch.zeros(ops.head_workspace_bytes(rows, in_f, out_f) // 4 + 16, device=dev)
parts, off = ops._head_split(rows, in_f, out_f)
st = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
names = ["W image", "logits", "loss+dl", "dZ", "wgrad ph0", "wgrad ph1", "rest+tail"]
per = {n: [] for n in names}
span = []
for it in range(12):
    st.zero_()
    lib.head_mo_fused(a.data_ptr(), rows, in_f, W.data_ptr(), b.data_ptr(), out_f, 0,
                      lab.data_ptr(), LOSS_CODES["xent"], 1.0 / rows, ACT_CODES["relu"],
                      dz.data_ptr(), gW.data_ptr(), gb.data_ptr(), ws[off:].data_ptr(),
                      ws[:parts].data_ptr(), 1.0 / rows, lo.data_ptr(), s, None, False,
                      st.data_ptr())
    torch.cuda.synchronize()
    if it < 2:
        continue
    t = [r for r in st.view(256, 8).cpu().tolist() if r[0] != 0]
    t0 = min(r[0] for r in t)
    span.append((max(r[7] for r in t) - t0) / 100.0)
    for r in t:
        for i, n in enumerate(names):
            per[n].append((r[i + 1] - r[i]) / 100.0)
print(f"blocks {len(t)} (NNMPI_HEAD_BLOCKS={os.environ.get('NNMPI_HEAD_BLOCKS', '-')}); kernel span "
      f"(first block start -> last block end): median {statistics.median(span):.2f} us")
for n in names:
    v = sorted(per[n])
    print(f"  {n:10s} median {statistics.median(v):6.2f} us   p90 {v[int(0.9 * len(v))]:6.2f} us")
starts = [r[0] for r in st.view(256, 8).cpu().tolist() if r[0] != 0]
print(f"block start spread (last run): {(max(starts) - min(starts)) / 100.0:.2f} us")

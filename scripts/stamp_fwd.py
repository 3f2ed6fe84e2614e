"""Where the forward GEMM's per-launch fixed cost goes: per-block entry/exit real-time stamps
(100 MHz) of the default 128x128 forward kernel at 8192 rows x 512 outputs, K = 64 .. 2048.

    python scripts/stamp_fwd.py      -> one JSON line per K
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402

lib = native.lib()
M, N = 8192, 512
dev = "cuda"
for K in (64, 128, 256, 512, 1024, 2048):
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    nb = (M // 128) * (N // 128)
    st = torch.zeros(2 * nb, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    h = int(s.cuda_stream)
    args = (X.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), Y.data_ptr(), N, M, N, K)
    for _ in range(20):
        lib.linear_fwd_bf16_stamped(*args, st.data_ptr(), h)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        lib.linear_fwd_bf16_stamped(*args, st.data_ptr(), h)
    e1.record()
    torch.cuda.synchronize()
    stamped_us = e0.elapsed_time(e1) / reps * 1e3
    e0.record()
    for _ in range(reps):
        lib.linear_fwd_bf16(X.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), Y.data_ptr(), N, M, N, K,
                            1, h)
    e1.record()
    torch.cuda.synchronize()
    plain_us = e0.elapsed_time(e1) / reps * 1e3
    t = st.view(nb, 2).cpu().double() * 0.01          # 100 MHz ticks -> us
    t0, t1 = t[:, 0], t[:, 1]
    span = (t1 - t0).sort().values
    out = {"K": K, "kernel_us_plain": round(plain_us, 2), "kernel_us_stamped": round(stamped_us, 2),
           "dispatch_skew_us": round(float(t0.max() - t0.min()), 2),
           "block_span_us_min_med_max": [round(float(span[0]), 2),
                                         round(float(span[len(span) // 2]), 2),
                                         round(float(span[-1]), 2)],
           "first_entry_to_last_exit_us": round(float(t1.max() - t0.min()), 2),
           "last_exit_minus_median_exit_us": round(float(t1.max() - t1.median()), 2)}
    print(json.dumps(out), flush=True)

"""Per-kernel GEMM durations of the stand-in sweep (scripts/r5_standin.sh): for each k, the mean
and median duration of every GEMM kernel kind over the last steps of the trace, and the same
split by whether a cu_hold kernel overlapped the GEMM in time.  Usage: r5_standin_table.py DIR"""
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]


def load(k):
    f = glob.glob(os.path.join(root, f"k{k}", "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return None
    rows = list(csv.DictReader(open(f[0])))
    out = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    out.sort(key=lambda x: x[1])
    return out


def kind(name):
    if "cu_hold" in name:
        return "hold"
    if "pp256" in name or "gemm_bf16" in name:
        epi = name.split("<")[1].split(",")[2:5] if "<" in name else ["?"]
        return "gemm " + ",".join(x.strip() for x in epi)
    return None


print(f"{'k':>3} {'kernel':42s} {'n':>5} {'mean us':>9} {'median':>9} | {'with hold':>10} {'n':>4} | {'no hold':>9} {'n':>4}")
for k in (0, 1, 8, 32):
    tr = load(k)
    if tr is None:
        continue
    # the last 60 % of the trace: steady steps (after warm-up, capture, tuning)
    tr = tr[int(len(tr) * 0.4):]
    holds = [(s, e) for n, s, e in tr if kind(n) == "hold"]
    by = {}
    for n, s, e in tr:
        kd = kind(n)
        if kd is None or kd == "hold":
            continue
        ov = any(hs < e and he > s for hs, he in holds)
        by.setdefault(kd, []).append(((e - s) / 1e3, ov))
    for kd, v in sorted(by.items()):
        d = [x for x, _ in v]
        w = [x for x, o in v if o]
        nw = [x for x, o in v if not o]
        print(f"{k:3d} {kd[:42]:42s} {len(d):5d} {statistics.mean(d):9.1f} {statistics.median(d):9.1f} | "
              f"{(statistics.median(w) if w else float('nan')):10.1f} {len(w):4d} | "
              f"{(statistics.median(nw) if nw else float('nan')):9.1f} {len(nw):4d}")
    if holds:
        hd = [(e - s) / 1e3 for s, e in holds]
        print(f"{k:3d} {'cu_hold':42s} {len(hd):5d} {statistics.mean(hd):9.1f} {statistics.median(hd):9.1f}")

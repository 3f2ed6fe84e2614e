#!/usr/bin/env python3
"""Steady-state step timeline from a rocprofv3 kernel trace: the last N dispatches in start
order with duration and the gap to the previous dispatch's end (any queue).
Usage: trace_step.py kernel_trace.csv [N]"""
import csv
import sys


def short(n):
    n = n.replace("void ", "").replace("nnmpi::", "")
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
prev_end = None
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{(s - t0) / 1e3:9.2f} us  q{r['Queue_Id']:>2}  dur {(e - s) / 1e3:7.2f}  gap {gap:6.2f}  "
          f"{short(r['Kernel_Name'])}")
    prev_end = e if prev_end is None else max(prev_end, e)

"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch over all groups).

    python scripts/pmc_summary.py gpurun_out/pmc/bench_g*  [--match head_fwd,bwd_group]
"""
import argparse
import collections
import csv
import glob
import os


def short(name):
    n = name.split("(")[0]
    return n.replace("void nnmpi::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="nnmpi")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            seen = set()
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if not any(m in r["Kernel_Name"] for m in a.match.split(",")):
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (r["Dispatch_Id"], f)
                if key not in seen:
                    seen.add(key)
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in vals.items():
        d = sorted(dur[k])[len(dur[k]) // 2]
        print(f"== {k}  (median dispatch {d:.2f} us)")
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()

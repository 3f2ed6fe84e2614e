"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch over all groups).

    python scripts/pmc_summary.py gpurun_out/pmc/bench_g*  [--match head_fwd,bwd_group]

Derived lines (when the counters are present): MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES /
(dispatch time x shader clock x 1024 SIMDs), the clock taken from GRBM_GUI_ACTIVE / 8 XCDs over
the dispatch (falls back to 2.1 GHz); L2 hit rate; LDS bank-conflict cycles per LDS instruction;
fraction of wave cycles spent waiting.
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
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for line in derived(m, d):
            print("   -> " + line)


def derived(m, us):
    out = []
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and us > 0:
        ghz = 2.1
        if "GRBM_GUI_ACTIVE" in m:
            ghz = min(2.4, m["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3))
        busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (us * 1e3 * 2.1 * 1024)
        out.append(f"MFMA pipe busy {100 * busy:5.1f} % at 2.1 GHz "
                   f"(GUI_ACTIVE clock {ghz:.2f} GHz)")
    if "TCC_HIT_sum" in m and m.get("TCC_MISS_sum", 0) + m["TCC_HIT_sum"] > 0:
        out.append(f"L2 hit rate {100 * m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):5.1f} %")
    if m.get("SQ_INSTS_LDS", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in m:
        out.append(f"LDS bank-conflict cycles per LDS instruction "
                   f"{m['SQ_LDS_BANK_CONFLICT'] / m['SQ_INSTS_LDS']:.2f}")
    if "FETCH_SIZE" in m and us > 0:
        out.append(f"HBM/MALL fetch {m['FETCH_SIZE'] / 1e3:8.2f} MB ({m['FETCH_SIZE'] / 1e3 / us:6.2f} TB/s "
                   "over the dispatch)")   # FETCH_SIZE is in KB
    if "WRITE_SIZE" in m and us > 0:
        out.append(f"write {m['WRITE_SIZE'] / 1e3:8.2f} MB ({m['WRITE_SIZE'] / 1e3 / us:6.2f} TB/s)")
    if m.get("SQ_WAVE_CYCLES", 0) > 0 and "SQ_WAIT_ANY" in m:
        out.append(f"wave cycles waiting {100 * m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:5.1f} %")
    return out


if __name__ == "__main__":
    main()

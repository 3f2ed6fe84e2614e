#!/usr/bin/env python3
"""Condensed view of a kernel's gfx950 assembly: waits, barriers, memory ops, MFMA runs and
the register/LDS/spill metadata.  Usage: asm_summary.py file.s [symbol-substring] [--full]"""
import re
import sys

KEEP = ("s_waitcnt", "s_barrier", "buffer_load", "buffer_store", "global_load", "global_store",
        "s_cbranch", "ds_read", "ds_write", "v_mfma", ".LBB", "scratch_", "s_setprio")
RUN = ("v_mfma", "ds_read", "buffer_load", "global_load", "ds_write", "global_store")


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    s = open(path).read()
    syms = re.findall(r"^(\S+):\s*;\s*@", s, re.M)
    for n in syms:
        if pat not in n:
            continue
        i = s.index(n + ":")
        j = s.index(".Lfunc_end", i)
        out, prev, cnt, prevline = [], None, 0, ""
        for line in s[i:j].split("\n"):
            t = line.strip().split(";")[0].strip()
            if not t.startswith(KEEP):
                continue
            key = t.split()[0]
            if key == prev and key.startswith(RUN):
                cnt += 1
                continue
            if prev:
                out.append(f"{prevline}  x{cnt}" if cnt > 1 else prevline)
            prev, cnt, prevline = key, 1, t[:70]
        if prev:
            out.append(f"{prevline}  x{cnt}" if cnt > 1 else prevline)
        meta = s[s.index(".name:           " + n) - 200:] if (".name:           " + n) in s else ""
        md = {}
        for k in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "vgpr_spill_count",
                  "private_segment_fixed_size", "agpr_count"):
            m = re.search(r"\." + k + r":\s+(\d+)", s[s.index(n + ":"):])
            md[k] = m.group(1) if m else "?"
        print("=" * 100)
        print(n)
        print(md)
        if "--full" in sys.argv or len(out) < 400:
            print("\n".join(out))


if __name__ == "__main__":
    main()

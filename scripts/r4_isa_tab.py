"""Per-K-tile instruction tabulation of a GEMM kernel's main loop.

Input: a hipcc device assembly file (``--cuda-device-only -S``) or an ``llvm-objdump -d`` listing
of a code object (e.g. a hipBLASLt .co), and a kernel symbol (substring).  The main loop is the
backward branch whose body holds the most MFMA instructions; its instruction mix is counted by
class and normalised per 100 MFMA-equivalents (one v_mfma_*_16x16x32_bf16 = 16384 FLOP): the
instruction stream is per wave, and kernels split a block's K tile over different wave counts,
so "instructions per unit of matrix work" is the comparable figure.

  python scripts/r4_isa_tab.py FILE SYMBOL [--k-flops-per-iter N]
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

MFMA_FLOPS = {  # per instruction (M*N*K*2) of the bf16 shapes
    "16x16x32": 16 * 16 * 32 * 2, "32x32x16": 32 * 32 * 16 * 2,
    "16x16x16": 16 * 16 * 16 * 2, "32x32x8": 32 * 32 * 8 * 2,
}
UNIT_FLOPS = 100 * 16 * 16 * 32 * 2   # 100 v_mfma_f32_16x16x32_bf16


def classify(op: str, args: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accvgpr_move"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return op
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_write"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith("buffer_load") or op.startswith("global_load"):
        return op + ("(lds)" if " lds" in (" " + args) else "")
    if op.startswith("buffer_") or op.startswith("global_"):
        return op
    if op == "s_waitcnt":
        return "s_waitcnt " + ("vmcnt" if "vmcnt" in args else "") + (
            "+" if "vmcnt" in args and "lgkmcnt" in args else "") + ("lgkmcnt" if "lgkmcnt" in args else "")
    if op in ("s_barrier", "s_setprio", "s_nop", "s_sleep") or op.startswith("s_cbranch") or op == "s_branch":
        return op if not op.startswith("s_cbranch") else "s_cbranch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other:" + op


def parse(path: str, sym: str):
    """(instructions [(addr_or_idx, op, args)], label -> index) of the first function whose
    name contains sym."""
    lines = open(path).read().splitlines()
    insts, labels = [], {}
    inside = False
    objdump = any(re.match(r"^[0-9a-f]{16} <", ln) for ln in lines[:2000])
    for ln in lines:
        if objdump:
            # a listing of exactly the kernel's address range (llvm-objdump --start/--stop-
            # address): Tensile kernels carry local label_* symbols, which are branch targets
            m = re.match(r"^[0-9a-f]{16} <(.+)>:", ln)
            if m:
                inside = True
                labels[m.group(1)] = len(insts)
                continue
            if not inside:
                continue
            m = re.match(r"^\s+(\w+)\s*(.*?)\s*//\s*([0-9A-F]+):", ln)
            if m:
                insts.append((int(m.group(3), 16), m.group(1), m.group(2)))
        else:
            if re.match(r"^[A-Za-z_.$][\w.$]*:", ln) and not ln.startswith(".L"):
                name = ln.split(":")[0]
                if inside and not name.startswith(".") and name != sym:
                    break
                if sym in name:
                    inside = True
                continue
            if not inside:
                continue
            m = re.match(r"^(\.LBB\w+):", ln)
            if m:
                labels[m.group(1)] = len(insts)
                continue
            s = ln.strip()
            if not s or s.startswith(";") or s.startswith("."):
                if s.startswith(".Lfunc_end"):
                    break
                continue
            s = s.split(";")[0].strip()
            parts = s.split(None, 1)
            insts.append((len(insts), parts[0], parts[1] if len(parts) > 1 else ""))
    return insts, labels, objdump


def loops(insts, labels, objdump):
    """(start, end) index ranges of backward branches."""
    out = []
    if objdump:
        idx = {a: i for i, (a, _, _) in enumerate(insts)}
        for i, (a, op, args) in enumerate(insts):
            if op.startswith("s_cbranch") or op == "s_branch":
                lab = args.split()[0] if args else ""
                if lab in labels:
                    if labels[lab] <= i:
                        out.append((labels[lab], i))
                    continue
                try:
                    simm = int(args.split(",")[0].split()[0], 0)
                except ValueError:
                    continue
                if simm >= 32768:
                    simm -= 65536
                tgt = a + 4 + 4 * simm
                if tgt < a and tgt in idx:
                    out.append((idx[tgt], i))
    else:
        for i, (_, op, args) in enumerate(insts):
            if op.startswith("s_cbranch") or op == "s_branch":
                lab = args.split()[0] if args else ""
                if lab in labels and labels[lab] <= i:
                    out.append((labels[lab], i))
    return out


def tabulate(path, sym):
    insts, labels, objdump = parse(path, sym)
    if not insts:
        raise SystemExit(f"symbol {sym!r} not found in {path}")
    best = None
    for (a, b) in loops(insts, labels, objdump):
        n = sum(1 for _, op, _ in insts[a:b + 1] if op.startswith("v_mfma"))
        if best is None or n > best[2]:
            best = (a, b, n)
    if best is None:
        raise SystemExit("no loop found")
    a, b, _ = best
    body = insts[a:b + 1]
    counts = collections.Counter(classify(op, args) for _, op, args in body)
    flops = 0
    shapes = collections.Counter()
    for _, op, _ in body:
        if op.startswith("v_mfma"):
            m = re.search(r"(\d+x\d+x\d+)", op)
            shapes[op] += 1
            flops += MFMA_FLOPS.get(m.group(1), 0) if m else 0
    per = flops / UNIT_FLOPS if flops else 1.0
    return {"kernel": sym, "file": path.split("/")[-1], "loop_instructions": len(body),
            "mfma_shapes": dict(shapes), "raw": dict(sorted(counts.items())),
            "per_100_mfma_16x16x32": {k: round(v / per, 1) for k, v in sorted(counts.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("symbol")
    a = ap.parse_args()
    print(json.dumps(tabulate(a.file, a.symbol)))


if __name__ == "__main__":
    sys.exit(main())

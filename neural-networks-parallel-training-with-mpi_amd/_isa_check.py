"""Static check of the built gfx950 code objects for matrix-core results read too early.

An MFMA writes its accumulator registers several passes after it issues; a VALU, LDS, global or
buffer instruction that reads those registers must sit enough wait states (instructions or
``s_nop`` cycles) behind it, and the compiler inserts the ``s_nop``s.  ROCm 7.2's hipcc missed
them once in this tree (head.hip, ``head_logits_stream_kernel<_, 1>``: a ``ds_write_b128`` of the
accumulators two instructions after the loop's last ``v_mfma_f32_16x16x4_f32``, which stored a
stale partial sum).  This module disassembles the library (``llvm-objdump --offloading`` into a
scratch directory, then ``-d --mcpu=gfx950``) and walks every kernel in straight-line order,
following fall-through only, and reports every read of an MFMA destination register fewer than
``min_ws`` wait states after the MFMA.  The threshold is deliberately below the hardware's
requirement (which depends on the pass count and on the consumer): it catches a missing guard,
not a guard that is one short.  ``tests/test_units.py::test_no_mfma_result_read_without_wait_states``
runs it on the built library.
"""
import glob
import os
import re
import shutil
import subprocess
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
OBJDUMP = os.path.join(ROCM, "lib", "llvm", "bin", "llvm-objdump")

_FN = re.compile(r"^[0-9a-f]+ <([^>]+)>:")
_RANGE = re.compile(r"^([av])\[(\d+):(\d+)\]$")
_ONE = re.compile(r"^([av])(\d+)$")
_END_FLOW = ("s_branch", "s_endpgm", "s_setpc_b64", "s_cbranch_execz_never")
_READERS = ("v_", "ds_", "global_", "buffer_", "flat_", "scratch_")


def _regs(tok):
    tok = tok.strip()
    m = _RANGE.match(tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = _ONE.match(tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def scan_disassembly(text: str, min_ws: int = 4):
    """Return (kernel, instruction, wait states) for every MFMA destination read too early."""
    hits = []
    fn = None
    last = {}
    ws = 0
    for line in text.splitlines():
        m = _FN.match(line)
        if m:
            fn, last, ws = m.group(1), {}, 0
            continue
        s = line.split("//")[0].strip()
        if not s or fn is None or s.endswith(":"):
            continue
        op, _, rest = s.partition(" ")
        ops = [t for t in rest.split(",")] if rest else []
        if op == "s_nop":
            ws += int(rest.strip(), 0) + 1
            continue
        if op.startswith("v_mfma"):
            # sources are read at issue; the destination becomes pending
            for r in _regs(ops[0]) if ops else ():
                last[r] = ws
            ws += 1
            continue
        if op.startswith(_READERS):
            stores = op.startswith(("ds_write", "global_store", "buffer_store", "flat_store",
                                    "scratch_store"))
            srcs = ops if stores else ops[1:]
            read = set()
            for t in srcs:
                read |= _regs(t)
            d = [ws - last[r] for r in read if r in last]
            if d and min(d) < min_ws:
                hits.append((fn, s, min(d)))
            # a VALU that overwrites a pending register ends the hazard on it
            if not stores and ops:
                for r in _regs(ops[0]):
                    last.pop(r, None)
        ws += 1
        if op in _END_FLOW:
            last, ws = {}, 0
    return hits


def scan_library(path: str, min_ws: int = 4):
    """Disassemble every gfx950 code object bundled in ``path`` and scan it."""
    if not os.path.exists(OBJDUMP):
        raise FileNotFoundError(OBJDUMP)
    tmp = tempfile.mkdtemp(prefix="nnmpi_isa_")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copyfile(path, lib)
        subprocess.run([OBJDUMP, "--offloading", lib], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        hits = []
        objs = sorted(glob.glob(os.path.join(tmp, "lib.so.*gfx950")))
        if not objs:
            raise RuntimeError(f"no gfx950 code object in {path}")
        for obj in objs:
            r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True,
                               capture_output=True, text=True)
            hits += scan_disassembly(r.stdout, min_ws)
        return hits
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    import sys
    from nnmpi_amd import _build
    for h in scan_library(sys.argv[1] if len(sys.argv) > 1 else _build.ext_path()):
        print(h)

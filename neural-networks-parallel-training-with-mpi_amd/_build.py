"""Build the native extension ``_nnmpi_hip`` in-tree with hipcc for gfx950.

Every ``csrc/**/*.hip`` / ``*.cpp`` is compiled to an object with
``hipcc --offload-arch=gfx950 -O3 -fPIC`` (in parallel, incremental on mtime), then linked
with the pybind11 bindings into ``_nnmpi_hip<EXT_SUFFIX>`` next to this file.  The library links
``libamdhip64``/``librccl`` by SONAME; at import time :mod:`nnmpi_amd.native` imports torch
first so both resolve to the copies torch already loaded (one HIP runtime per process).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(PKG_DIR, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("NNMPI_ARCH", "gfx950")
EXT_NAME = "_nnmpi_hip"


def ext_path() -> str:
    return os.path.join(PKG_DIR, EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))
    srcs += sorted(glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True))
    return srcs


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _common_flags():
    import pybind11
    return [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
        "-I", CSRC, "-I", os.path.join(ROCM, "include"),
        "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
        "-Wno-unused-result", "-Wno-unused-command-line-argument",
    ]


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def _compile(src: str, flags, force: bool) -> str:
    obj = _obj_for(src)
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + flags + ["-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    flags = _common_flags()
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, min(16, os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, force), srcs))
    out = ext_path()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(o) for o in objs):
        return out
    tmp = out + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + [
        "-L", os.path.join(ROCM, "lib"), "-lrccl", "-lamdhip64"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print(f"[nnmpi_amd] built {out}", file=sys.stderr)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)

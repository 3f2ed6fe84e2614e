"""Loader for the native extension ``_nnmpi_hip`` (HIP kernels + RCCL runtime).

torch is imported first so the extension's ``libamdhip64.so.7`` / ``librccl.so.1``
dependencies resolve (by SONAME) to the copies torch already mapped: one HIP runtime, one
device context, shared streams and pointers.  If the library is missing it is built in-tree
(hipcc, gfx950).  There is no silent fallback: on a GPU device every op goes through this
library and raises if it cannot be loaded.
"""
from __future__ import annotations

import importlib
import importlib.machinery
import importlib.util
import os
import sys

import torch  # noqa: F401  (must precede the extension import)

from . import _build

_lib = None


def _load():
    path = _build.ext_path()
    want = _build.source_hash()
    have = _build.built_hash(path) if os.path.exists(path) else ""
    if have != want:
        # a missing or STALE library (built from other csrc sources than these): rebuild it
        # (hipcc, in-tree) rather than run kernels that are not the ones in the tree; without
        # a toolchain this raises
        print(f"[nnmpi_amd] native library {'missing' if not have else 'stale'} "
              f"(built from {have or '-'}, sources are {want}): rebuilding", file=sys.stderr,
              flush=True)
        _build.build(verbose=True)
        have = _build.built_hash(path)
        if have != want:
            raise RuntimeError(f"rebuilt {path} but it carries source hash {have!r}, not {want!r}")
    name = __package__ + "._nnmpi_hip"
    if name in sys.modules:
        return sys.modules[name]
    loader = importlib.machinery.ExtensionFileLoader(name, path)
    spec = importlib.util.spec_from_file_location(name, path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules[name] = mod
    return mod


def lib():
    """The loaded extension module (raises if it cannot be built/loaded).  NNMPI_NATIVE=0
    refuses to load it (a host without the library: the CPU paths fall back to PyTorch)."""
    global _lib
    if _lib is None:
        if os.environ.get("NNMPI_NATIVE", "1") == "0":
            raise RuntimeError("native library disabled (NNMPI_NATIVE=0)")
        _lib = _load()
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:  # pragma: no cover - diagnostic helper
        return False


class stdout_to_stderr:
    """Redirect fd 1 to fd 2 for the duration (RCCL prints its version banner on stdout at
    communicator init, which would break one-JSON-line stdout contracts)."""

    def __enter__(self):
        import sys as _sys
        _sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import sys as _sys
        _sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def make_comm(uid: bytes, world: int, rank: int, device: int):
    """Create the native RCCL communicator (banner routed to stderr)."""
    with stdout_to_stderr():
        return lib().RcclComm(uid, world, rank, device)


def stream_handle(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return int(s.cuda_stream)


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())

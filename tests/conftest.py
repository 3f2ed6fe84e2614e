import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: longer multi-process runs")


def pytest_report_header(config):
    """The provenance of the native library under test: the hash of the csrc tree and the hash
    the built .so carries (they must match; nnmpi_amd.native rebuilds a stale library)."""
    try:
        import nnmpi_amd  # noqa: F401
        from nnmpi_amd import _build
        return (f"nnmpi_amd csrc source hash {_build.source_hash()}, built library "
                f"{_build.built_hash() or 'missing'} ({os.path.basename(_build.ext_path())})")
    except Exception as e:  # pragma: no cover
        return f"nnmpi_amd source hash unavailable: {e}"


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

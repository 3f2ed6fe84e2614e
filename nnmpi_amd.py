"""Import alias for the framework package.

The package source lives in ``neural-networks-parallel-training-with-mpi_amd/`` (a directory
name that is not a valid Python identifier).  Importing ``nnmpi_amd`` loads that directory as a
regular package and installs it under the name ``nnmpi_amd`` so that ``import nnmpi_amd.models``
and relative imports inside the package work as usual.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "neural-networks-parallel-training-with-mpi_amd")

_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)

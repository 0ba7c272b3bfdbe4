"""Import alias: ``import svdj`` -> the ``svd-jacobi-mpi-cuda_amd`` package.

The package directory name (required layout) is not a valid identifier, so
this module loads it by path name and installs it under ``svdj``.  Use
attribute access (``svdj.ops.kernels``), not ``import svdj.ops``.
"""
import importlib
import os
import sys

_here = os.path.dirname(os.path.abspath(__file__))
if _here not in sys.path:
    sys.path.insert(0, _here)
_pkg = importlib.import_module("svd-jacobi-mpi-cuda_amd")
sys.modules[__name__] = _pkg

#!/usr/bin/env python3
"""Reference-style driver: ``svd_jacobi.py N`` (see svd-jacobi-mpi-cuda_amd/cli.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdj  # noqa: E402

if __name__ == "__main__":
    sys.exit(svdj.cli.main())

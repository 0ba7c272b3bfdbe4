"""Solver families ("models"): CPU oracle, scalar pair path, MFMA block path.

The distributed block solver lives in ``parallel.distributed``.
"""
from .base import SVDResult, Solver  # noqa: F401
from .block import BlockJacobi  # noqa: F401
from .oracle import OracleJacobi  # noqa: F401
from .scalar import ScalarJacobi  # noqa: F401

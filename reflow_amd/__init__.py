"""reflow_amd -- MI355X (gfx950) engine for Reflow's memoization hot path.

The product is libreflow_hip.so (C-ABI in include/reflow_hip.h); this package
holds its Python binding (capi) used by the tests and bench.py.
"""
from . import capi  # noqa: F401

__all__ = ["capi"]

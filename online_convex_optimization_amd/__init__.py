"""MI355X-native engine for the FTRL/FTL online-convex-optimization hot path.

Drop-in modules (same names/signatures as the reference's):
  fast_algorithms, algorithms, exact_ftl, sequence_generation
Batched / device-resident API: engine
C ABI: include/ocx.h (libocx.so, built by _build.py)
"""
__version__ = "0.4.0"

from . import _lib  # noqa: F401

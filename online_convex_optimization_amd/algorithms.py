"""Import surface of the reference's ``algorithms.py`` (driver.py:22-27,
exact_ftl_driver.py:23) — **the float32 twin itself is not provided (parity unpinned).**

The reference's ``algorithms.py`` is a slower float32 NumPy twin of
``fast_algorithms.py``.  It is not built: its ``z @ x`` and
norm calls go through the host's BLAS kernel (platform-dependent order), reference
execution was denied, and the reference ships no fixture for it.
Its names are bound here to the float64 GPU engine so that ``driver.py``-style code and
``exact_ftl_driver.py``'s ``from algorithms import _rng`` run unchanged; results follow
the float64 reference path (``fast_algorithms.py``), not the float32 twin (they differ by
about 1e-6 relative, and return Python floats rather than ``np.float32``).
"""
from .fast_algorithms import (  # noqa: F401
    _rng,
    empirical_worst_case_thresholds,
    simulate_alg,
    simulate_empirical_g_SMART,
    simulate_SMART,
    simulate_SMART_like,
)

"""Drop-in for the reference's ``algorithms.py`` import surface (driver.py:22-27).

The reference's ``algorithms.py`` is a slower float32 NumPy twin of
``fast_algorithms.py`` (out of scope).  Its names are bound here to
the float64 GPU engine, so ``driver.py``-style code runs unchanged; results follow
the float64 reference path (they differ from the float32 twin by ~1e-6 relative).
"""
from .fast_algorithms import (  # noqa: F401
    _rng,
    empirical_worst_case_thresholds,
    simulate_alg,
    simulate_empirical_g_SMART,
    simulate_SMART,
    simulate_SMART_like,
)

"""Drop-in for the reference's ``algorithms.py`` — the float32 NumPy twin that
``driver.py:22-27`` imports — computed on the GPU (``csrc/ocx_twin32.hip``).

The twin keeps its parameters in float32 and its loss accumulators in Python floats, so
its results differ from ``fast_algorithms.py`` (float64) by about 1e-6 relative and come
back as ``np.float32`` (NumPy 2, NEP 50).  The kernels reproduce the float32 arithmetic of
the twin's NumPy calls on this image's NumPy / OpenBLAS: sdot's
double-accumulated float products, sgemv's row order, NumPy's pairwise sums, the float32
row clip of the g(T) sampler.  Parity: bit-identical to fixtures made by running those
NumPy calls (``tests/golden/make_twin32.py``; the reference module itself could not be
executed), for d = 5, the dimension every reference caller uses; other d
(<= 32) follow the same rules, which the host BLAS may order differently.

Inputs are taken as float32 (the reference's callers pass float32 streams).  Every call
runs on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

from . import engine
from .fast_algorithms import _rng  # noqa: F401  (algorithms.py:177-180; exact_ftl_driver.py:23)

__all__ = ["simulate_alg", "simulate_SMART_like", "simulate_SMART", "simulate_empirical_g_SMART",
           "empirical_worst_case_thresholds", "_rng"]

DEVICE = 0


def _one(z, y):
    z = np.asarray(z)
    y = np.asarray(y)
    if z.ndim != 2:
        raise ValueError(f"z must be [T, d], got shape {z.shape}")
    if y.shape != (z.shape[0],):
        raise ValueError(f"y must be [T] = {(z.shape[0],)}, got {y.shape}")
    return z[None], y[None]


def simulate_alg(z: np.ndarray, y: np.ndarray, alg_flag: int, eta0: float) -> np.float32:
    """algorithms.py:28-54: FTRL (alg_flag 0) or FTL (1) regret against FTL's final action."""
    zb, yb = _one(z, y)
    return engine.twin32_batch(zb, yb, 0 if int(alg_flag) == 0 else 1, eta0, device=DEVICE)[0]


def simulate_SMART_like(z: np.ndarray, y: np.ndarray, theta_thresh: float,
                        eta0: float) -> np.float32:
    """algorithms.py:65-120: FTL until its regret against the best constant action reaches
    ``theta_thresh``, then FTRL; regret against FTL's final action."""
    zb, yb = _one(z, y)
    return engine.twin32_batch(zb, yb, 2, eta0, thresh=float(theta_thresh), device=DEVICE)[0]


def simulate_SMART(z: np.ndarray, y: np.ndarray, *, eta0: float = math.sqrt(2)) -> np.float32:
    """algorithms.py:123-125 (threshold sqrt(2T))."""
    T = np.asarray(z).shape[0]
    return simulate_SMART_like(z, y, theta_thresh=math.sqrt(2 * T), eta0=eta0)


def simulate_empirical_g_SMART(z: np.ndarray, y: np.ndarray, theta_emp: float, *,
                               eta0: float = math.sqrt(2)) -> np.float32:
    """algorithms.py:127-128."""
    return simulate_SMART_like(z, y, theta_thresh=theta_emp, eta0=eta0)


def empirical_worst_case_thresholds(T_grid: np.ndarray, *, runs: int = 5,
                                    base_seed: int = 0) -> Dict[int, float]:
    """algorithms.py:135-171: for every T the largest FTRL regret over ``runs`` float32
    g(T) sequences (d = 5, rows clipped in float32), all runs of a T generated and simulated
    on the GPU in one call (``ocx_twin32_gT_regrets``)."""
    g_emp: Dict[int, float] = {}
    for T_val in T_grid:
        T = int(T_val)
        regs = engine.twin32_gT_regrets(T, int(runs), base_seed=int(base_seed), d=5,
                                        eta0=math.sqrt(2), device=DEVICE)
        max_regret = 0.0
        for reg in regs:  # the reference's `reg > max_regret` scan (np.float32 values)
            if reg > max_regret:
                max_regret = reg
        g_emp[T] = max_regret
    return g_emp

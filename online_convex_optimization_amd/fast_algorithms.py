"""Drop-in for the reference's ``fast_algorithms.py`` — same names, same signatures,
same results, computed by the HIP kernels in ``csrc/`` on an MI355X.

    from online_convex_optimization_amd.fast_algorithms import (
        empirical_worst_case_thresholds, simulate_alg, simulate_SMART,
        simulate_empirical_g_SMART)

is a one-line swap for ``fast_driver.py:23-28``.  Scalar calls run one sequence in
"exact" mode (``lanes_per_seq=1``: the reference's sequential sums, bit-identical
results); ``empirical_worst_case_thresholds`` regenerates its random sequences on
the GPU instead of drawing them with NumPy on the host and returns the reference's
values.  For throughput use the batched API in ``engine.py``.

Differences from the reference (documented, deliberate):
  * shape errors raise ``ValueError`` (numba would read out of bounds);
  * ``empirical_worst_case_thresholds`` accepts ``d`` (default 5 = the reference's
    hard-coded value, fast_algorithms.py:234), ``devices`` and ``progress``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np

from . import engine
from ._lib import ptr
from . import _lib

SQRT2 = math.sqrt(2)
EXACT = 1  # lanes_per_seq for scalar calls: sequential sums, bit-identical to the reference
_DEVICE = 0


def set_default_device(device: int) -> None:
    global _DEVICE
    _DEVICE = int(device)


def _as_2d(z, y):
    z_arr = np.ascontiguousarray(z, dtype=np.float64)
    y_arr = np.ascontiguousarray(y, dtype=np.float64)
    if z_arr.ndim != 2:
        raise ValueError(f"z must be [T, d], got shape {z_arr.shape}")
    if y_arr.shape != (z_arr.shape[0],):
        raise ValueError(f"y must be [T] = ({z_arr.shape[0]},), got {y_arr.shape}")
    return z_arr, y_arr


# ==============================================================
# Online simulation (FTL, FTRL), regret vs comparator
# ==============================================================

def simulate_alg(z: np.ndarray, y: np.ndarray, alg_flag: int, eta0: float) -> float:
    """fast_algorithms.py:171-177 → :88-115.  alg_flag 0 = FTRL, anything else = FTL."""
    z_arr, y_arr = _as_2d(z, y)
    T, d = z_arr.shape
    out = np.zeros(1)
    _lib.call("ocx_simulate_alg_batch", ptr(z_arr), ptr(y_arr), 1, T, d, int(alg_flag),
              float(eta0), None, ptr(out), None, None, None, EXACT, _DEVICE)
    return float(out[0])


# ==============================================================
# SMART (single switch)
# ==============================================================

def simulate_SMART_like(z: np.ndarray, y: np.ndarray, theta_thresh: float, eta0: float) -> float:
    """fast_algorithms.py:184-195 → :118-164.  Start with FTL; switch once to FTRL when
    FTL's regret against the best constant action so far reaches ``theta_thresh``."""
    z_arr, y_arr = _as_2d(z, y)
    T, d = z_arr.shape
    th = np.array([float(theta_thresh)])
    out = np.zeros(1)
    _lib.call("ocx_simulate_smart_batch", ptr(z_arr), ptr(y_arr), 1, T, d, ptr(th), float(eta0),
              ptr(out), None, EXACT, _DEVICE)
    return float(out[0])


def simulate_SMART(z: np.ndarray, y: np.ndarray, *, eta0: float = SQRT2) -> float:
    """fast_algorithms.py:198-200 (threshold sqrt(2T))."""
    T = z.shape[0]
    return simulate_SMART_like(z, y, theta_thresh=math.sqrt(2 * T), eta0=eta0)


def simulate_empirical_g_SMART(z: np.ndarray, y: np.ndarray, theta_emp: float, *,
                               eta0: float = SQRT2) -> float:
    """fast_algorithms.py:203-204."""
    return simulate_SMART_like(z, y, theta_thresh=theta_emp, eta0=eta0)


# ==============================================================
# Empirical g(T) for random sequences
# ==============================================================

def empirical_worst_case_thresholds(
    T_grid: np.ndarray,
    *,
    runs: int = 5,
    base_seed: int = 0,
    d: int = 5,
    devices: Optional[Sequence[int]] = None,
    progress: bool = False,
) -> Dict[int, float]:
    """fast_algorithms.py:211-247: for each T, the max FTRL regret (eta0 = sqrt 2) over
    ``runs`` sequences _rng(base_seed, T, r); the sequences are regenerated on the
    GPU (bit-compatible with NumPy's PCG64 / ziggurat streams) and never leave it."""
    g_emp: Dict[int, float] = {}
    it = T_grid
    if progress:
        from tqdm import tqdm
        it = tqdm(T_grid, desc="Estimating g(T) on random sequences")
    devs = list(devices) if devices else [_DEVICE]
    for T_val in it:
        T = int(T_val)
        res = engine.gT_sweep([T], int(runs), base_seed=int(base_seed), d=int(d), eta0=SQRT2,
                              devices=devs, lanes_per_seq=EXACT, return_regrets=False)
        g_emp[T] = res[T][0]
    return g_emp


# ==============================================================
# RNG helper (simple, reproducible)
# ==============================================================

def _rng(base_seed: int, T: int, run: int) -> np.random.Generator:
    """fast_algorithms.py:254-257 — host NumPy stream (the GPU generator reproduces it)."""
    ss = np.random.SeedSequence([base_seed, T, run])
    return np.random.Generator(np.random.PCG64(ss))

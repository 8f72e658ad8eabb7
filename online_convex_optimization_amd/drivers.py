"""Batched, device-resident versions of the reference's experiment sweeps
(fast_driver.py and exact_ftl_driver.py).

``evaluate_stream_with_stats`` (fast_driver.py:71-127) calls simulate_alg / SMART
once per (run, T, replicate) on host-built sequences.  Here every (run, replicate)
sequence of one T is generated on the GPU in a single batch (its ``sequence_generation``
family, bit-identical to the NumPy streams), the four algorithms run as four kernel
launches over that batch, and only the 4·runs·replicates regrets come back.  The
averaging then uses the same NumPy calls as the reference (fast_driver.py:113-125), so
the statistics are identical, not merely close.

``fast_driver_main`` is fast_driver.py:201-220 without the plotting: the g(T) sweep
(empirical_worst_case_thresholds) followed by the four cases.  ``driver_main`` is the
same for driver.py:204-226, which runs the float32 twin (algorithms.py).
"""
from __future__ import annotations

import math
from typing import Dict, Mapping, Optional, Sequence, Tuple

import numpy as np

from . import engine
from .fast_algorithms import empirical_worst_case_thresholds
from .sequence_generation import REPLICATES_BY_TITLE, RUNS_BY_TITLE

ALGO_KEYS = ("FTRL", "FTL", "SMART", "EMP")
CI_Z = 1.96
SQRT2 = math.sqrt(2)

# CASES title → (device family, stream-id base of the replicate streams, d)
CASE_FAMILIES = {
    "Random i.i.d. (separable)": ("iid", 13),
    "Massart noise 10%": ("massart", 23),
    "Label flips": ("flip", 0),
    "Switching leaders": ("switching", 0),
}

Stats = Dict[str, Tuple[np.ndarray, np.ndarray]]


def _sem(x: np.ndarray) -> float:
    """fast_driver.py:59-63."""
    n = x.size
    if n <= 1:
        return 0.0
    return float(np.std(x, ddof=1) / math.sqrt(n))


def case_regrets(title: str, T: int, g_emp_T: float, *, runs: int, replicates: int,
                 base_seed: int = 0, d: int = 5, p: float = 0.10, block_len: int = 20,
                 lanes_per_seq: int = 1, device: int = 0) -> Dict[str, np.ndarray]:
    """Regrets [runs, replicates] of FTRL, FTL, SMART(sqrt 2T), SMART(g_emp) for one case
    and one T — fast_driver.py:86-111 for every (run, rep) at once, on device."""
    family, stream0 = CASE_FAMILIES[title]
    B = runs * replicates
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes_per_seq, device=device)
    run_idx = np.repeat(np.arange(runs), replicates)
    rep_idx = np.tile(np.arange(replicates), runs)
    run_seeds = base_seed + 2025 * (run_idx + 1)  # fast_driver.py:88
    db.generate_family(family, run_seeds, stream0 + rep_idx, p=p, block_len=block_len)
    out = {}
    out["FTRL"] = db.simulate_alg(0, SQRT2).clone()
    out["FTL"] = db.simulate_alg(1, SQRT2).clone()
    out["SMART"] = db.simulate_smart(math.sqrt(2 * T), SQRT2).clone()
    out["EMP"] = db.simulate_smart(float(g_emp_T), SQRT2).clone()
    return {k: v[:B].cpu().numpy().reshape(runs, replicates) for k, v in out.items()}


def evaluate_stream_with_stats(title: str, T_grid: Sequence[int], g_emp: Mapping[int, float], *,
                               runs: int = 1, replicates: int = 1, base_seed: int = 0,
                               lanes_per_seq: int = 1, device: int = 0) -> Stats:
    """fast_driver.py:71-127 for the CASES entry ``title``: mean regret and 95 % CI per T."""
    by_T = {k: [[] for _ in range(len(T_grid))] for k in ALGO_KEYS}
    per_T = [case_regrets(title, int(T), g_emp[int(T)], runs=runs, replicates=replicates,
                          base_seed=base_seed, lanes_per_seq=lanes_per_seq, device=device)
             for T in T_grid]
    for run in range(runs):
        for ti in range(len(T_grid)):
            for k in ALGO_KEYS:
                by_T[k][ti].append(float(np.mean(list(per_T[ti][k][run]))))
    stats: Stats = {}
    for k in ALGO_KEYS:
        means, cis = [], []
        for vals in by_T[k]:
            arr = np.asarray(vals, dtype=float)
            mu = float(np.mean(arr)) if arr.size else 0.0
            ci = CI_Z * _sem(arr) if arr.size > 1 else 0.0
            means.append(mu)
            cis.append(ci)
        stats[k] = (np.array(means, dtype=float), np.array(cis, dtype=float))
    return stats


def fast_driver_main(T_grid: Optional[Sequence[int]] = None, *, g_runs: int = 1000,
                     base_seed: int = 0, runs_by_title: Optional[Mapping[str, int]] = None,
                     replicates_by_title: Optional[Mapping[str, int]] = None,
                     device: int = 0) -> Tuple[Dict[int, float], Dict[str, Stats]]:
    """fast_driver.py:201-220 minus the figures: (g_emp, stats_by_case)."""
    T_grid = list(range(100, 1100, 100)) if T_grid is None else [int(t) for t in T_grid]
    runs_by_title = RUNS_BY_TITLE if runs_by_title is None else runs_by_title
    replicates_by_title = REPLICATES_BY_TITLE if replicates_by_title is None else replicates_by_title
    g_emp = empirical_worst_case_thresholds(np.asarray(T_grid), runs=g_runs, base_seed=base_seed)
    stats = {}
    for title in CASE_FAMILIES:
        stats[title] = evaluate_stream_with_stats(
            title, T_grid, g_emp, runs=runs_by_title.get(title, 1),
            replicates=replicates_by_title.get(title, 1), base_seed=base_seed, device=device)
    return g_emp, stats


# ---------------------------------------------------------------------------
# driver.py: the same sweep on the float32 twin (algorithms.py)
# ---------------------------------------------------------------------------

def case_regrets_twin32(title: str, T: int, g_emp_T: float, *, runs: int, replicates: int,
                        base_seed: int = 0, d: int = 5, p: float = 0.10, block_len: int = 20,
                        device: int = 0) -> Dict[str, np.ndarray]:
    """driver.py:86-111 for every (run, rep) of one case and T at once: the four twin
    algorithms (algorithms.py) on the device-generated family, float32 regrets
    [runs, replicates]."""
    family, stream0 = CASE_FAMILIES[title]
    B = runs * replicates
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=-1, device=device)  # one lane per sequence
    run_idx = np.repeat(np.arange(runs), replicates)
    rep_idx = np.tile(np.arange(replicates), runs)
    db.generate_family(family, base_seed + 2025 * (run_idx + 1), stream0 + rep_idx, p=p,
                       block_len=block_len)
    out = {"FTRL": db.simulate_twin32(0, SQRT2), "FTL": db.simulate_twin32(1, SQRT2),
           "SMART": db.simulate_twin32(2, SQRT2, math.sqrt(2 * T)),
           "EMP": db.simulate_twin32(2, SQRT2, float(g_emp_T))}  # driver.py:95 float(g_emp[T])
    return {k: v[:B].cpu().numpy().reshape(runs, replicates) for k, v in out.items()}


def driver_evaluate_stream_with_stats(title: str, T_grid: Sequence[int],
                                      g_emp: Mapping[int, float], *, runs: int = 1,
                                      replicates: int = 1, base_seed: int = 0,
                                      device: int = 0) -> Stats:
    """driver.py:70-136 for the CASES entry ``title`` (float32 twin): mean regret and 95 % CI
    per T, the replicate means taken over the twin's np.float32 values as driver.py does."""
    by_T = {k: [[] for _ in range(len(T_grid))] for k in ALGO_KEYS}
    per_T = [case_regrets_twin32(title, int(T), g_emp[int(T)], runs=runs, replicates=replicates,
                                 base_seed=base_seed, device=device) for T in T_grid]
    for run in range(runs):
        for ti in range(len(T_grid)):
            for k in ALGO_KEYS:
                by_T[k][ti].append(float(np.mean(list(per_T[ti][k][run]))))
    stats: Stats = {}
    for k in ALGO_KEYS:
        means, cis = [], []
        for vals in by_T[k]:
            arr = np.asarray(vals, dtype=float)
            means.append(float(np.mean(arr)) if arr.size else 0.0)
            cis.append(CI_Z * _sem(arr) if arr.size > 1 else 0.0)
        stats[k] = (np.array(means, dtype=float), np.array(cis, dtype=float))
    return stats


def driver_main(T_grid: Optional[Sequence[int]] = None, *, g_runs: int = 1000,
                base_seed: int = 0, runs_by_title: Optional[Mapping[str, int]] = None,
                replicates_by_title: Optional[Mapping[str, int]] = None,
                device: int = 0):
    """driver.py:204-226 minus the figures (float32 twin): (g_emp, stats_by_case)."""
    from . import algorithms
    T_grid = list(range(100, 1100, 100)) if T_grid is None else [int(t) for t in T_grid]
    runs_by_title = RUNS_BY_TITLE if runs_by_title is None else runs_by_title
    replicates_by_title = REPLICATES_BY_TITLE if replicates_by_title is None else replicates_by_title
    g_emp = algorithms.empirical_worst_case_thresholds(np.asarray(T_grid), runs=g_runs,
                                                       base_seed=base_seed)
    stats = {}
    for title in CASE_FAMILIES:
        stats[title] = driver_evaluate_stream_with_stats(
            title, T_grid, g_emp, runs=runs_by_title.get(title, 1),
            replicates=replicates_by_title.get(title, 1), base_seed=base_seed, device=device)
    return g_emp, stats


# ---------------------------------------------------------------------------
# exact_ftl_driver.py: FTRL against the exact comparator, exact FTL replay
# ---------------------------------------------------------------------------
EXACT_ALGOS = ("FTRL", "FTL (exact)")


def exact_case_regrets(title: str, T: int, *, runs: int, replicates: int, base_seed: int = 0,
                       d: int = 5, p: float = 0.10, block_len: int = 20, lanes_per_seq: int = 1,
                       device: int = 0, norm: str = "l2") -> Dict[str, np.ndarray]:
    """exact_ftl_driver.py:157-186 for every (run, rep) of one case and T on device:
    exact FTL prefix actions over the ``norm`` ball (ExperimentConfig.norm, :46; closed
    form in its regime, else the general solver) replayed → "FTL (exact)" regret; FTRL
    (eta0 = sqrt 2) against actions[T] → "FTRL" regret."""
    import torch
    family, stream0 = CASE_FAMILIES[title]
    B = runs * replicates
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes_per_seq, device=device)
    run_idx = np.repeat(np.arange(runs), replicates)
    rep_idx = np.tile(np.arange(replicates), runs)
    db.generate_family(family, base_seed + 2025 * (run_idx + 1), stream0 + rep_idx, p=p,
                       block_len=block_len)
    return _exact_pair(db, B, d, torch, norm)


def _exact_pair(db, B, d, torch, norm: str = "l2") -> Dict[str, np.ndarray]:
    """Both regrets of exact_ftl_driver.py:169-184 in one read of the batch
    (ocx_dev_ftrl_vs_exact): FTRL and exact FTL against the exact comparator actions[T];
    sequences outside the closed form's regime take the general solver."""
    db.ftrl_vs_exact_general(SQRT2, norm=norm)
    ftrl = db.cum - db.comp
    ftl = db.cum_exact - db.comp
    return {"FTRL": ftrl[:B].cpu().numpy(), "FTL (exact)": ftl[:B].cpu().numpy()}


def exact_evaluate_stream_with_stats(title: str, T_grid: Sequence[int], *, runs: int,
                                     replicates: int, base_seed: int = 0, device: int = 0,
                                     norm: str = "l2") -> Stats:
    """exact_ftl_driver.py:120-206 for the CASES entry ``title``."""
    by_T = {k: [[] for _ in range(len(T_grid))] for k in EXACT_ALGOS}
    per_T = []
    for T in T_grid:
        r = exact_case_regrets(title, int(T), runs=runs, replicates=replicates,
                               base_seed=base_seed, device=device, norm=norm)
        per_T.append({k: v.reshape(runs, replicates) for k, v in r.items()})
    for run in range(runs):
        for ti in range(len(T_grid)):
            for k in EXACT_ALGOS:
                by_T[k][ti].append(float(np.mean(list(per_T[ti][k][run]))))
    stats: Stats = {}
    for k in EXACT_ALGOS:
        means, cis = [], []
        for vals in by_T[k]:
            arr = np.asarray(vals, dtype=float)
            means.append(float(np.mean(arr)) if arr.size else 0.0)
            cis.append(CI_Z * _sem(arr) if arr.size > 1 else 0.0)
        stats[k] = (np.array(means, dtype=float), np.array(cis, dtype=float))
    return stats


def exact_empirical_worst_case_thresholds(T_grid: Sequence[int], *, runs: int = 200,
                                          base_seed: int = 0, d: int = 5, device: int = 0,
                                          norm: str = "l2") -> Dict[int, float]:
    """exact_ftl_driver.py:64-117: max over runs of FTRL's regret against the exact
    comparator, on the g(T) adversary regenerated on device."""
    import torch
    g = {}
    for T in T_grid:
        T = int(T)
        db = engine.DeviceBatch(runs, T, d, lanes_per_seq=1, device=device)
        db.generate_gT(base_seed, 0)
        r = _exact_pair(db, runs, d, torch, norm)["FTRL"]
        g[T] = engine.max_regret(r)
    return g


def exact_ftl_driver_main(T_grid: Optional[Sequence[int]] = None, *, g_runs: int = 200,
                          base_seed: int = 0, device: int = 0, norm: str = "l2"):
    """exact_ftl_driver.py:268-293 minus the figures: (g_emp, stats_by_case); ``norm`` is
    ExperimentConfig.norm (:46)."""
    T_grid = list(range(100, 1100, 100)) if T_grid is None else [int(t) for t in T_grid]
    g = exact_empirical_worst_case_thresholds(T_grid, runs=g_runs, base_seed=base_seed,
                                              device=device, norm=norm)
    stats = {t: exact_evaluate_stream_with_stats(t, T_grid, runs=RUNS_BY_TITLE.get(t, 1),
                                                 replicates=REPLICATES_BY_TITLE.get(t, 1),
                                                 base_seed=base_seed, device=device, norm=norm)
             for t in CASE_FAMILIES}
    return g, stats

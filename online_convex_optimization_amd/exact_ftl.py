"""Drop-in for the FTRL / replay half of the reference's ``exact_ftl.py``.

Same names and signatures for ``RunResult``, ``run_ftrl``, ``replay_exact_ftl``,
``simulate`` and ``run_ftl_exact``; the FTRL loop (exact_ftl.py:230-277) and the
replay (:306-333) run in the HIP kernels.

The exact FTL solutions (the cvxpy SOCP of ``ExactFTLNoClip``, exact_ftl.py:62-193)
are computed on the GPU in closed form for the l2 ball whenever the data satisfy
||z_t|| <= 1 and y_t = ±1 — every sequence family and adversary of the reference does:
there ½Σ|z_i·x − y_i| is linear on the ball and its minimiser is S_t/||S_t||,
S_t = Σ_{i<t} y_i z_i (engine.ftl_exact_batch).  Outside that regime, and for the l1 /
linf balls, the general SOCP is out of scope: cvxpy is absent, so its results are
unpinned and those calls raise ``NotImplementedError`` unless the caller
supplies ``comparator_action`` / ``prefix_actions`` or a solver object with the
reference's methods.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Literal, Optional, Tuple

import numpy as np

from . import _lib
from . import engine as _engine
from . import fast_algorithms as _fa
from ._lib import ptr


@dataclass
class RunResult:
    """exact_ftl.py:217-222."""
    cum_loss: float
    regret: float
    comp_loss: float
    x_last: np.ndarray


def _ensure_float64_contiguous(arr) -> np.ndarray:
    """exact_ftl.py:52-55."""
    a = np.asarray(arr)
    if a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]:
        return a
    return np.ascontiguousarray(a, dtype=np.float64)


class ExactFTLNoClip:
    """exact_ftl.py:62-193 — the cvxpy SOCP/LP exact-FTL solver.  Not provided: cvxpy is
    absent and no reference oracle pins its outputs."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "ExactFTLNoClip (cvxpy SOCP comparator) is out of scope; pass comparator_action "
            "or prefix_actions instead")


def _simulate_ftrl(z_arr, y_arr, *, eta0, comparator_action=None, comparator_solver=None,
                   norm="l2", solver_name=None, solver_opts=None) -> RunResult:
    """exact_ftl.py:230-277 on the GPU."""
    T, d = z_arr.shape
    if comparator_action is None:
        if comparator_solver is not None:
            comparator_action = comparator_solver.solve_prefix_from_full(z_arr, y_arr, T)
        else:  # exact SOCP solution of the whole sequence, closed form on the GPU
            _, _, act, _ = _engine.ftl_exact_batch(z_arr[None], y_arr[None], norm=norm,
                                                   device=_fa._DEVICE)
            comparator_action = act[0]
    comp_vec = _ensure_float64_contiguous(comparator_action)
    if comp_vec.shape != (d,):
        raise ValueError(f"comparator_action must have shape ({d},)")
    out = np.zeros(3)
    x_last = np.zeros(d)
    _lib.call("ocx_simulate_alg_batch", ptr(z_arr), ptr(y_arr), 1, T, d, 0, float(eta0),
              ptr(comp_vec), ptr(out[0:1]), ptr(out[1:2]), ptr(out[2:3]), ptr(x_last), _fa.EXACT,
              _fa._DEVICE)
    return RunResult(cum_loss=float(out[1]), regret=float(out[0]), comp_loss=float(out[2]),
                     x_last=x_last)


def replay_exact_ftl(z: np.ndarray, y: np.ndarray, actions: np.ndarray) -> RunResult:
    """exact_ftl.py:306-333: losses of precomputed actions[t] (t < T), comparator
    actions[T]."""
    z_arr = _ensure_float64_contiguous(z)
    y_arr = _ensure_float64_contiguous(y)
    T, d = z_arr.shape
    acts = _ensure_float64_contiguous(actions)
    if acts.shape != (T + 1, d):
        raise ValueError("actions must have shape (T+1, d)")
    if y_arr.shape != (T,):
        raise ValueError("y must have shape (T,)")
    cum = np.zeros(1)
    comp = np.zeros(1)
    _lib.call("ocx_replay_batch", ptr(z_arr), ptr(y_arr), ptr(acts), 1, T, d, ptr(cum),
              ptr(comp), _fa._DEVICE)
    return RunResult(cum_loss=float(cum[0]), regret=float(cum[0] - comp[0]),
                     comp_loss=float(comp[0]), x_last=acts[T].copy())


def _prefix_actions_from_solver(ftl_solver, z_arr, y_arr) -> np.ndarray:
    """exact_ftl.py:280-303 compute_prefix_actions, driving a caller-supplied solver."""
    T, d = z_arr.shape
    actions = np.zeros((T + 1, d), dtype=np.float64)
    ftl_solver.reset_buffers()
    for i in range(T):
        actions[i + 1] = ftl_solver.append_row(z_arr[i], float(y_arr[i]))
    return actions


def _ftl_exact_gpu(z_arr, y_arr, norm) -> RunResult:
    """exact_ftl.py:423-453 with the prefix actions solved on the GPU (closed form)."""
    cum, comp, act, _ = _engine.ftl_exact_batch(z_arr[None], y_arr[None], norm=norm,
                                                device=_fa._DEVICE)
    return RunResult(cum_loss=float(cum[0]), regret=float(cum[0] - comp[0]),
                     comp_loss=float(comp[0]), x_last=act[0].copy())


def simulate(z, y, *, algo: Literal["ftrl", "ftl_exact"] = "ftl_exact", eta0: float = 1.0,
             norm: Literal["l2", "linf", "l1"] = "l2", solver: Optional[str] = None,
             solver_opts: Optional[dict] = None, ftl_solver=None, comparator_solver=None,
             prefix_actions: Optional[np.ndarray] = None,
             comparator_action: Optional[np.ndarray] = None) -> RunResult:
    """exact_ftl.py:336-392 unified front-end."""
    z_arr = _ensure_float64_contiguous(z)
    y_arr = _ensure_float64_contiguous(y)
    if algo == "ftl_exact":
        if prefix_actions is None and ftl_solver is None:
            return _ftl_exact_gpu(z_arr, y_arr, norm)
        if prefix_actions is None:
            prefix_actions = _prefix_actions_from_solver(ftl_solver, z_arr, y_arr)
        return replay_exact_ftl(z_arr, y_arr, prefix_actions)
    if algo == "ftrl":
        return _simulate_ftrl(z_arr, y_arr, eta0=eta0, comparator_action=comparator_action,
                              comparator_solver=comparator_solver, norm=norm,
                              solver_name=solver, solver_opts=solver_opts)
    raise ValueError("algo must be either 'ftrl' or 'ftl_exact'")


def run_ftrl(z, y, *, eta0: float = 1.0, norm: Literal["l2", "linf", "l1"] = "l2",
             solver: Optional[str] = None, solver_opts: Optional[dict] = None,
             comparator_solver=None, comparator_action: Optional[np.ndarray] = None) -> RunResult:
    """exact_ftl.py:399-420."""
    return simulate(z, y, algo="ftrl", eta0=eta0, norm=norm, solver=solver,
                    solver_opts=solver_opts, comparator_solver=comparator_solver,
                    comparator_action=comparator_action)


def run_ftl_exact(z, y, *, norm="l2", solver=None, solver_opts=None, ftl_solver=None,
                  prefix_actions: Optional[np.ndarray] = None, return_actions: bool = False
                  ) -> RunResult | Tuple[RunResult, np.ndarray]:
    """exact_ftl.py:423-453.  Without ``prefix_actions`` or ``ftl_solver`` the prefix
    actions are solved on the GPU (closed form, l2 ball) and replayed in the same kernel;
    the T+1 actions are not materialised, so ``return_actions=True`` needs one of the two."""
    z_arr = _ensure_float64_contiguous(z)
    y_arr = _ensure_float64_contiguous(y)
    actions = prefix_actions
    if actions is None and ftl_solver is None and not return_actions:
        return _ftl_exact_gpu(z_arr, y_arr, norm)
    if actions is None:
        if ftl_solver is None:
            raise NotImplementedError("return_actions=True needs prefix_actions or a solver "
                                      "object (the GPU path does not materialise T+1 actions)")
        actions = _prefix_actions_from_solver(ftl_solver, z_arr, y_arr)
    result = replay_exact_ftl(z_arr, y_arr, actions)
    if return_actions:
        return result, actions
    return result

"""Drop-in for the reference's ``exact_ftl.py`` (the module ``exact_ftl_driver.py:24-29``
imports): ``ExactFTLNoClip``, ``compute_prefix_actions``, ``replay_exact_ftl``,
``run_ftrl``, ``run_ftl_exact``, ``simulate`` and ``RunResult``, with the reference's
names, signatures and errors.  The FTRL loop (exact_ftl.py:230-277), the replay
(:306-333) and the exact FTL solutions all run in the HIP kernels.

Exact FTL (the cvxpy SOCP / LP of ``ExactFTLNoClip``, exact_ftl.py:62-193) is solved on
the GPU in closed form whenever every row's dual norm is <= 1 and y_t = ±1: then
|z_i·x| <= 1 on the ball, ½Σ|z_i·x − y_i| = ½(t − x·S_t), S_t = Σ_{i<t} y_i z_i, and the
minimiser maximises x·S_t over the ball (engine.ftl_prefix_actions_batch / ftl_exact_batch):

* l2 ball (regime ||z_t||_2 <= 1 — every sequence family and adversary of the reference):
  S_t/||S_t||;
* l1 ball (regime max_j |z_tj| <= 1 — implied by the l2 one, so again every family):
  sign(S_j*) e_j* with j* the first coordinate of largest |S_j|;
* linf ball (regime sum_j |z_tj| <= 1 — rows this small are rare in the reference's data):
  sign(S_t) componentwise.

* Degenerate prefixes: where the maximiser is not unique the closed forms would pick one
  vertex of the optimal face, while an interior-point solver (the ECOS / Clarabel backends
  cvxpy picks) approaches the face's analytic centre.  So tied prefixes leave the closed
  form (ocx_exact_poly_tie / the oracle's _poly_tie): for l1 two or more coordinates at the
  largest |S_j| > 0, for linf a zero coordinate of S_t that a row of the prefix touched.
  The general solver below answers those sequences (the analytic centre); for linf that
  sends the flip / switching families, whose rows touch one coordinate at a time, to the
  O(T^2) general path.  S_t = 0 (e.g. the empty prefix) keeps x = 0, which is that centre.
  Which point of the face cvxpy itself returns is solver-dependent: parity unpinned.
* Outside the regime (a row beyond the dual ball, a label other than ±1 — the linf ball on
  the reference's own rows) the GPU solves the SOCP / LP itself: a log-barrier path with a
  certified duality gap (engine.exact_ball_solve; d <= 256, larger d raises
  ``NotImplementedError``).  A caller can still pass ``comparator_action`` /
  ``prefix_actions`` or any solver object with the reference's methods
  (``reset_buffers`` / ``append_row`` / ``solve_prefix_from_full``).
* Parity against cvxpy is **unpinned**: cvxpy is absent here and the reference ships no
  fixture for it.  The closed forms are checked against the oracle's restatement and
  independently against scipy (SLSQP for l2, HiGHS LPs for l1 / linf) on the CPU
  (tests/test_exact_comparator_cpu.py); the general solver against the same scipy solvers
  on the GPU (tests/test_gpu_exact_general.py).
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


_NORMS = ("l2", "linf", "l1")


class ExactFTLNoClip:
    """exact_ftl.py:62-193: exact FTL over the unit norm ball, one reusable solver per
    (d, T_max) holding the current prefix in ``_Z_buf`` / ``_y_buf`` / ``_w_buf`` as the
    reference does.  Every solve runs on the GPU — in closed form where it is exact, by the
    general barrier solver elsewhere (module docstring); the ``solver`` / ``solver_opts``
    arguments are accepted and kept for signature parity (no cvxpy backend is involved).

    ``norm`` 'l2', 'l1' or 'linf'; anything else raises ValueError (exact_ftl.py:101-102)."""

    def __init__(self, d: int, T_max: int, *, norm: Literal["l2", "linf", "l1"] = "l2",
                 solver: Optional[str] = None, solver_opts: Optional[dict] = None) -> None:
        self.d = int(d)
        self.T_max = int(T_max)
        self.norm = norm
        self.solver = solver
        self.solver_opts = {} if solver_opts is None else dict(solver_opts)
        if norm not in _NORMS:
            raise ValueError("norm must be one of {'l2','linf','l1'}")
        self._Z_buf = np.zeros((self.T_max, self.d), dtype=np.float64)
        self._y_buf = np.zeros(self.T_max, dtype=np.float64)
        self._w_buf = np.zeros(self.T_max, dtype=np.float64)
        self._last_length = 0

    # -- solves ---------------------------------------------------------------
    def _solve_length(self, z_src: np.ndarray, y_src: np.ndarray, length: int) -> np.ndarray:
        """Exact FTL solution of the first ``length`` rows (GPU)."""
        _, _, act, _ = _engine.ftl_exact_batch(z_src[None, :length], y_src[None, :length],
                                               norm=self.norm, lanes_per_seq=_fa.EXACT,
                                               device=_fa._DEVICE)
        return act[0]

    def _solve_current(self) -> np.ndarray:
        """exact_ftl.py:120-128 for the cached prefix."""
        return self._solve_length(self._Z_buf, self._y_buf, self._last_length)

    def reset_buffers(self) -> None:
        """exact_ftl.py:130-139."""
        self._Z_buf.fill(0.0)
        self._y_buf.fill(0.0)
        self._w_buf.fill(0.0)
        self._last_length = 0

    def append_row(self, z_row: np.ndarray, y_val: float) -> np.ndarray:
        """exact_ftl.py:141-150: append one example to the cached prefix and solve."""
        if self._last_length >= self.T_max:
            raise ValueError("sequence longer than T_max")
        idx = self._last_length
        self._Z_buf[idx] = z_row
        self._y_buf[idx] = y_val
        self._w_buf[idx] = 1.0
        self._last_length += 1
        return self._solve_current()

    def _set_prefix(self, z_source: np.ndarray, y_source: np.ndarray, length: int) -> None:
        """exact_ftl.py:152-169."""
        t = int(length)
        if t < 0 or t > self.T_max:
            raise ValueError("length must be between 0 and T_max inclusive")
        if t > 0:
            np.copyto(self._Z_buf[:t], z_source[:t])
            np.copyto(self._y_buf[:t], y_source[:t])
            self._w_buf[:t] = 1.0
        if t < self._last_length:
            tail = slice(t, self._last_length)
            self._Z_buf[tail] = 0.0
            self._y_buf[tail] = 0.0
            self._w_buf[tail] = 0.0
        self._last_length = t

    def solve_prefix_from_full(self, z_full: np.ndarray, y_full: np.ndarray,
                               length: int) -> np.ndarray:
        """exact_ftl.py:171-181: solve over the first ``length`` rows of z_full/y_full."""
        z_src = _ensure_float64_contiguous(z_full)
        y_src = _ensure_float64_contiguous(y_full)
        self._set_prefix(z_src, y_src, length)
        return self._solve_current()

    def solve_prefix(self, z_prefix: np.ndarray, y_prefix: np.ndarray) -> np.ndarray:
        """exact_ftl.py:183-193."""
        z_src = _ensure_float64_contiguous(z_prefix)
        y_src = _ensure_float64_contiguous(y_prefix)
        t, d = z_src.shape
        if d != self.d:
            raise ValueError(f"Expected {self.d}-dimensional data, got {d}")
        if t > self.T_max:
            raise ValueError("prefix longer than T_max")
        self._set_prefix(z_src, y_src, t)
        return self._solve_current()


def compute_prefix_actions(solver, z: np.ndarray, y: np.ndarray) -> np.ndarray:
    """exact_ftl.py:280-303: exact FTL solutions for every prefix length 0..T → [T+1, d].

    With this module's ``ExactFTLNoClip`` all T+1 solutions come from one GPU launch
    (ocx_ftl_prefix_actions_batch) and the solver is left holding the whole sequence, as
    after the reference's append loop.  Any other solver object is driven row by row
    through its ``reset_buffers`` / ``append_row``, as the reference does."""
    z_arr = _ensure_float64_contiguous(z)
    y_arr = _ensure_float64_contiguous(y)
    T, d = z_arr.shape
    if solver.d != d:
        raise ValueError(f"Solver dimension {solver.d} incompatible with data dimension {d}")
    if solver.T_max < T:
        raise ValueError("Solver T_max is smaller than sequence length")
    if isinstance(solver, ExactFTLNoClip):
        actions, _ = _engine.ftl_prefix_actions_batch(z_arr[None], y_arr[None], norm=solver.norm,
                                                      lanes_per_seq=_fa.EXACT,
                                                      device=_fa._DEVICE)
        solver._set_prefix(z_arr, y_arr, T)
        return actions[0]
    actions = np.zeros((T + 1, d), dtype=np.float64)
    solver.reset_buffers()
    for idx in range(T):
        actions[idx + 1] = solver.append_row(z_arr[idx], float(y_arr[idx]))
    return actions


def _comparator_loss(z_arr, y_arr, x) -> float:
    """exact_ftl.py:224-227 on the GPU, in the reference's operation order (dgemv_t row sums,
    NumPy's pairwise sum; ocx_comparator_loss_blas_batch)."""
    T, d = z_arr.shape
    out = np.zeros(1)
    _lib.call("ocx_comparator_loss_blas_batch", ptr(z_arr), ptr(y_arr),
              ptr(_ensure_float64_contiguous(x)), 1, T, d, ptr(out), _fa._DEVICE)
    return float(out[0])


def _simulate_ftrl(z_arr, y_arr, *, eta0, comparator_action=None, comparator_solver=None,
                   norm="l2", solver_name=None, solver_opts=None) -> RunResult:
    """exact_ftl.py:230-277 on the GPU: the FTRL loop, then the comparator loss of the
    caller's action or of the solver's solution over the whole sequence."""
    T, d = z_arr.shape
    if comparator_action is None:
        solver = comparator_solver
        if solver is None:
            solver = ExactFTLNoClip(d=d, T_max=T, norm=norm, solver=solver_name,
                                    solver_opts=solver_opts)
        comparator_action = solver.solve_prefix_from_full(z_arr, y_arr, T)
    comp_vec = _ensure_float64_contiguous(comparator_action)
    if comp_vec.shape != (d,):
        raise ValueError(f"comparator_action must have shape ({d},)")
    out = np.zeros(3)
    x_last = np.zeros(d)
    _lib.call("ocx_simulate_alg_batch", ptr(z_arr), ptr(y_arr), 1, T, d, 0, float(eta0),
              ptr(comp_vec), ptr(out[0:1]), ptr(out[1:2]), ptr(out[2:3]), ptr(x_last), _fa.EXACT,
              _fa._DEVICE)
    cum = float(out[1])
    comp = _comparator_loss(z_arr, y_arr, comp_vec)
    return RunResult(cum_loss=cum, regret=float(cum - comp), comp_loss=comp, x_last=x_last)


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
    c = _comparator_loss(z_arr, y_arr, acts[T])
    return RunResult(cum_loss=float(cum[0]), regret=float(cum[0] - c), comp_loss=c,
                     x_last=acts[T].copy())


def _ftl_exact_gpu(z_arr, y_arr, norm) -> RunResult:
    """exact_ftl.py:423-453 without materialising the T+1 actions: prefix solutions and
    replay in one kernel (closed form; bit-identical to replaying
    compute_prefix_actions' output)."""
    if norm not in _NORMS:
        raise ValueError("norm must be one of {'l2','linf','l1'}")
    cum, comp, act, _ = _engine.ftl_exact_batch(z_arr[None], y_arr[None], norm=norm,
                                                lanes_per_seq=_fa.EXACT, device=_fa._DEVICE)
    c = _comparator_loss(z_arr, y_arr, act[0])
    return RunResult(cum_loss=float(cum[0]), regret=float(cum[0] - c), comp_loss=c,
                     x_last=act[0].copy())


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
            prefix_actions = compute_prefix_actions(ftl_solver, z_arr, y_arr)
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
    """exact_ftl.py:423-453."""
    z_arr = _ensure_float64_contiguous(z)
    y_arr = _ensure_float64_contiguous(y)
    if prefix_actions is None and ftl_solver is None and not return_actions:
        return _ftl_exact_gpu(z_arr, y_arr, norm)
    actions = prefix_actions
    if actions is None:
        T, d = z_arr.shape
        solver_obj = ftl_solver if ftl_solver is not None else ExactFTLNoClip(
            d=d, T_max=T, norm=norm, solver=solver, solver_opts=solver_opts)
        actions = compute_prefix_actions(solver_obj, z_arr, y_arr)
    result = replay_exact_ftl(z_arr, y_arr, actions)
    if return_actions:
        return result, actions
    return result

"""Batched API of the MI355X engine (new surface; the reference has only scalar calls).

Two ways in:

* host arrays (numpy) — ``simulate_alg_batch``, ``simulate_smart_batch``,
  ``replay_batch``, ``gT_regrets``: one synchronous call per batch, results back
  as numpy;
* device-resident batches — ``DeviceBatch``: z/y live in HBM in the engine's tiled
  layout (``include/ocx.h``), generated on device or packed once, then simulated
  any number of times without touching the host.  Device memory and streams come
  from PyTorch (plumbing only); every kernel is the HIP code in ``csrc/``.

Every batched call defaults to ``lanes_per_seq=LANES_BEST`` (include/ocx.h,
OCX_LANES_BEST), the fastest certified mode: the exact layout's sequential sums wherever its
lane chains are short and d < 64 (every d <= 16 batch, the drivers' d=5 batches), butterfly
sums (~1e-16 relative) where an exact chain of 8+ lanes would leave the kernel latency-bound
(d >= 512, few-wave batches such as the capacity-limited T=1e5 g(T) batch) and for batches
of >= 4096 sequences at 64 <= d <= 128 (the pipelined 8 x 8 kernel: the bench's 32 768 x 1e4
batch), and — for the g(T), DeviceBatch and FTRL-vs-exact
paths — the closed-form comparator losses wherever the kernel certifies them (one HBM pass
instead of two; about 1e-13 relative on the regret).  LANES_BEST results are therefore NOT
bit-identical to the reference.  ``lanes_per_seq=1`` forces the bit-exact mode (sequential
sums, streamed comparator pass); the drop-in modules (fast_algorithms, exact_ftl) always use
it.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import ptr

SQRT2 = math.sqrt(2.0)
LANES_BEST = 128  # OCX_LANES_BEST: exact where it streams at the roofline, butterfly elsewhere
LANES_EXACT = 1   # bit-identical to the reference's sequential sums


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def _check_zy(z: np.ndarray, y: np.ndarray):
    if z.ndim != 3:
        raise ValueError(f"z must be [B, T, d], got shape {z.shape}")
    B, T, d = z.shape
    if y.shape != (B, T):
        raise ValueError(f"y must be [B, T] = {(B, T)}, got {y.shape}")
    return B, T, d


def simulate_alg_batch(z, y, alg_flag: int = 0, eta0: float = SQRT2, comparator=None, *,
                       lanes_per_seq: int = LANES_BEST, device: int = 0, return_all: bool = False):
    """fast_algorithms.py:88-115 over B independent sequences on one GPU.

    z [B, T, d], y [B, T]; comparator [B, d] optional (exact_ftl.py:266-269).
    Returns regret [B] or, with ``return_all``, (regret, cum_loss, comp_loss, x_last)."""
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    cmp = None
    if comparator is not None:
        cmp = _f64(comparator)
        if cmp.shape != (B, d):
            raise ValueError(f"comparator must be [B, d] = {(B, d)}, got {cmp.shape}")
    reg = np.zeros(B)
    cum = np.zeros(B) if return_all else None
    comp = np.zeros(B) if return_all else None
    xl = np.zeros((B, d)) if return_all else None
    _lib.call("ocx_simulate_alg_batch", ptr(z), ptr(y), B, T, d, int(alg_flag), float(eta0),
              ptr(cmp), ptr(reg), ptr(cum), ptr(comp), ptr(xl), int(lanes_per_seq), int(device))
    if return_all:
        return reg, cum, comp, xl
    return reg


def simulate_smart_batch(z, y, thresh, eta0: float = SQRT2, *, lanes_per_seq: int = LANES_BEST,
                         device: int = 0, return_switch: bool = False):
    """fast_algorithms.py:118-164 over B sequences; thresh scalar or [B].  Bit-exact modes
    (lanes_per_seq 1 / -k) run the reference's O(T²·d) prefix re-scan; the others the
    O(T·d) kernel (guarded closed-form prefix: the same switch steps; closed-form final
    comparator where certified: the regret within its rounding)."""
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    th = _f64(np.broadcast_to(np.asarray(thresh, dtype=np.float64), (B,)))
    reg = np.zeros(B)
    sw = np.zeros(B, dtype=np.int64)
    _lib.call("ocx_simulate_smart_batch", ptr(z), ptr(y), B, T, d, ptr(th), float(eta0), ptr(reg),
              sw.ctypes.data_as(_lib.c_i64p), int(lanes_per_seq), int(device))
    return (reg, sw) if return_switch else reg


def replay_batch(z, y, actions, *, device: int = 0):
    """exact_ftl.py:306-333 over B sequences: actions [B, T+1, d] → (cum_loss, comp_loss)."""
    z = _f64(z)
    y = _f64(y)
    a = _f64(actions)
    B, T, d = _check_zy(z, y)
    if a.shape != (B, T + 1, d):
        raise ValueError(f"actions must be [B, T+1, d] = {(B, T + 1, d)}, got {a.shape}")
    cum = np.zeros(B)
    comp = np.zeros(B)
    _lib.call("ocx_replay_batch", ptr(z), ptr(y), ptr(a), B, T, d, ptr(cum), ptr(comp),
              int(device))
    return cum, comp


NORMS = {"l2": 0, "l1": 1, "linf": 2}  # the ball of exact FTL (exact_ftl.py:83-105)


def _norm_code(norm: str) -> int:
    if norm not in NORMS:
        raise ValueError("norm must be one of {'l2','linf','l1'}")
    return NORMS[norm]


def exact_ball_solve(z, y, *, norm: str = "l2", all_prefixes: bool = True, device: int = 0):
    """The general exact-FTL solver (include/ocx.h, ocx_exact_ball_solve): ExactFTLNoClip's
    problem min ½Σ_{i<n}|z_i·x − y_i| over the unit ``norm`` ball (exact_ftl.py:83-105) for
    any rows and labels, on the GPU by a log-barrier path.  Problems are every prefix
    n = 0..T of each sequence (``all_prefixes``) or n = T only.

    Returns a dict of arrays over [B, NP] (NP = T+1 or 1): ``actions`` [B, NP, d]
    (actions[:, n] the prefix-n minimiser, as compute_prefix_actions returns), ``obj``
    (½Σ|r| at it), ``gap`` (a certified bound on obj − optimum), ``step_loss`` (½|z_n·x_n −
    y_n|, 0 at n = T) and ``info`` (Newton steps, negative where the cap ended a solve)."""
    code = _norm_code(norm)
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    if d > _lib.OCX_EXACT_BALL_MAX_D:
        raise NotImplementedError(f"the general exact-FTL solver takes d <= "
                                  f"{_lib.OCX_EXACT_BALL_MAX_D} (got {d})")
    NP = T + 1 if all_prefixes else 1
    out = {"actions": np.zeros((B, NP, d)), "obj": np.zeros((B, NP)), "gap": np.zeros((B, NP)),
           "step_loss": np.zeros((B, NP)), "info": np.zeros((B, NP), dtype=np.int32)}
    _lib.call("ocx_exact_ball_solve", ptr(z), ptr(y), B, T, d, code, int(bool(all_prefixes)),
              ptr(out["actions"]), ptr(out["obj"]), ptr(out["gap"]), ptr(out["step_loss"]),
              out["info"].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(device))
    return out


# A general solve is accepted iff info >= 0 and gap <= EXACT_GAP_RTOL * (1 + |obj|).  The gap
# comes from the better of two duals: the barrier's multipliers (exact for the rows the optimum
# does not interpolate, only as good as μ_end = 1e-10 for the ones it does) and the dual the
# certificate polish rebuilds from the KKT system at the solver's x (ocx_exact_polish_kernel:
# ±½ on the first kind, least squares on stationarity for the second), which certifies the
# objective to the primal's own accuracy (~1e-10) where the optimum interpolates rows (n > d,
# real-valued rows: the barrier's certificate alone stayed near 1e-5 there).
EXACT_GAP_RTOL = 1e-8


def check_certificates(obj, gap, info, what: str = "exact FTL") -> float:
    """The general solver's answers are only as good as their certificates
    (include/ocx.h, ocx_exact_ball_solve): every solve must have finished (info >= 0: not
    ended by the step cap; 0 is the empty prefix, solved without a step) and certify obj − optimum <= gap <= EXACT_GAP_RTOL·(1 + |obj|).
    A breakdown stop (OCX_EXACT_INFO_BREAKDOWN) passes only on its certificate.  Raises
    RuntimeError otherwise — what exact_ftl.py:125-126 does when cvxpy's solve fails — and
    returns the worst gap."""
    obj = np.asarray(obj, dtype=np.float64)
    gap = np.asarray(gap, dtype=np.float64)
    info = np.asarray(info)
    if obj.size == 0:
        return 0.0
    bad = ~((info >= 0) & (gap <= EXACT_GAP_RTOL * (1.0 + np.abs(obj))))
    if bad.any():
        k = int(np.flatnonzero(bad.ravel())[0])
        raise RuntimeError(f"{what}: the general solver did not certify {int(bad.sum())} of "
                           f"{bad.size} problems (first: info {int(info.ravel()[k])}, gap "
                           f"{float(gap.ravel()[k]):.3g}, obj {float(obj.ravel()[k]):.6g})")
    return float(gap.max())


def _general_fill(z, y, ok: np.ndarray, norm: str, device: int):
    """Sequences outside the closed form's regime, solved by the general solver: (their
    indices, exact_ball_solve over all prefixes, exact FTL's cumulative loss Σ_n step_loss in
    step order, the comparator loss obj[:, T], the worst certified gap); None when every
    sequence is in the regime.  Raises RuntimeError where a solve is not certified."""
    bad = np.flatnonzero(~ok)
    if bad.size == 0:
        return None
    T = z.shape[1]
    res = exact_ball_solve(z[bad], y[bad], norm=norm, all_prefixes=True, device=device)
    worst = check_certificates(res["obj"], res["gap"], res["info"])
    sl = res["step_loss"][:, :T]
    cum = np.cumsum(sl, axis=1)[:, -1] if T > 0 else np.zeros(bad.size)  # sequential order
    return bad, res, cum, res["obj"][:, T], worst


def ftl_exact_batch(z, y, *, norm: str = "l2", lanes_per_seq: int = LANES_BEST, device: int = 0,
                    check_regime: bool = True):
    """exact_ftl.py:280-333 (compute_prefix_actions + replay) for B sequences on the GPU,
    over the unit ball of ``norm`` ('l2', 'l1', 'linf'), in the closed form that is the
    exact SOCP / LP solution when every row's dual norm is <= 1 and y_t = ±1
    (include/ocx.h, ocx_ftl_exact_batch).

    Returns (cum_loss [B], comp_loss [B], comparator actions[T] [B, d], in_regime [B]);
    with ``check_regime`` the sequences outside the regime are solved by the general solver
    (exact_ball_solve, d <= 256) — their numbers are the SOCP / LP's; without it they keep the
    closed form's (not the solution there: callers must reject them)."""
    code = _norm_code(norm)
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    cum = np.zeros(B)
    comp = np.zeros(B)
    act = np.zeros((B, d))
    rg = np.zeros(B, dtype=np.int32)
    _lib.call("ocx_ftl_exact_batch", ptr(z), ptr(y), B, T, d, code, ptr(cum), ptr(comp),
              ptr(act), rg.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(lanes_per_seq),
              int(device))
    ok = rg.astype(bool)
    if check_regime:
        g = _general_fill(z, y, ok, norm, device)
        if g is not None:
            bad, res, gcum, gcomp, _ = g
            cum[bad], comp[bad], act[bad] = gcum, gcomp, res["actions"][:, T]
    return cum, comp, act, ok


def ftl_prefix_actions_batch(z, y, *, norm: str = "l2", lanes_per_seq: int = LANES_BEST, device: int = 0,
                             check_regime: bool = True):
    """exact_ftl.py:280-303 compute_prefix_actions for B sequences on the GPU
    (include/ocx.h, ocx_ftl_prefix_actions_batch): actions [B, T+1, d] with actions[:, t]
    the exact FTL solution of the first t rows, in the closed form of ftl_exact_batch.

    Returns (actions, in_regime [B]); with ``check_regime`` the sequences outside the regime
    get the general solver's actions (exact_ball_solve)."""
    code = _norm_code(norm)
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    act = np.zeros((B, T + 1, d))
    rg = np.zeros(B, dtype=np.int32)
    _lib.call("ocx_ftl_prefix_actions_batch", ptr(z), ptr(y), B, T, d, code, ptr(act),
              rg.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(lanes_per_seq), int(device))
    ok = rg.astype(bool)
    if check_regime:
        g = _general_fill(z, y, ok, norm, device)
        if g is not None:
            act[g[0]] = g[1]["actions"]
    return act, ok


def ftrl_vs_exact_batch(z, y, eta0: float = SQRT2, *, norm: str = "l2",
                        lanes_per_seq: int = LANES_BEST, device: int = 0,
                        check_regime: bool = True, with_ftl_comparator: bool = False):
    """exact_ftl_driver.py:157-186 for B sequences in one read of the data: exact FTL
    (closed form, as ftl_exact_batch) and FTRL against its comparator actions[T].

    Returns a dict of [B] arrays: ``ftrl`` and ``exact`` regrets, ``cum_ftrl``,
    ``cum_exact``, ``comp`` (the loss of actions[T], shared by both), ``action``
    [B, d], ``in_regime``; with ``with_ftl_comparator`` also ``comp_ftl``, the loss of
    FTL(theta_ftrl) (the comparator simulate_alg itself uses).  With ``check_regime`` the
    exact side of sequences outside the closed form's regime comes from the general solver
    (exact_ball_solve), as in ftl_exact_batch."""
    z = _f64(z)
    y = _f64(y)
    B, T, d = _check_zy(z, y)
    cr, ce, cmp_e, cmp_f = (np.zeros(B) for _ in range(4))
    act = np.zeros((B, d))
    rg = np.zeros(B, dtype=np.int32)
    _lib.call("ocx_ftrl_vs_exact_batch_ex", ptr(z), ptr(y), B, T, d, float(eta0), ptr(cr), ptr(ce),
              ptr(cmp_e), ptr(cmp_f) if with_ftl_comparator else None, ptr(act),
              rg.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _norm_code(norm),
              int(lanes_per_seq), int(device))
    ok = rg.astype(bool)
    worst = 0.0
    if check_regime:
        g = _general_fill(z, y, ok, norm, device)
        if g is not None:
            bad, res, gcum, gcomp, worst = g
            ce[bad], cmp_e[bad], act[bad] = gcum, gcomp, res["actions"][:, T]
    out = {"ftrl": cr - cmp_e, "exact": ce - cmp_e, "cum_ftrl": cr, "cum_exact": ce,
           "comp": cmp_e, "action": act, "in_regime": ok, "exact_gap_max": worst}
    if with_ftl_comparator:
        out["comp_ftl"] = cmp_f
    return out


def gT_regrets(T: int, runs: int, *, base_seed: int = 0, d: int = 5, eta0: float = SQRT2,
               run0: int = 0, lanes_per_seq: int = LANES_BEST, device: int = 0) -> np.ndarray:
    """Regrets of FTRL on _rng(base_seed, T, run) sequences, run in [run0, run0+runs),
    generated on device (fast_algorithms.py:230-241 with a ``d`` parameter)."""
    if base_seed < 0 or base_seed >= 2 ** 64:
        raise ValueError("base_seed must be in [0, 2**64)")
    out = np.zeros(int(runs))
    _lib.call("ocx_gT_regrets", int(base_seed), int(T), int(run0), int(runs), int(d),
              float(eta0), ptr(out), int(lanes_per_seq), int(device))
    return out


def gT_regrets_device(T: int, runs: int, *, base_seed: int = 0, d: int = 5,
                      eta0: float = SQRT2, run0: int = 0, lanes_per_seq: int = LANES_BEST,
                      device: int = 0, out=None):
    """gT_regrets with the regrets left in HBM (``ocx_gT_regrets_dev``): a float64 torch
    tensor [runs] on cuda:``device`` (``out`` if given), complete when this returns.  What a
    rank hands to an RCCL all-gather (parallel.gT_sweep_distributed): no host round trip."""
    import torch
    if base_seed < 0 or base_seed >= 2 ** 64:
        raise ValueError("base_seed must be in [0, 2**64)")
    dev = torch.device("cuda", int(device))
    if out is None:
        out = torch.empty(int(runs), dtype=torch.float64, device=dev)
    if out.dtype != torch.float64 or out.device != dev or not out.is_contiguous() \
            or out.numel() != int(runs):
        raise ValueError(f"out must be a contiguous float64 tensor of {runs} on {dev}")
    # the library writes on its own stream: let the allocating stream's pending work on
    # this memory finish first
    torch.cuda.current_stream(dev).synchronize()
    _lib.call("ocx_gT_regrets_dev", int(base_seed), int(T), int(run0), int(runs), int(d),
              float(eta0), ctypes.c_void_p(out.data_ptr()), int(lanes_per_seq), int(device))
    return out


TWIN32_ALGOS = {"FTRL": 0, "FTL": 1, "SMART": 2}


def twin32_batch(z, y, algo: int = 0, eta0: float = SQRT2, thresh=None, *, device: int = 0,
                 return_all: bool = False):
    """The float32 twin (algorithms.py:28-54 simulate_alg, algo 0 FTRL / 1 FTL; :65-120
    simulate_SMART_like, algo 2 with thresh scalar or [B]) over B sequences, in NumPy 2's
    float32 arithmetic; d <= 32.

    z [B, T, d] and y [B, T] are taken as float32 (the twin's callers pass float32).
    Returns the twin's np.float32 results [B] or, with ``return_all``, (result, cum_loss
    float64, comp_loss float32, switch_step int64; -1 = no switch / not SMART)."""
    z = np.ascontiguousarray(z, dtype=np.float32)
    y = np.ascontiguousarray(y, dtype=np.float32)
    B, T, d = _check_zy(z, y)
    algo = int(algo)
    if algo not in (0, 1, 2):
        raise ValueError("algo must be 0 (FTRL), 1 (FTL) or 2 (SMART)")
    th = None
    if algo == 2:
        if thresh is None:
            raise ValueError("SMART needs thresh")
        th = _f64(np.broadcast_to(np.asarray(thresh, dtype=np.float64), (B,)))
    res = np.zeros(B, dtype=np.float32)
    cum = np.zeros(B) if return_all else None
    comp = np.zeros(B, dtype=np.float32) if return_all else None
    sw = np.full(B, -1, dtype=np.int64) if return_all else None
    fp = _lib.c_fp
    _lib.call("ocx_twin32_batch", z.ctypes.data_as(fp), y.ctypes.data_as(fp), B, T, d, algo,
              float(eta0), ptr(th), res.ctypes.data_as(fp), ptr(cum),
              comp.ctypes.data_as(fp) if comp is not None else None,
              sw.ctypes.data_as(_lib.c_i64p) if sw is not None else None, int(device))
    return (res, cum, comp, sw) if return_all else res


def twin32_gT_regrets(T: int, runs: int, *, base_seed: int = 0, d: int = 5,
                      eta0: float = SQRT2, run0: int = 0, device: int = 0) -> np.ndarray:
    """The float32 twin's g(T) regrets (algorithms.py:150-169) for runs [run0, run0+runs),
    generated and simulated on device: float32 [runs]."""
    if base_seed < 0 or base_seed >= 2 ** 64:
        raise ValueError("base_seed must be in [0, 2**64)")
    out = np.zeros(int(runs), dtype=np.float32)
    _lib.call("ocx_twin32_gT_regrets", int(base_seed), int(T), int(run0), int(runs), int(d),
              float(eta0), out.ctypes.data_as(_lib.c_fp), int(device))
    return out


def release_buffers(device: int = 0) -> None:
    """Free the HBM the engine caches on `device` for host-array calls and g(T) sweeps
    (it regrows on the next call): do this before allocating a large DeviceBatch."""
    _lib.release_buffers(device)


def max_regret(regrets: np.ndarray) -> float:
    """fast_algorithms.py:228, :242-243 — max over runs starting from 0.0 (`reg > max`)."""
    r = np.asarray(regrets, dtype=np.float64)
    pos = r[r > 0.0]
    return float(pos.max()) if pos.size else 0.0


def gT_max(T: int, runs: int, *, base_seed: int = 0, d: int = 5, eta0: float = SQRT2,
           run0: int = 0, lanes_per_seq: int = LANES_BEST, device: int = 0) -> float:
    """max(0, max of gT_regrets(...)) reduced on device (``ocx_gT_max``): the regrets never
    leave the GPU (fast_algorithms.py:228, :242-243)."""
    if base_seed < 0 or base_seed >= 2 ** 64:
        raise ValueError("base_seed must be in [0, 2**64)")
    out = np.zeros(1)
    _lib.call("ocx_gT_max", int(base_seed), int(T), int(run0), int(runs), int(d), float(eta0),
              int(lanes_per_seq), int(device), ptr(out))
    return float(out[0])


def gT_sweep(T_grid: Sequence[int], runs: int, *, base_seed: int = 0, d: int = 5,
             eta0: float = SQRT2, devices: Optional[Sequence[int]] = None,
             lanes_per_seq: int = LANES_BEST, return_regrets: bool = True) -> dict:
    """empirical_worst_case_thresholds on one or several GPUs of this process
    (``ocx_gT_sweep_devices``).

    For every T the runs are split into contiguous shards, one per device, each generated
    and simulated on its own GPU by a native host thread; the per-shard regrets land in
    run order.  Returns {T: (g(T), regrets[runs])}; with ``return_regrets=False`` each
    shard's max is reduced on its GPU and the regrets entry is None."""
    devs = [int(v) for v in devices] if devices else [0]
    grid = np.ascontiguousarray([int(T) for T in T_grid], dtype=np.int64)
    regs = np.zeros((len(grid), int(runs)), dtype=np.float64) if return_regrets else None
    gmax = np.zeros(len(grid), dtype=np.float64)
    dv = (ctypes.c_int * len(devs))(*devs)
    if base_seed < 0 or base_seed >= 2 ** 64:
        raise ValueError("base_seed must be in [0, 2**64)")
    _lib.call("ocx_gT_sweep_devices", grid.ctypes.data_as(_lib.c_i64p), len(grid), int(runs),
              int(base_seed), int(d), float(eta0), dv, len(devs), int(lanes_per_seq),
              ptr(gmax), ptr(regs))
    return {int(T): (float(gmax[i]), regs[i] if regs is not None else None)
            for i, T in enumerate(grid)}


# ---------------------------------------------------------------------------
# Device-resident batches (torch tensors as HBM buffers)
# ---------------------------------------------------------------------------

class DeviceBatch:
    """B sequences of T steps in d dimensions, resident in HBM in the tiled layout.

    ``stream`` is a torch.cuda.Stream (default: the current stream); every kernel
    of this object is launched on it, so torch events recorded on that stream
    bracket the HIP kernels exactly."""

    def __init__(self, B: int, T: int, d: int, *, lanes_per_seq: int = LANES_BEST, device: int = 0,
                 stream=None):
        import torch
        self.torch = torch
        self.L = _lib.layout(B, T, d, lanes_per_seq)
        # bit-exact modes keep the reference's two-pass comparator sum (see simulate_alg)
        self.exact = lanes_per_seq == LANES_EXACT or lanes_per_seq < 0
        self.best = lanes_per_seq == LANES_BEST
        self.rows_clipped = False  # set by generate_gT: every ||z_t|| <= 1
        self.device = torch.device("cuda", device)
        with torch.cuda.device(self.device):
            self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            self.z = torch.empty(max(self.L.z_elems, 1), dtype=torch.float64, device=self.device)
            self.y = torch.empty(max(self.L.y_elems, 1), dtype=torch.float64, device=self.device)
            self.regret = torch.zeros(max(B, 1), dtype=torch.float64, device=self.device)
            self.cum = torch.zeros_like(self.regret)
            self.comp = torch.zeros_like(self.regret)
        self.cum_exact = None  # allocated by ftrl_vs_exact

    @property
    def _sp(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def _on_stream(self):
        """Context that makes self.stream current on this device: helper tensors (seeds,
        thresholds, device-side dtype conversions) are then produced in the same stream
        order as the HIP kernels that read them."""
        return self.torch.cuda.stream(self.stream)

    def _hold(self, *tensors):
        """Keep helper tensors alive for the kernels queued on self.stream, and tell the
        caching allocator they are in use there (record_stream), so their memory is not
        handed out again before those kernels ran even if the next call replaces them."""
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(self.stream)
        return tensors

    def _lp(self):
        return ctypes.byref(self.L)

    def _call(self, name, *args):
        """_lib.call with this batch's device current: the null stream of a torch device is
        the current device's, and the library sizes its launches and forks its streams
        from the current device (a DeviceBatch on device 1 works without set_device)."""
        with self.torch.cuda.device(self.device):
            return _lib.call(name, *args)

    def generate_gT(self, base_seed: int = 0, run0: int = 0):
        """Fill z/y with _rng(base_seed, T, run0 + b) sequences (on device)."""
        self._call("ocx_dev_gen_gT", self._lp(), int(base_seed), int(run0), self.z.data_ptr(),
                  self.y.data_ptr(), self._sp)
        self.rows_clipped = True
        return self

    FAMILIES = {"iid": 1, "massart": 2, "flip": 3, "switching": 4}

    def generate_family(self, family, run_seeds=None, stream_ids=None, *, p: float = 0.10,
                        block_len: int = 20):
        """Fill z/y with a sequence_generation.py family (ocx_dev_gen_family): for the
        random families sequence b is _rng(run_seeds[b], T, stream_ids[b])."""
        torch = self.torch
        fam = self.FAMILIES[family] if isinstance(family, str) else int(family)
        rs = si = None
        if fam in (1, 2):
            with self._on_stream():
                rs = torch.as_tensor(np.asarray(run_seeds, dtype=np.uint64).astype(np.int64)
                                     ).to(self.device)
                si = torch.as_tensor(np.asarray(stream_ids, dtype=np.uint64).astype(np.int64)
                                     ).to(self.device)
            if rs.numel() != self.L.B or si.numel() != self.L.B:
                raise ValueError("need one run seed and one stream id per sequence")
        self.rows_clipped = False
        self._call("ocx_dev_gen_family", self._lp(), fam,
                  rs.data_ptr() if rs is not None else None,
                  si.data_ptr() if si is not None else None, float(p), int(block_len),
                  self.z.data_ptr(), self.y.data_ptr(), self._sp)
        self._keep_seeds = self._hold(rs, si)
        return self

    def pack(self, z, y):
        """Copy host/device arrays z [B,T,d], y [B,T] into the tiled layout."""
        torch = self.torch
        with self._on_stream():
            zt = torch.as_tensor(np.ascontiguousarray(z, dtype=np.float64)
                                 if isinstance(z, np.ndarray) else z
                                 ).to(self.device, torch.float64).contiguous()
            yt = torch.as_tensor(np.ascontiguousarray(y, dtype=np.float64)
                                 if isinstance(y, np.ndarray) else y
                                 ).to(self.device, torch.float64).contiguous()
        if tuple(zt.shape) != (self.L.B, self.L.T, self.L.d) or tuple(yt.shape) != (self.L.B, self.L.T):
            raise ValueError("z/y shape does not match the batch")
        self.rows_clipped = False
        self._call("ocx_dev_pack", self._lp(), zt.data_ptr(), yt.data_ptr(), self.z.data_ptr(),
                  self.y.data_ptr(), self._sp)
        self._keep = self._hold(zt, yt)
        return self

    def simulate_alg(self, alg_flag: int = 0, eta0: float = SQRT2, comparator=None,
                     x_last=None, closed_comparator: Optional[bool] = None, closed_out=None):
        """Launch the FTRL/FTL kernel; results land in self.regret/cum/comp (async).

        ``closed_comparator`` (default: the layout is not a bit-exact mode) takes the
        comparator loss in closed form, T/2 - ||theta_T||, wherever the kernel certifies
        it — every row inside the unit ball, every sub-gradient -y_t/2, checked on device
        per sequence — and so reads z once instead of twice (ocx_dev_simulate_alg_ex,
        OCX_ALG_CLIPPED_ROWS); the regret then equals the reference's up to rounding.  It is
        safe on any data: sequences that fail the check stream the second pass and are
        bit-identical to ``closed_comparator=False``.
        ``closed_out`` ([B] int32 device tensor, optional) receives 1 per sequence that took
        the closed form, 0 where the kernel streamed the second pass."""
        cp = comparator.data_ptr() if comparator is not None else None
        xp = x_last.data_ptr() if x_last is not None else None
        if closed_comparator is None:
            closed_comparator = not self.exact and comparator is None
        flags = _lib.OCX_ALG_CLIPPED_ROWS if closed_comparator else 0
        self._call("ocx_dev_simulate_alg_ex", self._lp(), self.z.data_ptr(), self.y.data_ptr(),
                  int(alg_flag), float(eta0), cp, self.regret.data_ptr(), self.cum.data_ptr(),
                  self.comp.data_ptr(), xp, flags,
                  closed_out.data_ptr() if closed_out is not None else None, self._sp)
        return self.regret

    def simulate_smart(self, thresh, eta0: float = SQRT2, switch_step=None,
                       closed_prefix: Optional[bool] = None,
                       closed_comparator: Optional[bool] = None, stats=None):
        """SMART (fast_algorithms.py:118-164) on the resident batch; thresh scalar or [B].

        ``closed_prefix`` (default: not a bit-exact layout) runs in O(T·d): the pre-switch
        prefix loss in closed form, deciding the switch only outside a rounding guard band
        and re-scanning the prefix inside it (the reference's switch steps; see
        include/ocx.h, OCX_SMART_CLOSED_PREFIX).  ``closed_comparator`` (same default) takes
        the final comparator loss in closed form where certified.  ``stats`` ([2] uint64
        (int64) device tensor, optional) accumulates re-scanned steps and closed-comparator
        sequences."""
        with self._on_stream():
            th = self.torch.as_tensor(np.broadcast_to(np.asarray(thresh, dtype=np.float64),
                                                      (self.L.B,)).copy()).to(self.device)
        sp = switch_step.data_ptr() if switch_step is not None else None
        if closed_prefix is None:
            closed_prefix = not self.exact
        if closed_comparator is None:
            closed_comparator = not self.exact
        flags = ((_lib.OCX_SMART_CLOSED_PREFIX if closed_prefix else 0) |
                 (_lib.OCX_ALG_CLOSED_COMPARATOR if closed_comparator else 0))
        self._call("ocx_dev_simulate_smart_ex", self._lp(), self.z.data_ptr(), self.y.data_ptr(),
                  th.data_ptr(), float(eta0), self.regret.data_ptr(), sp, flags,
                  stats.data_ptr() if stats is not None else None, self._sp)
        self._keep_th = self._hold(th)
        return self.regret

    def simulate_twin32(self, algo: int = 0, eta0: float = SQRT2, thresh=None):
        """The float32 twin (algorithms.py; twin32_batch) on the resident batch, which must
        use the one-lane layout (``lanes_per_seq=-1``): float32 results [B] on device."""
        torch = self.torch
        th = None
        with self._on_stream():
            res = torch.empty(max(self.L.B, 1), dtype=torch.float32, device=self.device)
            if int(algo) == 2:
                th = torch.as_tensor(np.broadcast_to(np.asarray(thresh, dtype=np.float64),
                                                     (self.L.B,)).copy()).to(self.device)
        self._call("ocx_dev_twin32", self._lp(), self.z.data_ptr(), self.y.data_ptr(), int(algo),
                  float(eta0), th.data_ptr() if th is not None else None, res.data_ptr(), None,
                  None, None, self._sp)
        if th is not None:
            self._keep_th = self._hold(th)
        return res

    def ftl_exact(self, cmp_action=None, regime=None, norm: str = "l2"):
        """Exact FTL (l2 ball, closed form; see ftl_exact_batch) on the resident batch:
        self.cum / self.comp get the replay and comparator losses, ``cmp_action``
        [B, d] (device, optional) the exact comparator, ``regime`` [B] int32 the
        regime flags (allocated when None).  Returns regime."""
        torch = self.torch
        if regime is None:
            with self._on_stream():
                regime = torch.zeros(max(self.L.B, 1), dtype=torch.int32, device=self.device)
        self._call("ocx_dev_ftl_exact", self._lp(), self.z.data_ptr(), self.y.data_ptr(),
                  _norm_code(norm),
                  self.cum.data_ptr(), self.comp.data_ptr(),
                  cmp_action.data_ptr() if cmp_action is not None else None,
                  regime.data_ptr(), self._sp)
        return regime

    def ftrl_vs_exact(self, eta0: float = SQRT2, comp_ftl=None, cmp_action=None, regime=None,
                      closed_comparator: Optional[bool] = None, norm: str = "l2"):
        """ftrl_vs_exact_batch on the resident batch: self.cum gets FTRL's cumulative loss,
        self.comp the exact comparator's loss, self.cum_exact exact FTL's (allocated on first
        use); ``comp_ftl`` [B] (device, optional) the loss of FTL(theta_ftrl).  Returns the
        regime flags.  ``closed_comparator`` (default: not a bit-exact layout) takes both
        comparator losses in closed form for the sequences the kernel finds in the unit-ball
        regime (ocx_dev_ftrl_vs_exact_ex): one HBM pass instead of two.  Under
        OCX_LANES_BEST the kernel sums with the butterfly (OCX_ALG_TREE_SUMS)."""
        torch = self.torch
        n = max(self.L.B, 1)
        with self._on_stream():
            if self.cum_exact is None:
                self.cum_exact = torch.zeros(n, dtype=torch.float64, device=self.device)
            if regime is None:
                regime = torch.zeros(n, dtype=torch.int32, device=self.device)
        if closed_comparator is None:
            closed_comparator = not self.exact
        flags = _lib.OCX_ALG_CLOSED_COMPARATOR if closed_comparator else 0
        if self.best and self.L.chain:
            # OCX_LANES_BEST: chained totals leave this kernel latency-bound (43 vs 28 ms at
            # 32768 x 1e4 x 64, profiles/r02_fused_exact_lanes.jsonl): butterfly sums instead
            flags |= _lib.OCX_ALG_TREE_SUMS
        self._call("ocx_dev_ftrl_vs_exact_ex", self._lp(), self.z.data_ptr(), self.y.data_ptr(),
                  float(eta0), self.cum.data_ptr(), self.cum_exact.data_ptr(),
                  self.comp.data_ptr(), comp_ftl.data_ptr() if comp_ftl is not None else None,
                  cmp_action.data_ptr() if cmp_action is not None else None, regime.data_ptr(),
                  _norm_code(norm), flags, self._sp)
        return regime

    def exact_general(self, norm: str = "l2", all_prefixes: bool = True):
        """The general exact-FTL solver (exact_ball_solve) on the resident batch
        (ocx_dev_exact_ball_solve_tiled, d <= 256): a dict of device tensors ``actions``
        [B, NP, d], ``obj``, ``gap``, ``step_loss`` [B, NP] and ``info`` (int32), NP = T+1
        or 1 (async on self.stream)."""
        torch = self.torch
        B, T, d = self.L.B, self.L.T, self.L.d
        if d > _lib.OCX_EXACT_BALL_MAX_D:
            raise NotImplementedError(f"the general exact-FTL solver takes d <= "
                                      f"{_lib.OCX_EXACT_BALL_MAX_D} (got {d})")
        NP = T + 1 if all_prefixes else 1
        with self._on_stream():
            out = {"actions": torch.zeros((max(B, 1), NP, d), dtype=torch.float64,
                                          device=self.device)}
            for k in ("obj", "gap", "step_loss"):
                out[k] = torch.zeros((max(B, 1), NP), dtype=torch.float64, device=self.device)
            out["info"] = torch.zeros((max(B, 1), NP), dtype=torch.int32, device=self.device)
        self._call("ocx_dev_exact_ball_solve_tiled", self._lp(), self.z.data_ptr(),
                  self.y.data_ptr(), _norm_code(norm), int(bool(all_prefixes)),
                  out["actions"].data_ptr(), out["obj"].data_ptr(), out["gap"].data_ptr(),
                  out["step_loss"].data_ptr(), out["info"].data_ptr(), self._sp)
        return out

    def ftrl_vs_exact_general(self, eta0: float = SQRT2, norm: str = "l2"):
        """ftrl_vs_exact with every sequence's exact side valid: the closed form where the
        kernel finds the regime, the general solver (exact_general) elsewhere.  Leaves
        self.cum (FTRL), self.cum_exact and self.comp as ftrl_vs_exact does; returns the
        regime flags.  Synchronises once (to see whether any sequence left the regime)."""
        torch = self.torch
        regime = self.ftrl_vs_exact(eta0, norm=norm)
        B, T, d = self.L.B, self.L.T, self.L.d
        self.exact_gap_max = 0.0
        with self._on_stream():
            ok = regime[:B].bool()
            if bool(ok.all().item()):
                return regime
            # only the sequences outside the regime: their rows out of the tile, row-major
            bad = torch.nonzero(~ok).flatten()
            zb, yb = self.rows_of(bad)
            nb = int(bad.numel())
            res = {"actions": torch.zeros((nb, T + 1, d), dtype=torch.float64, device=self.device)}
            for k in ("obj", "gap", "step_loss"):
                res[k] = torch.zeros((nb, T + 1), dtype=torch.float64, device=self.device)
            res["info"] = torch.zeros((nb, T + 1), dtype=torch.int32, device=self.device)
            self._call("ocx_dev_exact_ball_solve", zb.data_ptr(), yb.data_ptr(), nb, T, d,
                      _norm_code(norm), 1, res["actions"].data_ptr(), res["obj"].data_ptr(),
                      res["gap"].data_ptr(), res["step_loss"].data_ptr(),
                      res["info"].data_ptr(), self._sp)
            self._hold(zb, yb)
            host = {k: res[k].cpu().numpy() for k in ("obj", "gap", "info", "step_loss")}
            self.exact_gap_max = check_certificates(host["obj"], host["gap"], host["info"])
            # exact FTL's cumulative loss in step order (the host path's and the replay's)
            gcum = np.cumsum(host["step_loss"][:, :T], axis=1)[:, -1] if T > 0 else np.zeros(nb)
            self.cum_exact[bad] = torch.as_tensor(gcum).to(self.device)
            self.comp[bad] = res["obj"][:, T]
        return regime

    def rows_of(self, seqs):
        """z [n, T, d] and y [n, T] (device, row-major, contiguous) of the sequences ``seqs``
        (device int64 tensor of batch indices), gathered out of the tiled layout
        (include/ocx.h ocx_layout: z_tiled[((k*G + g)*T + t)*128 + L*2 + e])."""
        L = self.L
        K, G, T, S, P = L.C // 2, L.G, L.T, L.S, L.P
        g, s = seqs // S, seqs % S
        z5 = self.z[:K * G * T * 128].view(K, G, T, S, P, 2)
        zs = z5[:, g, :, s, :, :]                      # [n, K, T, P, 2]
        zs = zs.permute(0, 2, 3, 1, 4).reshape(seqs.numel(), T, P * L.C)[:, :, :L.d]
        ys = self.y[:G * T * S].view(G, T, S)[g, :, s]  # [n, T]
        return zs.contiguous(), ys.contiguous()

    def generate_simulate(self, base_seed: int = 0, run0: int = 0, nbatch: int = 1,
                          eta0: float = SQRT2, gmax=None, pipelined: bool = True,
                          sub_seqs: int = 0):
        """fast_algorithms.py:230-247's loop over ``nbatch`` resident batches in one call
        (ocx_dev_gen_simulate): batch k holds runs run0 + k*B .. run0 + (k+1)*B - 1,
        generated on device into this batch's z/y and simulated by FTRL.  self.regret gets
        the last batch's regrets; ``gmax`` ([1] float64 device tensor, optional) the max over
        every batch, from 0.0.  ``pipelined`` overlaps generation of one sub-batch with the
        FTRL pass over the previous one (d = 64, 8 x 8 / 16 x 4 butterfly layouts; otherwise,
        or with False, batch by batch).  The closed-form comparator is taken as in
        simulate_alg (the bit-exact layouts keep the streamed pass).  Same regrets either way,
        bit for bit."""
        flags = 0 if pipelined else _lib.OCX_GENSIM_SEQUENTIAL
        if self.exact:
            flags |= _lib.OCX_GENSIM_TWO_PASS
        self._call("ocx_dev_gen_simulate", self._lp(), int(base_seed), int(run0), int(nbatch),
                  self.z.data_ptr(), self.y.data_ptr(), float(eta0), self.regret.data_ptr(),
                  gmax.data_ptr() if gmax is not None else None, flags, int(sub_seqs), self._sp)
        self.rows_clipped = True
        return self.regret

    def max_regret(self, out=None):
        torch = self.torch
        if out is None:
            with self._on_stream():
                out = torch.zeros(1, dtype=torch.float64, device=self.device)
        self._call("ocx_dev_max_regret", self.regret.data_ptr(), int(self.L.B), out.data_ptr(),
                  self._sp)
        return out

    @property
    def z_bytes(self) -> int:
        return int(self.L.z_elems) * 8

    @property
    def y_bytes(self) -> int:
        return int(self.L.y_elems) * 8

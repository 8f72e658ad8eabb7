"""CPU oracle for the FTRL/FTL hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product package
(``online_convex_optimization_amd``) never imports it and has no CPU fallback.

Contents
--------
* ctypes bindings to ``ocx_oracle.c`` — a C restatement of
  ``fast_algorithms.py:11-164`` / ``exact_ftl.py:230-333`` in the reference's exact
  floating-point operation order (bit-identical to numba's default mode);
* restatements of the reference's sequence sources on top of NumPy, the
  third-party dependency that owns the RNG arithmetic (NumPy 2.2.6 here; the
  reference pins no version):
    - ``rng``            = ``_rng`` (fast_algorithms.py:254-257),
    - ``gT_sample``      = the g(T) sampler (fast_algorithms.py:231-239) with ``d``,
    - ``flip_sequence`` / ``switching_two_leaders_sequence`` /
      ``random_iid_sample`` / ``noisy_iid_sample`` (sequence_generation.py:24-100).

Parity status: pinned.  ``tests/test_oracle_golden.py`` checks these functions
bit-for-bit against fixtures produced by running the reference itself
(``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Dict, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libocx_oracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build() -> str:
    """Compile ocx_oracle.c (make) if the shared object is missing or stale."""
    src = os.path.join(_HERE, "ocx_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oc_simulate_alg.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_double, _dp, _dp, _dp, _dp, _dp]
        L.oc_simulate_smart.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                        ctypes.c_double, _dp, _i64p]
        L.oc_replay.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp]
        L.oc_simulate_alg_batch.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp, _dp,
                                            ctypes.c_int]
        L.oc_simulate_smart_batch.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, _dp, ctypes.c_double, _dp, _i64p,
                                              ctypes.c_int]
        L.oc_max_threads.restype = ctypes.c_int
        L.oc_ftl_exact.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp, _dp,
                                   ctypes.POINTER(ctypes.c_int)]
        L.oc_ftl_prefix_actions.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp,
                                            ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(_dp)


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


# ---------------------------------------------------------------------------
# Hot-path restatement (C)
# ---------------------------------------------------------------------------

def simulate_alg_full(z, y, alg_flag: int, eta0: float, comparator=None):
    """fast_algorithms.py:88-115 (+ exact_ftl.py:230-277 outputs).

    Returns (regret, cum_loss, comp_loss, x_last)."""
    z = _f64(z)
    y = _f64(y)
    T, d = z.shape
    comp = None if comparator is None else _f64(comparator)
    out = np.zeros(3, dtype=np.float64)
    x_last = np.zeros(d, dtype=np.float64)
    rc = lib().oc_simulate_alg(_ptr(z), _ptr(y), T, d, int(alg_flag), float(eta0), _ptr(comp),
                               _ptr(out[0:1]), _ptr(out[1:2]), _ptr(out[2:3]), _ptr(x_last))
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return float(out[0]), float(out[1]), float(out[2]), x_last


def simulate_alg(z, y, alg_flag: int, eta0: float) -> float:
    """fast_algorithms.py:171-177."""
    return simulate_alg_full(z, y, alg_flag, eta0)[0]


def simulate_SMART_like(z, y, theta_thresh: float, eta0: float, return_switch: bool = False):
    """fast_algorithms.py:184-195 → :118-164."""
    z = _f64(z)
    y = _f64(y)
    T, d = z.shape
    reg = np.zeros(1, dtype=np.float64)
    sw = np.zeros(1, dtype=np.int64)
    lib().oc_simulate_smart(_ptr(z), _ptr(y), T, d, float(theta_thresh), float(eta0), _ptr(reg),
                            sw.ctypes.data_as(_i64p))
    if return_switch:
        return float(reg[0]), int(sw[0])
    return float(reg[0])


def simulate_SMART(z, y, *, eta0: float = math.sqrt(2)) -> float:
    """fast_algorithms.py:198-200."""
    return simulate_SMART_like(z, y, math.sqrt(2 * z.shape[0]), eta0)


def replay_cum_loss(z, y, actions) -> float:
    """exact_ftl.py:317-322 (the replay loop)."""
    z = _f64(z)
    y = _f64(y)
    a = _f64(actions)
    T, d = z.shape
    out = np.zeros(1, dtype=np.float64)
    lib().oc_replay(_ptr(z), _ptr(y), T, d, _ptr(a), _ptr(out))
    return float(out[0])


def _poly_action(theta: np.ndarray, norm: str) -> np.ndarray:
    """Exact FTL over the l1 / linf unit ball for theta = -S (exact_ftl.py:83-105 in its
    linear regime): maximise x.S over the ball.  l1: sign(S_j*) e_j* at the FIRST largest
    |S_j| (0 if S = 0); linf: sign(S) componentwise (0 where S_j = 0)."""
    x = np.zeros_like(theta)
    if norm == "linf":
        x[theta > 0.0] = -1.0
        x[theta < 0.0] = 1.0
        return x
    a = np.abs(theta)
    j = int(np.argmax(a))            # first index of the maximum
    if a[j] > 0.0:
        x[j] = -1.0 if theta[j] > 0.0 else 1.0
    return x


def _dual_ok(zt: np.ndarray, norm: str) -> bool:
    if norm == "l1":
        return float(np.max(np.abs(zt), initial=0.0)) <= 1.0 + 1e-12
    acc = 0.0
    for v in zt:                     # sequential (the kernels' exact-mode order)
        acc += abs(float(v))
    return acc <= 1.0 + 1e-12


def _seqdot(a: np.ndarray, b: np.ndarray) -> float:
    acc = 0.0
    for u, v in zip(a, b):           # fast_algorithms.py:11-16 order
        acc += float(u) * float(v)
    return acc


def ftl_exact_poly(z, y, norm: str):
    """exact_ftl.py:280-333 over the l1 / linf ball in closed form (pure Python loops, small
    cases only) → (cum_loss, comp_loss, actions[T], in_regime, actions [T+1, d]).  The same
    operation order as the kernels in exact mode: theta += -y_t z_t, x_t from theta,
    q_t = z_t.x_t summed sequentially, the comparator loss in a second pass."""
    z = _f64(z)
    y = _f64(y)
    T, d = z.shape
    th = np.zeros(d)
    acts = np.zeros((T + 1, d))
    cum = 0.0
    ok = True
    for t in range(T):
        x = _poly_action(th, norm)
        acts[t] = x
        cum += 0.5 * abs(_seqdot(z[t], x) - y[t])
        ok = ok and _dual_ok(z[t], norm) and abs(y[t]) == 1.0
        th = th + (-y[t]) * z[t]
    xs = _poly_action(th, norm)
    acts[T] = xs
    comp = 0.0
    for t in range(T):
        comp += 0.5 * abs(_seqdot(z[t], xs) - y[t])
    return cum, comp, xs, ok, acts


def ftl_exact_closed_form(z, y, norm: str = "l2"):
    """exact_ftl.py:280-333 in closed form → (cum_loss, comp_loss, actions[T], in_regime).
    l2: oc_ftl_exact in ocx_oracle.c; l1 / linf: ftl_exact_poly."""
    if norm != "l2":
        cum, comp, xs, ok, _ = ftl_exact_poly(z, y, norm)
        return cum, comp, xs, ok
    z = _f64(z)
    y = _f64(y)
    T, d = z.shape
    out = np.zeros(2)
    a = np.zeros(d)
    rg = ctypes.c_int(0)
    lib().oc_ftl_exact(_ptr(z), _ptr(y), T, d, _ptr(out[0:1]), _ptr(out[1:2]), _ptr(a),
                       ctypes.byref(rg))
    return float(out[0]), float(out[1]), a, bool(rg.value)


def ftl_prefix_actions(z, y, norm: str = "l2"):
    """exact_ftl.py:280-303 in closed form → (actions [T+1, d], in_regime).
    l2: oc_ftl_prefix_actions in ocx_oracle.c; l1 / linf: ftl_exact_poly."""
    if norm != "l2":
        _, _, _, ok, acts = ftl_exact_poly(z, y, norm)
        return acts, ok
    z = _f64(z)
    y = _f64(y)
    T, d = z.shape
    a = np.zeros((T + 1, d))
    rg = ctypes.c_int(0)
    lib().oc_ftl_prefix_actions(_ptr(z), _ptr(y), T, d, _ptr(a), ctypes.byref(rg))
    return a, bool(rg.value)


def comparator_loss_blas(z, y, x) -> float:
    """exact_ftl.py:224-227 `_comparator_loss` (BLAS dgemv + pairwise |r| sum)."""
    r = _f64(z) @ _f64(x) - _f64(y)
    return 0.5 * float(np.abs(r).sum())


def simulate_alg_batch(z, y, alg_flag: int, eta0: float, comparator=None, nthreads: int = 1):
    """B independent sequences (z [B,T,d], y [B,T]) → (regret, cum_loss, comp_loss, x_last)."""
    z = _f64(z)
    y = _f64(y)
    B, T, d = z.shape
    comp = None if comparator is None else _f64(comparator)
    reg = np.zeros(B)
    cum = np.zeros(B)
    cl = np.zeros(B)
    xl = np.zeros((B, d))
    rc = lib().oc_simulate_alg_batch(_ptr(z), _ptr(y), B, T, d, int(alg_flag), float(eta0),
                                     _ptr(comp), _ptr(reg), _ptr(cum), _ptr(cl), _ptr(xl),
                                     int(nthreads))
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return reg, cum, cl, xl


def simulate_smart_batch(z, y, thresh, eta0: float, nthreads: int = 1):
    z = _f64(z)
    y = _f64(y)
    B, T, d = z.shape
    th = _f64(np.broadcast_to(np.asarray(thresh, dtype=np.float64), (B,)))
    reg = np.zeros(B)
    sw = np.zeros(B, dtype=np.int64)
    lib().oc_simulate_smart_batch(_ptr(z), _ptr(y), B, T, d, _ptr(th), float(eta0), _ptr(reg),
                                  sw.ctypes.data_as(_i64p), int(nthreads))
    return reg, sw


def max_threads() -> int:
    return int(lib().oc_max_threads())


# ---------------------------------------------------------------------------
# Sequence sources (NumPy owns the RNG arithmetic)
# ---------------------------------------------------------------------------

def rng(base_seed: int, T: int, run: int) -> np.random.Generator:
    """fast_algorithms.py:254-257 / algorithms.py:177-180."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([base_seed, T, run])))


def gT_sample(base_seed: int, T: int, run: int, d: int = 5) -> Tuple[np.ndarray, np.ndarray]:
    """fast_algorithms.py:231-239 (d=5 there; d is a parameter here)."""
    gen = rng(base_seed, T, run)
    z = gen.standard_normal((T, d)).astype(np.float64, copy=False)
    norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float64, copy=False)
    z *= (1.0 / np.maximum(norms, 1.0))
    y = gen.choice([-1.0, 1.0], size=T).astype(np.float64, copy=False)
    return z, y


def empirical_worst_case_thresholds(T_grid, *, runs: int = 5, base_seed: int = 0,
                                    d: int = 5) -> Dict[int, float]:
    """fast_algorithms.py:211-247 (max over runs, starting from 0.0)."""
    g: Dict[int, float] = {}
    for T_val in T_grid:
        T = int(T_val)
        m = 0.0
        for r in range(runs):
            z, y = gT_sample(base_seed, T, r, d)
            reg = simulate_alg(z, y, 0, math.sqrt(2))
            if reg > m:
                m = reg
        g[T] = m
    return g


def flip_sequence(T: int, d: int = 5):
    """sequence_generation.py:24-28."""
    z = np.zeros((T, d), dtype=np.float32)
    z[:, 0] = 1.0
    y = np.array([1.0 if t % 2 else -1.0 for t in range(1, T + 1)], dtype=np.float32)
    return z, y, np.zeros(d, dtype=np.float32)


def switching_two_leaders_sequence(T: int, *, block_len: int = 20, d: int = 5):
    """sequence_generation.py:36-47."""
    y = np.empty(T, dtype=np.float32)
    sign = 1.0
    idx = 0
    while idx < T:
        run = min(block_len, T - idx)
        y[idx:idx + run] = sign
        idx += run
        sign = -sign
    z = np.zeros((T, d), dtype=np.float32)
    z[:, 0] = 1.0
    return z, y, np.zeros(d, dtype=np.float32)


def _unit_u(run_seed: int, stream_id: int, d: int) -> np.ndarray:
    gen_u = rng(run_seed, 0, stream_id)
    u = gen_u.standard_normal(d).astype(np.float32, copy=False)
    n = float(np.linalg.norm(u))
    if n > 0:
        u /= n
    return u


def random_iid_sample(run_seed: int, T: int, rep: int = 0, d: int = 5):
    """sequence_generation.py:54-69 (make_random_iid_stream → sample)."""
    u = _unit_u(run_seed, 11, d)
    gen = rng(run_seed, T, 13 + rep)
    z = gen.standard_normal((T, d)).astype(np.float32, copy=False)
    norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float32, copy=False)
    np.maximum(norms, 1.0, out=norms)
    z *= (1.0 / norms)
    y = np.sign(z @ u).astype(np.float32, copy=False)
    y[y == 0.0] = 1.0
    return z, y, u


def noisy_iid_sample(run_seed: int, T: int, rep: int = 0, p: float = 0.10, d: int = 5):
    """sequence_generation.py:72-89 (make_noisy_iid_stream → sample)."""
    u = _unit_u(run_seed, 21, d)
    gen = rng(run_seed, T, 23 + rep)
    z = gen.standard_normal((T, d)).astype(np.float32, copy=False)
    norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float32, copy=False)
    np.maximum(norms, 1.0, out=norms)
    z *= (1.0 / norms)
    y = np.sign(z @ u).astype(np.float32, copy=False)
    y[y == 0.0] = 1.0
    flips = gen.random(T) < p
    y[flips] *= -1.0
    return z, y, u

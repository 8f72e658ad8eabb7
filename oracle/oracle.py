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


def _poly_tie(theta: np.ndarray, touched: np.ndarray, norm: str) -> bool:
    """Prefixes whose LP optimum is a face the closed form does not centre (kernels:
    ocx_exact_poly_tie): l1 with two or more coordinates at max |S_j| > 0; linf with S_j = 0
    in a coordinate some row of the prefix touched.  The engine answers those sequences with
    the general solver (the analytic centre of the face, as interior-point cvxpy backends)."""
    if norm == "l1":
        a = np.abs(theta)
        m = float(a.max(initial=0.0))
        return m > 0.0 and int((a == m).sum()) >= 2
    if norm == "linf":
        return bool(np.any((theta == 0.0) & touched))
    return False


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
    touched = np.zeros(d, dtype=bool)
    for t in range(T):
        x = _poly_action(th, norm)
        acts[t] = x
        ok = ok and not _poly_tie(th, touched, norm)
        cum += 0.5 * abs(_seqdot(z[t], x) - y[t])
        ok = ok and _dual_ok(z[t], norm) and abs(y[t]) == 1.0
        touched |= z[t] != 0.0
        th = th + (-y[t]) * z[t]
    xs = _poly_action(th, norm)
    ok = ok and not _poly_tie(th, touched, norm)
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


# ---------------------------------------------------------------------------
# float32 twin (algorithms.py:10-171) in explicit operation order
# ---------------------------------------------------------------------------
# The twin's NumPy calls, as this image's NumPy 2.2 / OpenBLAS 0.3.29 compute them
# (probed, and pinned by tests/golden/twin32.npz, made by running the calls themselves):
#   sdot (np.dot, np.linalg.norm, 1-D @ 1-D), n < 32: float products summed in double;
#   sgemv (z @ x): rows in blocks of four by a float fma chain over the columns, the
#     n mod 4 tail rows by a plain float chain, a one-row matrix by the sdot rule (d = 5);
#   np.sum (float32): pairwise (leaves <= 128, 8 accumulators) per 8192-element buffer;
#   NEP 50: Python scalars take float32; Python float - np.float32 -> float32.
# Only the fma is emulated through float64 (exact product, then the sum rounded twice):
# the double rounding differs from a true fma with probability ~2^-29 per operation.

_F = np.float32


def t32_sdot(a, b) -> np.float32:
    """OpenBLAS sdot for n < 32 (algorithms.py:14, :19, :41, :91)."""
    p = (np.asarray(a, _F) * np.asarray(b, _F)).astype(np.float64)
    acc = 0.0
    for v in p:
        acc += float(v)
    return _F(acc)


def t32_gemv(z, x) -> np.ndarray:
    """z @ x for a float32 [n, d] matrix (algorithms.py:52, :110, :117)."""
    z = np.asarray(z, _F)
    x = np.asarray(x, _F)
    n, d = z.shape
    if n == 1:
        return np.array([t32_sdot(z[0], x)], dtype=_F)
    nb = 4 * (n // 4)
    q = np.empty(n, dtype=_F)
    acc = np.zeros(nb, dtype=_F)
    for j in range(d):
        acc = (z[:nb, j].astype(np.float64) * float(x[j]) + acc.astype(np.float64)).astype(_F)
    q[:nb] = acc
    acc = np.zeros(n - nb, dtype=_F)
    for j in range(d):
        acc = acc + z[nb:, j] * x[j]
    q[nb:] = acc
    return q


def _t32_leaf(a: np.ndarray) -> np.float32:
    n = len(a)
    if n < 8:
        r = _F(-0.0)
        for v in a:
            r = _F(r + v)
        return r
    m = n - n % 8
    r = a[:8].copy()
    for i in range(8, m, 8):
        r = r + a[i:i + 8]
    res = _F(_F(_F(r[0] + r[1]) + _F(r[2] + r[3])) + _F(_F(r[4] + r[5]) + _F(r[6] + r[7])))
    for v in a[m:]:
        res = _F(res + v)
    return res


def _t32_pairwise(a: np.ndarray) -> np.float32:
    n = len(a)
    if n <= 128:
        return _t32_leaf(a)
    n2 = n // 2
    n2 -= n2 % 8
    return _F(_t32_pairwise(a[:n2]) + _t32_pairwise(a[n2:]))


def t32_sum(a) -> np.float32:
    """np.sum of a contiguous float32 vector."""
    a = np.asarray(a, _F)
    tot = None
    for s in range(0, len(a), 8192):
        p = _t32_pairwise(a[s:s + 8192])
        tot = p if tot is None else _F(tot + p)
    return _F(0.0) if tot is None else tot


def t32_row_norms(z) -> np.ndarray:
    """np.linalg.norm(z, axis=1) of a float32 [n, d] matrix (algorithms.py:159)."""
    z = np.asarray(z, _F)
    sq = z * z
    return np.sqrt(np.array([_t32_leaf(r) for r in sq], dtype=_F))


def t32_action_ftl(theta) -> np.ndarray:
    """algorithms.py:13-15."""
    n = np.sqrt(t32_sdot(theta, theta))
    if n == 0.0:
        return np.zeros_like(theta)
    return (-(_F(1.0) / n)) * theta


def t32_action_ftrl(theta, t: int, eta0: float) -> np.ndarray:
    """algorithms.py:17-21."""
    x = _F(-(eta0 / math.sqrt(max(1, t)))) * theta
    n = np.sqrt(t32_sdot(x, x))
    if n > 1.0:
        x = x * (_F(1.0) / n)
    return x


def _t32_grad(diff: float) -> float:
    return 0.5 if diff > 0.0 else -0.5 if diff < 0.0 else 0.0


def _t32_comp(z, y, x) -> np.float32:
    return t32_sum(_F(0.5) * np.abs(t32_gemv(z, x) - y))


def t32_simulate_alg_full(z, y, alg_flag: int, eta0: float):
    """algorithms.py:28-54 → (np.float32 result, cum_loss, comp_loss)."""
    z = np.ascontiguousarray(z, dtype=_F)
    y = np.ascontiguousarray(y, dtype=_F)
    T, d = z.shape
    theta = np.zeros(d, dtype=_F)
    cum = 0.0
    for t in range(T):
        x = t32_action_ftrl(theta, t + 1, eta0) if alg_flag == 0 else t32_action_ftl(theta)
        q = float(t32_sdot(z[t], x))
        yt = float(y[t])
        cum += 0.5 * abs(q - yt)
        theta = theta + _F(_t32_grad(q - yt)) * z[t]
    comp = _t32_comp(z, y, t32_action_ftl(theta))
    return _F(_F(cum) - comp), cum, comp


def t32_simulate_smart_full(z, y, theta_thresh: float, eta0: float):
    """algorithms.py:65-120 → (np.float32 result, total_loss, comp_loss, switch step or -1)."""
    z = np.ascontiguousarray(z, dtype=_F)
    y = np.ascontiguousarray(y, dtype=_F)
    T, d = z.shape
    th_ftl = np.zeros(d, dtype=_F)
    th_ftrl = np.zeros(d, dtype=_F)
    thr = _F(theta_thresh)
    switched, sw = False, -1
    ftl_loss = total = 0.0
    for t in range(T):
        yt = float(y[t])
        pf = float(t32_sdot(z[t], t32_action_ftl(th_ftl)))
        th_ftl = th_ftl + _F(_t32_grad(pf - yt)) * z[t]
        lf = 0.5 * abs(pf - yt)
        ftl_loss += lf
        if switched:
            pr = float(t32_sdot(z[t], t32_action_ftrl(th_ftrl, t + 1, eta0)))
            total += 0.5 * abs(pr - yt)
            th_ftrl = th_ftrl + _F(_t32_grad(pr - yt)) * z[t]
        else:
            total += lf
            sl = _t32_comp(z[:t + 1], y[:t + 1], t32_action_ftl(th_ftl))
            if _F(_F(ftl_loss) - sl) >= thr:
                switched, sw = True, t
    comp = _t32_comp(z, y, t32_action_ftl(th_ftl))
    return _F(_F(total) - comp), total, comp, sw


def t32_gT_sample(base_seed: int, T: int, run: int, d: int = 5):
    """The twin's g(T) sampler (algorithms.py:155-163) with ``d`` as a parameter."""
    gen = rng(base_seed, T, run)
    z = gen.standard_normal((T, d)).astype(_F)
    norms = t32_row_norms(z)[:, None]
    z = z * (_F(1.0) / np.maximum(norms, _F(1.0)))
    y = gen.choice([-1.0, 1.0], size=T).astype(_F)
    return z, y


def t32_empirical_worst_case_thresholds(T_grid, *, runs: int = 5, base_seed: int = 0):
    """algorithms.py:135-171."""
    out = {}
    for T_val in T_grid:
        T = int(T_val)
        m = 0.0
        for r in range(runs):
            z, y = t32_gT_sample(base_seed, T, r)
            reg = t32_simulate_alg_full(z, y, 0, math.sqrt(2))[0]
            if reg > m:
                m = reg
        out[T] = m
    return out


# ---------------------------------------------------------------------------
# exact_ftl.py:224-227 `_comparator_loss` in explicit operation order
# ---------------------------------------------------------------------------
# z @ x - y goes to OpenBLAS dgemv_t (this image: 0.3.29, Haswell-class kernels); probed
# and pinned against tests/golden (made by the reference itself):
#   rows in groups of four (the 4x4 kernel): per row a 4-lane fma accumulation over the
#     first m1 = d & ~3 coordinates, lanes summed as (l0 + l2) + (l1 + l3);
#   where T mod 4 >= 2, the next two rows (the 4x2 kernel): per row a 2-lane accumulation
#     of plain products over the first m1 coordinates (lane j: coordinates 2i + j), l0 + l1;
#   a last single row (T mod 4 = 1 or 3; the 4x1 kernel): 4-lane products summed block
#     after block with plain adds, lanes (l0 + l2) + (l1 + l3);
#   then the d mod 4 tail: 1 -> fma(a0, x0, s); 2 -> s + fma(a0, x0, a1 x1);
#     3 -> s + fma(a2, x2, fma(a0, x0, a1 x1));
#   a one-row matrix goes to ddot: an fma chain for d < 16; from d = 16 four 4-lane fma
#     accumulators over 16-coordinate blocks — for the first d & ~31 coordinates four 8-lane
#     fma accumulators over 32-coordinate blocks, each folded to 4 lanes as l_k + l_(k+4)
#     before the 16-blocks continue them —, then ((a0 + a1) + a2) + a3,
#     (l0 + l2) + (l1 + l3), and an fma tail over the last d mod 16 coordinates.
#   (The 4x2 rows and the d >= 32 ddot were probed against numpy on this image in round 3:
#   tests/test_oracle_golden.py::test_comparator_blas_order_matches_numpy.)
# np.abs(r).sum(): NumPy's pairwise sum (float64, 8192-element buffers); then 0.5 * sum.
from fractions import Fraction as _Fr  # noqa: E402


def _fma64(a, b, c) -> float:
    return float(_Fr(float(a)) * _Fr(float(b)) + _Fr(float(c)))


def _dgemv_tail(s: float, a, x) -> float:
    m3 = len(a)
    if m3 == 1:
        return _fma64(a[0], x[0], s)
    if m3 == 2:
        return s + _fma64(a[0], x[0], float(a[1]) * float(x[1]))
    if m3 == 3:
        return s + _fma64(a[2], x[2], _fma64(a[0], x[0], float(a[1]) * float(x[1])))
    return s


def dgemv_row(r, x, t: int, T: int) -> float:
    """Row t of the T-row dgemv z @ x (see the block comment above)."""
    d = len(r)
    r = [float(v) for v in r]
    x = [float(v) for v in x]
    if T == 1:
        if d < 16:
            s = 0.0
            for i in range(d):
                s = _fma64(r[i], x[i], s)
            return s
        n1, n32 = d & ~15, d & ~31
        a8 = [[0.0] * 8 for _ in range(4)]
        for b in range(0, n32, 32):
            a8 = [[_fma64(r[b + 8 * j + k], x[b + 8 * j + k], a8[j][k]) for k in range(8)]
                  for j in range(4)]
        acc = [[a8[j][k] + a8[j][k + 4] for k in range(4)] for j in range(4)]
        for b in range(n32, n1, 16):
            acc = [[_fma64(r[b + 4 * j + k], x[b + 4 * j + k], acc[j][k]) for k in range(4)]
                   for j in range(4)]
        tot = [((acc[0][k] + acc[1][k]) + acc[2][k]) + acc[3][k] for k in range(4)]
        s = (tot[0] + tot[2]) + (tot[1] + tot[3])
        for i in range(n1, d):
            s = _fma64(r[i], x[i], s)
        return s
    m1 = d & ~3
    s = 0.0
    if m1:
        q4 = 4 * (T // 4)
        if t < q4:  # 4x4 kernel
            acc = [0.0] * 4
            for i in range(0, m1, 4):
                acc = [_fma64(r[i + k], x[i + k], acc[k]) for k in range(4)]
            s = (acc[0] + acc[2]) + (acc[1] + acc[3])
        elif T % 4 >= 2 and t < q4 + 2:  # 4x2 kernel
            a2 = [r[0] * x[0], r[1] * x[1]]
            for i in range(2, m1, 2):
                a2 = [a2[j] + r[i + j] * x[i + j] for j in range(2)]
            s = a2[0] + a2[1]
        else:  # 4x1 kernel
            acc = [r[k] * x[k] for k in range(4)]
            for i in range(4, m1, 4):
                acc = [acc[k] + r[i + k] * x[i + k] for k in range(4)]
            s = (acc[0] + acc[2]) + (acc[1] + acc[3])
    return _dgemv_tail(s, r[m1:], x[m1:])


def _pw64_leaf(a) -> float:
    n = len(a)
    if n < 8:
        s = -0.0
        for v in a:
            s = s + v
        return s
    m = n - n % 8
    r = list(a[:8])
    for i in range(8, m, 8):
        r = [r[k] + a[i + k] for k in range(8)]
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    for v in a[m:]:
        s = s + v
    return s


def _pw64(a) -> float:
    n = len(a)
    if n <= 128:
        return _pw64_leaf(a)
    n2 = n // 2
    n2 -= n2 % 8
    return _pw64(a[:n2]) + _pw64(a[n2:])


def sum64_numpy_order(a) -> float:
    """np.sum of a contiguous float64 vector."""
    a = [float(v) for v in a]
    tot = None
    for s in range(0, len(a), 8192):
        p = _pw64(a[s:s + 8192])
        tot = p if tot is None else tot + p
    return 0.0 if tot is None else tot


def comparator_loss_blas_order(z, y, x) -> float:
    """exact_ftl.py:224-227 with every operation in the order OpenBLAS and NumPy use."""
    z = _f64(z)
    y = _f64(y)
    T = z.shape[0]
    r = [abs(dgemv_row(z[t], x, t, T) - float(y[t])) for t in range(T)]
    return 0.5 * sum64_numpy_order(r)

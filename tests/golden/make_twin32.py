"""Fixtures for the float32 twin (reference ``algorithms.py:10-171``) — test data only.

Usage (build container; writes ``tests/golden/twin32.npz``)::

    python tests/golden/make_twin32.py

Importing the reference module was refused by the environment, so the
expected values come from the twin's own NumPy calls, made here by the functions below
(``np_*``): the same calls, on the same float32 arrays, with the same Python-float
accumulators, in the same order as ``algorithms.py``.  On this image (NumPy 2.2,
OpenBLAS 0.3.29) they are what the reference module returns.  The script then checks that
the explicit-order restatement in ``oracle/oracle.py`` (``t32_*``: the arithmetic the GPU
kernel implements) reproduces every value bit for bit, and stores inputs and outputs:

* ``alg_T{T}_*``   — explicit random sequences (d = 5), FTRL with three eta0 and FTL;
* ``fam_*``        — the deterministic families (exact ties) and i.i.d./noisy streams;
* ``long_*``       — one T = 10000 sequence (two 8192-element sum buffers);
* ``smart_*``      — SMART with thresholds that switch early, late and never;
* ``dim{d}_*``     — d in {1, 2, 8, 16, 31} (the host BLAS orders sgemv differently for
                     some of them; the GPU is held to a tolerance there);
* ``gT_*``         — the twin's g(T) sampler and its thresholds (runs 0..15);
* ``cfg0_*``       — BASELINE configs[0]: d = 2, T = 1000 (an i.i.d. stream, a g(T) sample).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

F = np.float32


# ---- the twin's NumPy calls --------------------------------------------------------------
def _np_ftl(theta, out):
    n = np.linalg.norm(theta)
    out[:] = 0.0 if n == 0.0 else -(1.0 / n) * theta


def _np_ftrl(theta, t, eta0, out):
    out[:] = -(eta0 / math.sqrt(max(1, t))) * theta
    n = np.linalg.norm(out)
    if n > 1.0:
        out *= 1.0 / n


def _np_grad(q, y):
    diff = q - y
    return 0.5 if diff > 0.0 else -0.5 if diff < 0.0 else 0.0


def np_simulate_alg(z, y, alg_flag, eta0):
    T, d = z.shape
    theta = np.zeros(d, dtype=np.float32)
    x = np.zeros(d, dtype=np.float32)
    cum = 0.0
    for t in range(T):
        if alg_flag == 0:
            _np_ftrl(theta, t + 1, eta0, x)
        else:
            _np_ftl(theta, x)
        q = float(np.dot(z[t], x))
        yt = float(y[t])
        cum += 0.5 * abs(q - yt)
        theta += _np_grad(q, yt) * z[t]
    _np_ftl(theta, x)
    comp = np.sum(0.5 * np.abs(z @ x - y))
    return cum - comp, cum, comp


def np_simulate_smart(z, y, thresh, eta0):
    T, d = z.shape
    th_f = np.zeros(d, dtype=np.float32)
    th_r = np.zeros(d, dtype=np.float32)
    x = np.zeros(d, dtype=np.float32)
    s = np.zeros(d, dtype=np.float32)
    switched, sw = False, -1
    ftl_loss = total = 0.0
    for t in range(T):
        zt = z[t]
        yt = float(y[t])
        _np_ftl(th_f, x)
        pf = float(zt @ x)
        th_f += _np_grad(pf, yt) * zt
        lf = 0.5 * abs(pf - yt)
        ftl_loss += lf
        if switched:
            _np_ftrl(th_r, t + 1, eta0, x)
            pr = float(zt @ x)
            total += 0.5 * abs(pr - yt)
            th_r += _np_grad(pr, yt) * zt
        else:
            total += lf
            _np_ftl(th_f, s)
            s_loss = np.sum(0.5 * np.abs(z[:t + 1] @ s - y[:t + 1]))
            if ftl_loss - s_loss >= thresh:
                switched, sw = True, t
    _np_ftl(th_f, s)
    comp = np.sum(0.5 * np.abs(z @ s - y))
    return total - comp, total, comp, sw


def np_gT_sample(T, run, d=5, base_seed=0):
    gen = O.rng(base_seed, T, run)
    z = gen.standard_normal((T, d)).astype(np.float32, copy=False)
    norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float32, copy=False)
    z *= (1.0 / np.maximum(norms, 1.0))
    y = gen.choice([-1.0, 1.0], size=T).astype(np.float32, copy=False)
    return z, y


# ---- fixtures ------------------------------------------------------------------------------
def _alg_group(out, key, z, y, runs):
    """runs: list of (alg_flag, eta0); one output row per run per sequence."""
    B = z.shape[0]
    res = np.zeros((len(runs), B), np.float32)
    cum = np.zeros((len(runs), B))
    comp = np.zeros((len(runs), B), np.float32)
    for i, (a, e) in enumerate(runs):
        for b in range(B):
            r, c, p = np_simulate_alg(z[b], y[b], a, e)
            o = O.t32_simulate_alg_full(z[b], y[b], a, e)
            assert type(r) is np.float32 and r == o[0] and c == o[1] and p == o[2], (key, a, e, b)
            res[i, b], cum[i, b], comp[i, b] = r, c, p
    out[key + "_z"], out[key + "_y"] = z, y
    out[key + "_runs"] = np.array(runs, dtype=np.float64)
    out[key + "_res"], out[key + "_cum"], out[key + "_comp"] = res, cum, comp


def _smart_group(out, key, z, y, thresholds, eta0=math.sqrt(2)):
    B = z.shape[0]
    nt = len(thresholds)
    res = np.zeros((nt, B), np.float32)
    cum = np.zeros((nt, B))
    comp = np.zeros((nt, B), np.float32)
    sw = np.zeros((nt, B), np.int64)
    for i, th in enumerate(thresholds):
        for b in range(B):
            r, c, p, s = np_simulate_smart(z[b], y[b], th, eta0)
            o = O.t32_simulate_smart_full(z[b], y[b], th, eta0)
            assert type(r) is np.float32 and (r, c, p, s) == o, (key, th, b)
            res[i, b], cum[i, b], comp[i, b], sw[i, b] = r, c, p, s
    out[key + "_z"], out[key + "_y"] = z, y
    out[key + "_thresh"] = np.array(thresholds, dtype=np.float64)
    out[key + "_res"], out[key + "_cum"], out[key + "_comp"], out[key + "_sw"] = res, cum, comp, sw


def main():
    rng = np.random.default_rng(20261016)
    out = {}
    runs = [(0, math.sqrt(2)), (0, 1.0), (0, 0.1), (1, math.sqrt(2))]
    for T in (1, 2, 3, 5, 7, 8, 64, 100, 1000):
        B = 6 if T <= 100 else 3
        z = rng.standard_normal((B, T, 5)).astype(F)
        z[: B // 2] *= F(0.3)  # short rows (FTRL's unclipped branch) and long ones
        y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0).astype(F)
        _alg_group(out, f"alg_T{T}", z, y, runs)
    # families: exact ties (flip, switching leaders), i.i.d. and 10 % noisy labels
    T = 200
    fam = [O.flip_sequence(T), O.switching_two_leaders_sequence(T),
           O.random_iid_sample(7, T, 0), O.noisy_iid_sample(7, T, 1)]
    zf = np.stack([np.asarray(f[0], F) for f in fam])
    yf = np.stack([np.asarray(f[1], F) for f in fam])
    _alg_group(out, "fam", zf, yf, runs)
    # two sum buffers
    zl = (rng.standard_normal((1, 10000, 5)) * 0.4).astype(F)
    yl = np.where(rng.random((1, 10000)) < 0.5, -1.0, 1.0).astype(F)
    _alg_group(out, "long", zl, yl, [(0, math.sqrt(2)), (1, math.sqrt(2))])
    # SMART: random rows and the families
    T = 300
    zs = (rng.standard_normal((4, T, 5)) * 0.5).astype(F)
    ys = np.where(rng.random((4, T)) < 0.5, -1.0, 1.0).astype(F)
    fam = [O.flip_sequence(T), O.switching_two_leaders_sequence(T),
           O.random_iid_sample(8, T, 0), O.noisy_iid_sample(8, T, 1)]
    zs = np.concatenate([zs, np.stack([np.asarray(f[0], F) for f in fam])])
    ys = np.concatenate([ys, np.stack([np.asarray(f[1], F) for f in fam])])
    _smart_group(out, "smart", zs, ys, [0.5, 2.0, 5.0, math.sqrt(2 * T), 1e9])
    # other dimensions
    for d in (1, 2, 8, 16, 31):
        z = rng.standard_normal((3, 50, d)).astype(F) * F(0.4)
        y = np.where(rng.random((3, 50)) < 0.5, -1.0, 1.0).astype(F)
        _alg_group(out, f"dim{d}", z, y, [(0, math.sqrt(2)), (1, math.sqrt(2))])
    # the twin's g(T) sampler (inputs are regenerated on device from the seeds)
    for T in (10, 100, 1000):
        regs = np.zeros(16, np.float32)
        for r in range(16):
            z, y = np_gT_sample(T, r)
            zo, yo = O.t32_gT_sample(0, T, r)
            assert np.array_equal(z, zo) and np.array_equal(y, yo), (T, r)
            regs[r] = np_simulate_alg(z, y, 0, math.sqrt(2))[0]
            assert regs[r] == O.t32_simulate_alg_full(zo, yo, 0, math.sqrt(2))[0]
        out[f"gT_T{T}_regrets"] = regs
    # BASELINE configs[0]: driver.py's single FTL run, d = 2, T = 1000, one random sequence
    # (the i.i.d. family of sequence_generation.py:54-69 at d = 2, and one g(T) sample)
    zc, yc, _ = O.random_iid_sample(2025, 1000, 0, d=2)
    zg, yg = np_gT_sample(1000, 0, d=2)
    _alg_group(out, "cfg0", np.stack([np.asarray(zc, F), zg]), np.stack([np.asarray(yc, F), yg]),
               runs)
    grid = [100, 200, 300]
    g = O.t32_empirical_worst_case_thresholds(grid, runs=8)
    out["gT_grid"] = np.array(grid, np.int64)
    out["gT_grid_g"] = np.array([g[T] for T in grid], np.float32)
    out["meta"] = np.array([f"numpy {np.__version__}"])
    path = os.path.join(HERE, "twin32.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} bytes, {len(out)} arrays)")


if __name__ == "__main__":
    main()

"""The pipelined butterfly FTRL/FTL kernel (ocx_alg_pipe.hip), which DeviceBatch.simulate_alg
runs for butterfly layouts (lanes_per_seq >= 2) when no input comparator or x_last is asked
for: every (C, P) instance it dispatches, FTRL and FTL, the closed-form comparator and the
second pass, against the C oracle (fast_algorithms.py:88-115).

Bars: the butterfly layouts' 1e-12 relative (two-pass) and close_closed (closed form), as in
test_gpu_parity.py; bit for bit on rows with one nonzero coordinate (the flip / switching
families), where every quantity of the pipelined step is exact."""
import math

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
SQ2 = math.sqrt(2.0)


@pytest.fixture(scope="module")
def eng():
    from online_convex_optimization_amd import _lib, engine
    _lib.load()
    return engine


def close(a, b, tol=1e-12):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


def close_closed(a, b, T):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    bar = np.maximum(1e-12 * np.maximum(1.0, np.abs(b)), 4 * 2.2e-16 * max(T, 1) ** 1.5)
    return np.all(np.abs(a - b) <= bar)


# (lanes per sequence, d): C = d / P coordinates per lane in {4, 8, 16, 32}
SHAPES = [(8, 32), (8, 64), (8, 128), (8, 256), (16, 64), (16, 128), (16, 512), (32, 128),
          (32, 1024)]


@pytest.mark.parametrize("P,d", SHAPES)
def test_pipe_kernel_matches_oracle(eng, P, d):
    import torch
    B, T = 21, 257
    rng = np.random.default_rng(P * 7919 + d)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    z[3] *= 1.7                     # a sequence outside the ball: the second pass
    y[5, ::9] = 0.5                 # labels other than ±1: the second pass
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).pack(z, y)
    assert (db.L.P, db.L.chain) == (P, 0)
    for flag in (0, 1):
        ref = O.simulate_alg_batch(z, y, flag, SQ2, nthreads=4)
        closed = torch.zeros(B, dtype=torch.int32, device=db.device)
        r2 = db.simulate_alg(flag, SQ2, closed_comparator=False).clone()
        cum2 = db.cum.clone()
        r1 = db.simulate_alg(flag, SQ2, closed_comparator=True, closed_out=closed).clone()
        torch.cuda.synchronize()
        r1, r2, cum2 = r1.cpu().numpy(), r2.cpu().numpy(), cum2.cpu().numpy()
        assert close(r2[:B], ref[0]) and close(cum2[:B], ref[1]), (P, d, flag)
        assert np.array_equal(db.cum[:B].cpu().numpy(), cum2[:B])   # the loop is the same
        flags = closed[:B].cpu().numpy()
        assert flags[3] == 0 and flags[5] == 0                     # not certified
        assert np.array_equal(r1[[3, 5]], r2[[3, 5]])               # second pass, bit for bit
        assert close_closed(r1[:B], ref[0], T), (P, d, flag)


@pytest.mark.parametrize("P", [8, 16, 32])
def test_pipe_kernel_exact_on_single_coordinate_rows(eng, P):
    """Flip / switching rows (one nonzero coordinate): exact ties q = y survive the
    pipelined step — regrets bit-identical to the reference's."""
    d = 64 if P < 32 else 128
    for fn in (O.flip_sequence, O.switching_two_leaders_sequence):
        z, y, _ = fn(1000, d=d)
        Z = np.repeat(z[None].astype(np.float64), 5, axis=0)
        Y = np.repeat(y[None].astype(np.float64), 5, axis=0)
        db = eng.DeviceBatch(5, Z.shape[1], d, lanes_per_seq=P).pack(Z, Y)
        assert db.L.P == P and db.L.chain == 0
        for flag in (0, 1):
            ref = O.simulate_alg(z, y, flag, SQ2)
            got = db.simulate_alg(flag, SQ2, closed_comparator=False).cpu().numpy()[:5]
            assert np.all(got == ref), (fn.__name__, P, flag, got, ref)


def test_pipe_kernel_long_horizon_drift(eng):
    """||θ||² is carried by a running update and summed afresh every 64 steps: over T = 2e4
    the regrets stay within the butterfly bar of the oracle."""
    import torch
    B, T, d = 8, 20000, 64
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=8).generate_gT(base_seed=11, run0=0)
    r = db.simulate_alg(0, SQ2, closed_comparator=False).clone()
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    for b in (0, 3, 7):
        zz, yy = O.gT_sample(11, T, b, d)
        assert close(r[b], O.simulate_alg(zz, yy, 0, SQ2)), b


@pytest.mark.parametrize("P,d", [(8, 64), (16, 64), (32, 1024)])
def test_spec_step_is_bit_identical(eng, P, d, monkeypatch):
    """The SPEC step (ĝ_{t-1} = −y_{t-1}/2 assumed, every step checked, a wave whose check
    fails runs the plain loop again) against the plain pipelined step, OCX_PIPE_SPEC read per
    launch: bit for bit on g(T) rows (no check fails) and on a batch whose checks fail in some
    waves (a row outside the ball, labels other than ±1, exact ties on one-coordinate rows)."""
    import torch
    B, T = 70, 300
    rng = np.random.default_rng(P + d)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    z[3] *= 1.7
    y[40, ::9] = 0.5
    zf, yf, _ = O.flip_sequence(T, d=d)
    z[60], y[60] = zf, yf
    batches = [eng.DeviceBatch(B, T, d, lanes_per_seq=P).pack(z, y),
               eng.DeviceBatch(3 * 64 // P + 5, 2000, d, lanes_per_seq=P).generate_gT(7)]
    for db in batches:
        for flag in (0, 1):
            out = {}
            for spec in ("0", "1"):
                monkeypatch.setenv("OCX_PIPE_SPEC", spec)
                closed = torch.zeros(db.L.B, dtype=torch.int32, device=db.device)
                r = db.simulate_alg(flag, SQ2, closed_comparator=True, closed_out=closed)
                torch.cuda.synchronize()
                out[spec] = (r[:db.L.B].cpu().numpy().copy(), db.cum[:db.L.B].cpu().numpy().copy(),
                             closed[:db.L.B].cpu().numpy().copy())
            for a, b in zip(out["0"], out["1"]):
                assert np.array_equal(a, b), (P, d, flag)


@pytest.mark.parametrize("T", [1, 2, 64, 65])
def test_spec_step_short_horizons(eng, T, monkeypatch):
    """SPEC at horizons around its pending-step bookkeeping (the step before step 0, the
    last step finished after the loop, the 64-step refresh): bit for bit with the plain step
    and within the bar of the C oracle."""
    import torch
    B, d, P = 24, 64, 8
    rng = np.random.default_rng(T)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).pack(z, y)
    for flag in (0, 1):
        ref = O.simulate_alg_batch(z, y, flag, SQ2, nthreads=4)
        out = {}
        for spec in ("0", "1"):
            monkeypatch.setenv("OCX_PIPE_SPEC", spec)
            r = db.simulate_alg(flag, SQ2, closed_comparator=True)
            torch.cuda.synchronize()
            out[spec] = (r[:B].cpu().numpy().copy(), db.cum[:B].cpu().numpy().copy())
        assert np.array_equal(out["0"][0], out["1"][0]) and np.array_equal(out["0"][1], out["1"][1])
        assert close(out["1"][1], ref[1]), (T, flag)
        assert close_closed(out["1"][0], ref[0], T), (T, flag)

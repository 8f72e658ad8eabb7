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
          (32, 1024), (64, 1024)]


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


@pytest.mark.parametrize("P", [8, 16, 32, 64])
def test_pipe_kernel_exact_on_single_coordinate_rows(eng, P):
    """Flip / switching rows (one nonzero coordinate): exact ties q = y survive the
    pipelined step — regrets bit-identical to the reference's."""
    d = {8: 64, 16: 64, 32: 128, 64: 1024}[P]
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


@pytest.mark.parametrize("P,d,T,chunk", [(8, 64, 300, 64), (16, 64, 257, 128), (8, 128, 640, 192),
                                         (32, 1024, 200, 64), (16, 512, 129, 64),
                                         (64, 1024, 300, 128)])
def test_chunked_pipe_is_bit_identical(eng, P, d, T, chunk):
    """The pipelined kernel run in launches of `chunk` steps, its state carried through HBM
    (the trailing pipeline's FTRL side, ocx_test_alg_pipe_chunked), against one launch:
    bit-identical regrets for every sequence the closed form certifies; NaN and the bad flag
    for the sequences it cannot (a row outside the ball, labels other than ±1), which a
    chunked run cannot stream a second pass for."""
    import ctypes
    import torch
    from online_convex_optimization_amd import _lib
    B = 70
    rng = np.random.default_rng(P + d + T)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    z[3, T // 2] *= 1.7
    y[40, ::9] = 0.5
    packed = eng.DeviceBatch(B, T, d, lanes_per_seq=P).pack(z, y)
    gen = eng.DeviceBatch(3 * 64 // P + 5, T, d, lanes_per_seq=P).generate_gT(7)
    for db, unclean in ((packed, [3, 40]), (gen, [])):
        assert (db.L.P, db.L.chain) == (P, 0)
        n = db.L.B
        whole = db.simulate_alg(0, SQ2, closed_comparator=True).clone()
        got = torch.zeros(n, dtype=torch.float64, device=db.device)
        bad = torch.zeros(1, dtype=torch.int32, device=db.device)
        _lib.call("ocx_test_alg_pipe_chunked", ctypes.byref(db.L), db.z.data_ptr(),
                  db.y.data_ptr(), SQ2, chunk, got.data_ptr(), bad.data_ptr(),
                  db.stream.cuda_stream)
        torch.cuda.synchronize()
        w, g = whole[:n].cpu().numpy(), got.cpu().numpy()
        ok = np.ones(n, dtype=bool)
        ok[unclean] = False
        assert np.array_equal(g[ok], w[ok]), (P, d, T, chunk)
        assert np.all(np.isnan(g[~ok]))
        assert int(bad.item()) == (1 if unclean else 0)

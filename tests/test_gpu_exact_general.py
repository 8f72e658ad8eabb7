"""The general exact-FTL solver on the GPU (ocx_exact_ball.hip; include/ocx.h
ocx_exact_ball_solve): ExactFTLNoClip's problem (exact_ftl.py:83-105) for rows and labels
outside the closed forms' regime, e.g. the linf ball on the reference's own rows.

The reference solves it with cvxpy (absent here), so parity is UNPINNED; the mathematics is
pinned by independent solvers — scipy HiGHS on the l1 / linf LPs, SLSQP on the l2 SOCP —
and by the certificate the kernel returns (obj − gap is a dual bound: never above the
optimum).  Tolerances: objective within 1e-8·(1+f) of HiGHS (the barrier stops at μ = 1e-10;
cvxpy's own default tolerances are ≈1e-8), actions within 1e-6 where the LP minimiser is
unique."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests._scipy_solvers import lp_solve, objective, socp_solve

pytestmark = pytest.mark.gpu
SQ2 = math.sqrt(2.0)
NORM_CODES = {"l2": 0, "l1": 1, "linf": 2}


@pytest.fixture(scope="module")
def eng():
    from online_convex_optimization_amd import _lib, engine
    _lib.load()
    return engine


def _norm_of(x, norm):
    return {"l2": np.linalg.norm(x), "l1": np.abs(x).sum(), "linf": np.abs(x).max()}[norm]


def _data(seed, B, T, d, *, clip=True, labels="pm1"):
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((B, T, d))
    if clip:
        z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = (np.where(rng.random((B, T)) < 0.5, -1.0, 1.0) if labels == "pm1"
         else rng.standard_normal((B, T)))
    return z, y


def _check_certificate(res, ref_f, b, n, gap_rtol=1e-8):
    f = res["obj"][b, n]
    gap = res["gap"][b, n]
    assert 0.0 <= gap < gap_rtol * (1.0 + f), (b, n, gap)
    assert f - gap <= ref_f + 1e-9 * (1.0 + ref_f), (b, n)     # a valid dual bound
    assert res["info"][b, n] > 0, (b, n, res["info"][b, n])    # converged, not capped


@pytest.mark.parametrize("norm", ["linf", "l1"])
@pytest.mark.parametrize("d,clip,labels", [(5, True, "pm1"), (2, False, "pm1"), (8, True, "real"),
                                           (10, False, "real"), (10, True, "pm1")])
def test_general_lp_matches_highs(eng, norm, d, clip, labels):
    B, T = 3, 40
    z, y = _data(11 * d + (norm == "l1"), B, T, d, clip=clip, labels=labels)
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    assert res["actions"].shape == (B, T + 1, d)
    for b in range(B):
        assert np.all(res["actions"][b, 0] == 0.0)              # the empty prefix: x = 0
        for n in (1, 2, 3, d // 2, d, d + 1, T // 2, T):
            x_lp, f_lp = lp_solve(z[b, :n], y[b, :n], norm)
            x = res["actions"][b, n]
            f = res["obj"][b, n]
            assert _norm_of(x, norm) <= 1.0 + 1e-12
            assert abs(objective(z[b, :n], y[b, :n], x) - f) <= 1e-12 * (1.0 + f)
            assert abs(f - f_lp) <= 1e-8 * (1.0 + f_lp), (b, n, f, f_lp)
            _check_certificate(res, f_lp, b, n)
        # FTL's step losses are those of the prefix actions (replay_exact_ftl :318-323)
        for n in (0, 3, T - 1):
            q = 0.0
            for j in range(d):
                q = q + z[b, n, j] * res["actions"][b, n, j]
            assert res["step_loss"][b, n] == 0.5 * abs(q - y[b, n])
        assert res["step_loss"][b, T] == 0.0


def test_general_lp_actions_where_unique(eng):
    """n >= d generic rows: the LP minimiser is a unique vertex, and the barrier's limit is
    that vertex."""
    z, y = _data(3, 4, 60, 5, clip=True)
    for norm in ("linf", "l1"):
        res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=False)
        assert res["actions"].shape == (4, 1, 5)
        for b in range(4):
            x_lp, f_lp = lp_solve(z[b], y[b], norm)
            assert np.allclose(res["actions"][b, 0], x_lp, atol=1e-6), (norm, b)
            assert abs(res["obj"][b, 0] - f_lp) <= 1e-8 * (1.0 + f_lp)


@pytest.mark.parametrize("d,clip", [(3, False), (5, False), (7, True)])
def test_general_l2_vs_slsqp(eng, d, clip):
    B, T = 2, 30
    z, y = _data(40 + d, B, T, d, clip=clip, labels="real" if clip else "pm1")
    if clip:
        z *= 2.5                                                  # rows outside the ball
    res = eng.exact_ball_solve(z, y, norm="l2")
    for b in range(B):
        for n in (2, T // 2, T):
            x_s, f_s = socp_solve(z[b, :n], y[b, :n])
            f = res["obj"][b, n]
            assert np.linalg.norm(res["actions"][b, n]) <= 1.0 + 1e-12
            assert f <= f_s + 1e-9 * (1.0 + f_s), (b, n)          # no worse than SLSQP
            assert f_s - f < 1e-5 * (1.0 + f), (b, n)
            _check_certificate(res, f_s, b, n)


@pytest.mark.parametrize("norm", ["l2", "l1"])
def test_general_agrees_with_closed_form_in_regime(eng, norm):
    """On the reference's data (clipped rows, ±1 labels) the closed forms are exact; the
    general solver must land on the same minimisers."""
    B, T, d = 4, 80, 5
    z = np.stack([O.gT_sample(0, T, r, d)[0] for r in range(B)])
    y = np.stack([O.gT_sample(0, T, r, d)[1] for r in range(B)])
    closed, ok = eng.ftl_prefix_actions_batch(z, y, norm=norm, check_regime=False)
    assert ok.all()
    res = eng.exact_ball_solve(z, y, norm=norm)
    for b in range(B):
        for n in range(1, T + 1, 7):
            fc = objective(z[b, :n], y[b, :n], closed[b, n])
            assert abs(res["obj"][b, n] - fc) <= 1e-8 * (1.0 + fc), (b, n)
            S = (y[b, :n, None] * z[b, :n]).sum(axis=0)
            unique = (np.linalg.norm(S) > 1e-6 if norm == "l2" else
                      np.sort(np.abs(S))[-1] - np.sort(np.abs(S))[-2] > 1e-6)
            if unique:
                assert np.allclose(res["actions"][b, n], closed[b, n], atol=1e-6), (b, n)


def test_tiled_equals_row_major(eng):
    """DeviceBatch.exact_general (tiled input) is the same computation as the row-major
    entry point: bit-identical outputs."""
    import torch
    B, T, d = 70, 33, 4
    z, y = _data(5, B, T, d, clip=False)
    ref = eng.exact_ball_solve(z, y, norm="linf")
    for lanes in (1, eng.LANES_BEST, 4):
        db = eng.DeviceBatch(B, T, d, lanes_per_seq=lanes).pack(z, y)
        g = db.exact_general("linf")
        torch.cuda.synchronize()
        for k in ("actions", "obj", "gap", "step_loss", "info"):
            assert np.array_equal(g[k][:B].cpu().numpy(), ref[k]), (lanes, k)


def test_dropin_out_of_regime(eng):
    """The exact_ftl.py drop-in now answers outside the regime (it used to raise):
    compute_prefix_actions / run_ftl_exact / run_ftrl over the linf ball on the
    reference's rows, and unclipped rows under l2."""
    from online_convex_optimization_amd import exact_ftl as ef
    z, y, _ = O.random_iid_sample(2025, 50, 0)
    for zz, yy, norm in ((z, y, "linf"), (3.0 * z, y, "l2"), (z, 0.5 * y, "l1")):
        s = ef.ExactFTLNoClip(5, 50, norm=norm)
        acts = ef.compute_prefix_actions(s, zz, yy)
        res = eng.exact_ball_solve(zz[None], yy[None], norm=norm)
        assert np.array_equal(acts, res["actions"][0])
        x_t = s.solve_prefix_from_full(zz, yy, 50)
        assert np.array_equal(x_t, acts[-1])
        r = ef.run_ftl_exact(zz, yy, norm=norm)
        rep = ef.replay_exact_ftl(zz, yy, acts)
        assert abs(r.cum_loss - rep.cum_loss) <= 1e-12 * (1.0 + rep.cum_loss)
        assert abs(r.comp_loss - rep.comp_loss) <= 1e-12 * (1.0 + rep.comp_loss)
        if norm != "l2":
            _, f_lp = lp_solve(zz, yy, norm)
            assert abs(rep.comp_loss - f_lp) <= 1e-8 * (1.0 + f_lp)
        rf = ef.run_ftrl(zz, yy, eta0=SQ2, norm=norm)
        assert abs(rf.comp_loss - rep.comp_loss) <= 1e-12 * (1.0 + rep.comp_loss)


def test_batch_entry_points_fill_out_of_regime(eng):
    B, T, d = 6, 45, 5
    z, y = _data(8, B, T, d, clip=True)
    z[::2] *= 2.0                      # half the batch leaves the l2 regime
    r = eng.ftrl_vs_exact_batch(z, y, SQ2, norm="l2")
    assert list(r["in_regime"]) == [False, True] * 3
    g = eng.exact_ball_solve(z[::2], y[::2], norm="l2")
    cum = np.cumsum(g["step_loss"][:, :T], axis=1)[:, -1]
    assert np.array_equal(r["cum_exact"][::2], cum)
    assert np.array_equal(r["comp"][::2], g["obj"][:, T])
    assert np.array_equal(r["action"][::2], g["actions"][:, T])
    c, p, a, ok = eng.ftl_exact_batch(z, y, norm="l2")
    assert np.array_equal(c[::2], cum) and np.array_equal(a[::2], g["actions"][:, T])
    acts, ok2 = eng.ftl_prefix_actions_batch(z, y, norm="l2")
    assert np.array_equal(acts[::2], g["actions"]) and np.array_equal(ok, ok2)
    # FTRL's side does not depend on the comparator's regime
    ref = eng.ftrl_vs_exact_batch(z, y, SQ2, norm="l2", check_regime=False)
    assert np.array_equal(r["cum_ftrl"], ref["cum_ftrl"])


def test_device_batch_general_matches_host(eng):
    import torch
    B, T, d = 9, 60, 5
    z, y = _data(12, B, T, d, clip=True)
    host = eng.ftrl_vs_exact_batch(z, y, SQ2, norm="linf", lanes_per_seq=1)
    assert not host["in_regime"].any()
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=1).pack(z, y)
    reg = db.ftrl_vs_exact_general(SQ2, norm="linf")
    torch.cuda.synchronize()
    assert not reg[:B].bool().any().item()
    assert np.allclose(db.cum_exact[:B].cpu().numpy(), host["cum_exact"], rtol=1e-13, atol=1e-12)
    assert np.array_equal(db.comp[:B].cpu().numpy(), host["comp"])
    assert np.array_equal(db.cum[:B].cpu().numpy(), host["cum_ftrl"])


def test_exact_driver_linf(eng):
    """exact_ftl_driver.py with ExperimentConfig(norm='linf') (:46): every sequence of the
    families leaves the linf closed form's regime and goes through the general solver."""
    from online_convex_optimization_amd import drivers
    r = drivers.exact_case_regrets("Random i.i.d. (separable)", 60, runs=2, replicates=2,
                                   norm="linf")
    assert r["FTRL"].shape == (4,) and np.all(np.isfinite(r["FTL (exact)"]))
    assert np.all(np.isfinite(r["FTRL"]))


def test_general_limits_are_loud(eng):
    z, y = _data(1, 2, 10, 257, clip=False)
    with pytest.raises(NotImplementedError):
        eng.exact_ball_solve(z, y, norm="linf")
    with pytest.raises(NotImplementedError):
        eng.ftl_exact_batch(z, y, norm="linf")
    with pytest.raises(ValueError):
        eng.exact_ball_solve(z[..., :3], y, norm="l3")


# ---- 10 < d <= 64: the LDS-resident system (ocx_exact_wide.hip) -------------------------
@pytest.mark.parametrize("norm", ["linf", "l1"])
@pytest.mark.parametrize("d,T,clip,labels", [(16, 40, True, "pm1"), (16, 30, False, "real"),
                                             (64, 80, True, "pm1"), (33, 50, False, "pm1")])
def test_wide_lp_matches_highs(eng, norm, d, T, clip, labels):
    """configs[2]'s d = 64 (and 16, 33) outside the closed forms: the linf ball on the
    reference's clipped rows, unclipped rows, real labels — against HiGHS, with the
    certificate.  Parity with cvxpy: unpinned."""
    B = 2
    z, y = _data(7 * d + (norm == "l1"), B, T, d, clip=clip, labels=labels)
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    assert res["actions"].shape == (B, T + 1, d)
    for b in range(B):
        assert np.all(res["actions"][b, 0] == 0.0)
        for n in (1, 2, d // 2, d, d + 1, T):
            x_lp, f_lp = lp_solve(z[b, :n], y[b, :n], norm)
            x = res["actions"][b, n]
            f = res["obj"][b, n]
            assert _norm_of(x, norm) <= 1.0 + 1e-12
            assert abs(objective(z[b, :n], y[b, :n], x) - f) <= 1e-11 * (1.0 + f)
            assert abs(f - f_lp) <= 1e-7 * (1.0 + f_lp), (b, n, f, f_lp)
            _check_certificate(res, f_lp, b, n, gap_rtol=1e-8)
        for n in (0, d, T - 1):
            q = 0.0
            for j in range(d):
                q = q + z[b, n, j] * res["actions"][b, n, j]
            assert res["step_loss"][b, n] == 0.5 * abs(q - y[b, n])


@pytest.mark.parametrize("d", [16, 40])
def test_wide_l2_vs_slsqp(eng, d):
    B, T = 2, 30
    z, y = _data(90 + d, B, T, d, clip=True, labels="real")
    z *= 2.5                                                      # rows outside the ball
    res = eng.exact_ball_solve(z, y, norm="l2")
    for b in range(B):
        for n in (2, T // 2, T):
            x_s, f_s = socp_solve(z[b, :n], y[b, :n])
            f = res["obj"][b, n]
            assert np.linalg.norm(res["actions"][b, n]) <= 1.0 + 1e-12
            assert f <= f_s + 1e-9 * (1.0 + f_s), (b, n)          # no worse than SLSQP
            _check_certificate(res, f_s, b, n, gap_rtol=1e-8)


def test_wide_tiled_and_engine_paths(eng):
    """d = 64: the tiled entry point equals the row-major one bit for bit, and the batched
    FTRL-vs-exact paths (host arrays and DeviceBatch.ftrl_vs_exact_general, which now solves
    only the sequences outside the regime) agree, with every solve certified."""
    import torch
    B, T, d = 10, 40, 64
    z, y = _data(21, B, T, d, clip=True)
    ref = eng.exact_ball_solve(z, y, norm="linf")
    db = eng.DeviceBatch(B, T, d).pack(z, y)
    g = db.exact_general("linf")
    torch.cuda.synchronize()
    for k in ("actions", "obj", "gap", "step_loss", "info"):
        assert np.array_equal(g[k][:B].cpu().numpy(), ref[k]), k
    host = eng.ftrl_vs_exact_batch(z, y, SQ2, norm="linf")
    assert not host["in_regime"].any() and host["exact_gap_max"] < 1e-7
    want_cum = np.cumsum(ref["step_loss"][:, :T], axis=1)[:, -1]
    assert np.array_equal(host["cum_exact"], want_cum)
    assert np.array_equal(host["comp"], ref["obj"][:, T])
    db2 = eng.DeviceBatch(B, T, d).pack(z, y)
    rg = db2.ftrl_vs_exact_general(SQ2, norm="linf")
    torch.cuda.synchronize()
    assert not rg[:B].cpu().numpy().any()
    assert np.array_equal(db2.cum_exact[:B].cpu().numpy(), want_cum)
    assert np.array_equal(db2.comp[:B].cpu().numpy(), ref["obj"][:, T])
    assert db2.exact_gap_max < 1e-7


def test_uncertified_solve_raises(eng, monkeypatch):
    """A solve whose certificate is not within the tolerance makes every engine path raise
    RuntimeError (exact_ftl.py:125-126 raises on a solver failure) instead of returning it."""
    from online_convex_optimization_amd import engine as E
    z, y = _data(4, 2, 20, 5, clip=False)
    monkeypatch.setattr(E, "EXACT_GAP_RTOL", -1.0)  # no gap passes
    with pytest.raises(RuntimeError, match="did not certify"):
        E.ftl_exact_batch(z, y, norm="linf")


@pytest.mark.parametrize("norm", ["l1", "linf"])
def test_tied_prefixes_take_the_general_solvers_centre(eng, norm):
    """Constructed ties (exact_ftl.py:119-128 leaves the choice to cvxpy): rows alternating
    e_1, e_2 with +1 labels make |S_1| = |S_2| at every even prefix (l1), and a coordinate
    touched by rows of both signs returns to S_j = 0 (linf).  The closed form would play the
    first coordinate / 0 there; such sequences now leave the closed form's regime and the
    engine answers with the general solver — the analytic centre of the optimal face, the
    interior-point limit — so the batched closed-form path and the general solver give the
    same actions, at the LP optimum."""
    T, d = 24, 5
    z = np.zeros((2, T, d))
    y = np.ones((2, T))
    z[0, 0::2, 0] = 1.0
    z[0, 1::2, 1] = 1.0
    z[1, :, 2] = 0.5                       # a sequence without ties: stays closed form
    z[1, :, 3] = 0.25
    if norm == "linf":
        z[0, 1::2, 1] = 0.0
        z[0, :, 0] = 0.5
        y[0, 1::2] = -1.0                  # S_1 returns to 0 every second step
    raw, ok_raw = eng.ftl_prefix_actions_batch(z, y, norm=norm, check_regime=False)
    assert list(ok_raw) == [False, True]
    acts, ok = eng.ftl_prefix_actions_batch(z, y, norm=norm)
    gen = eng.exact_ball_solve(z[:1], y[:1], norm=norm)
    assert np.array_equal(acts[0], gen["actions"][0])        # the general solver's answer
    assert np.array_equal(acts[1], raw[1])                   # untied: the closed form
    for n in range(1, T + 1):
        _, f_lp = lp_solve(z[0, :n], y[0, :n], norm)
        assert abs(objective(z[0, :n], y[0, :n], acts[0, n]) - f_lp) <= 1e-8 * (1.0 + f_lp)
    cum, comp, act, in_regime = eng.ftl_exact_batch(z, y, norm=norm)
    assert list(in_regime) == [False, True]
    assert np.array_equal(act[0], gen["actions"][0, T])


@pytest.mark.parametrize("norm", ["linf", "l1", "l2"])
@pytest.mark.parametrize("d", [5, 11, 33, 64])
def test_interpolating_optimum_certifies(eng, norm, d):
    """n > d unclipped rows (3·N(0,1)) with real-valued labels: the optimum interpolates rows
    exactly (a vertex of the LAD fit; at d = 64 inside the ball it interpolates 64 rows, the
    most the polish's active set holds), where the barrier's multipliers of those rows are only
    as good as μ_end (their certificate stayed near 1e-5 relative).  The polished dual
    (ocx_exact_polish_kernel: ±½ on the other rows, least squares on stationarity for the
    interpolated ones) certifies every prefix to 1e-8·(1 + obj), and it is a valid bound."""
    B, T = 2, 3 * d + 20
    rng = np.random.default_rng(1000 + d + NORM_CODES[norm])
    z = 3.0 * rng.standard_normal((B, T, d))
    y = rng.standard_normal((B, T))
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    assert np.all(res["info"][:, 1:] > 0)
    ok = res["gap"] <= 1e-8 * (1.0 + np.abs(res["obj"]))
    assert ok.all(), (np.argwhere(~ok)[:5], res["gap"][~ok][:5])
    assert eng.check_certificates(res["obj"], res["gap"], res["info"]) <= 1e-8 * (1.0 + res["obj"].max())
    for b in range(B):
        for n in (d + 1, 2 * d, T):
            if norm == "l2":
                _, f_ref = socp_solve(z[b, :n], y[b, :n])
                assert res["obj"][b, n] <= f_ref + 1e-9 * (1.0 + f_ref)
            else:
                _, f_ref = lp_solve(z[b, :n], y[b, :n], norm)
                assert abs(res["obj"][b, n] - f_ref) <= 1e-8 * (1.0 + f_ref), (b, n)
            assert res["obj"][b, n] - res["gap"][b, n] <= f_ref + 1e-9 * (1.0 + f_ref)


# ---- 64 < d <= 256: the system in HBM scratch (ocx_exact_big.hip) -------------------------
@pytest.mark.parametrize("norm", ["linf", "l1"])
@pytest.mark.parametrize("d,T,clip,labels,prefixes", [(100, 130, True, "pm1", True),
                                                      (65, 80, False, "real", True),
                                                      (256, 300, True, "pm1", False),
                                                      (256, 60, False, "real", False)])
def test_big_lp_matches_highs(eng, norm, d, T, clip, labels, prefixes):
    """d in {65, 100, 256}: the linf / l1 balls against HiGHS with the certificate, all
    prefixes where the batch is small (the reference's cvxpy has no dimension limit,
    exact_ftl.py:119-128).  Parity with cvxpy: unpinned."""
    B = 2
    z, y = _data(5 * d + (norm == "l1"), B, T, d, clip=clip, labels=labels)
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=prefixes)
    NP = T + 1 if prefixes else 1
    assert res["actions"].shape == (B, NP, d)
    # every problem (every prefix) finished and certifies to 1e-8 (engine.check_certificates)
    assert eng.check_certificates(res["obj"], res["gap"], res["info"]) <= 1e-8 * (1.0 + res["obj"].max())
    ns = [n for n in (1, 2, d // 2, d, d + 1, T) if n <= T] if prefixes else [T]
    for b in range(B):
        if prefixes:
            assert np.all(res["actions"][b, 0] == 0.0)
        for n in ns:
            k = n if prefixes else 0
            x_lp, f_lp = lp_solve(z[b, :n], y[b, :n], norm)
            x = res["actions"][b, k]
            f = res["obj"][b, k]
            assert _norm_of(x, norm) <= 1.0 + 1e-12
            assert abs(objective(z[b, :n], y[b, :n], x) - f) <= 1e-11 * (1.0 + f)
            assert abs(f - f_lp) <= 1e-7 * (1.0 + f_lp), (b, n, f, f_lp)
            _check_certificate(res, f_lp, b, k, gap_rtol=1e-8)
        if prefixes:
            for n in (0, d // 2, T - 1):
                q = 0.0
                for j in range(d):
                    q = q + z[b, n, j] * res["actions"][b, n, j]
                assert res["step_loss"][b, n] == 0.5 * abs(q - y[b, n])


@pytest.mark.parametrize("d", [100, 256])
def test_big_l2_vs_slsqp(eng, d):
    B, T = 2, 40
    z, y = _data(190 + d, B, T, d, clip=True, labels="real")
    z *= 2.5                                                      # rows outside the ball
    res = eng.exact_ball_solve(z, y, norm="l2", all_prefixes=False)
    for b in range(B):
        x_s, f_s = socp_solve(z[b], y[b])
        f = res["obj"][b, 0]
        assert np.linalg.norm(res["actions"][b, 0]) <= 1.0 + 1e-12
        assert f <= f_s + 1e-9 * (1.0 + f_s), b                   # no worse than SLSQP
        _check_certificate(res, f_s, b, 0, gap_rtol=1e-8)


@pytest.mark.parametrize("norm", ["linf", "l1", "l2"])
def test_big_interpolating_optimum_certifies(eng, norm):
    """n > d = 100 unclipped rows with real labels: the optimum interpolates up to 100 rows,
    which the polish's active set (DP = 128 rows) holds; every prefix's certificate passes."""
    d, T, B = 100, 140, 1
    rng = np.random.default_rng(2000 + NORM_CODES[norm])
    z = 3.0 * rng.standard_normal((B, T, d))
    y = rng.standard_normal((B, T))
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    assert np.all(res["info"][:, 1:] > 0)
    assert eng.check_certificates(res["obj"], res["gap"], res["info"]) <= 1e-8 * (1.0 + res["obj"].max())
    for n in (d + 1, T):
        if norm == "l2":
            _, f_ref = socp_solve(z[0, :n], y[0, :n])
            assert res["obj"][0, n] <= f_ref + 1e-9 * (1.0 + f_ref)
        else:
            _, f_ref = lp_solve(z[0, :n], y[0, :n], norm)
            assert abs(res["obj"][0, n] - f_ref) <= 1e-8 * (1.0 + f_ref), n
        assert res["obj"][0, n] - res["gap"][0, n] <= f_ref + 1e-9 * (1.0 + f_ref)


def test_big_tiled_and_engine_paths(eng):
    """d = 100: the tiled entry point equals the row-major one bit for bit, and the batched
    FTRL-vs-exact path answers out of the regime with every solve certified."""
    import torch
    B, T, d = 3, 50, 100
    z, y = _data(31, B, T, d, clip=True)
    ref = eng.exact_ball_solve(z, y, norm="linf")
    db = eng.DeviceBatch(B, T, d).pack(z, y)
    g = db.exact_general("linf")
    torch.cuda.synchronize()
    for k in ("actions", "obj", "gap", "step_loss", "info"):
        assert np.array_equal(g[k][:B].cpu().numpy(), ref[k]), k
    host = eng.ftrl_vs_exact_batch(z, y, SQ2, norm="linf")
    assert not host["in_regime"].any() and host["exact_gap_max"] < 1e-7
    assert np.array_equal(host["cum_exact"], np.cumsum(ref["step_loss"][:, :T], axis=1)[:, -1])
    assert np.array_equal(host["comp"], ref["obj"][:, T])


@pytest.mark.parametrize("d,B,T,norm", [(70, 5, 110, "linf"), (150, 3, 100, "l1")])
def test_big_persistent_blocks_reuse_scratch(eng, d, B, T, norm):
    """More problems than resident blocks (512 at DP = 128, 256 at DP = 256): each block solves
    several problems in turn in the same scratch matrices, and every answer is the one the
    problem gets alone (a one-sequence call), bit for bit, and certified."""
    z, y = _data(77 + d, B, T, d, clip=False, labels="real")
    res = eng.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
    assert B * (T + 1) > (512 if d <= 128 else 256)
    eng.check_certificates(res["obj"], res["gap"], res["info"])
    for b in (0, B - 1):
        one = eng.exact_ball_solve(z[b:b + 1], y[b:b + 1], norm=norm, all_prefixes=True)
        for k in ("actions", "obj", "gap", "step_loss", "info"):
            assert np.array_equal(res[k][b], one[k][0]), (b, k)
    for n in (d // 2, T):
        _, f_lp = lp_solve(z[0, :n], y[0, :n], norm)
        assert abs(res["obj"][0, n] - f_lp) <= 1e-8 * (1.0 + f_lp), n


@pytest.mark.parametrize("norm", ["linf", "l1", "l2"])
def test_big_degenerate_inputs(eng, norm):
    """d = 100 edge cases: the empty horizon (T = 0: the empty prefix only, x = 0), all-zero rows
    with ±1 labels (every x is optimal at ½Σ|y|; the path's centre is x = 0) and zero labels
    (optimum 0 at x = 0) — every answer certified, as the d ≤ 64 kernels'."""
    d = 100
    res = eng.exact_ball_solve(np.zeros((2, 0, d)), np.zeros((2, 0)), norm=norm)
    assert res["actions"].shape == (2, 1, d) and np.all(res["actions"] == 0.0)
    assert np.all(res["obj"] == 0.0) and np.all(res["info"] == 0)
    T = 12
    y = np.where(np.arange(T) % 3 == 0, -1.0, 1.0)[None].repeat(2, axis=0)
    res = eng.exact_ball_solve(np.zeros((2, T, d)), y, norm=norm)
    eng.check_certificates(res["obj"], res["gap"], res["info"])
    assert np.allclose(res["obj"][:, T], T / 2, rtol=0, atol=1e-12)
    assert np.abs(res["actions"]).max() <= 1e-9
    z, _ = _data(61, 2, T, d, clip=False)
    res = eng.exact_ball_solve(z, np.zeros((2, T)), norm=norm)
    eng.check_certificates(res["obj"], res["gap"], res["info"])
    assert res["obj"].max() <= 1e-8

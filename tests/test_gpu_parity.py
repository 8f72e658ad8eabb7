"""GPU parity: the HIP kernels (through the C ABI) against the golden fixtures and the
CPU oracle.  Bars: bit-exact in exact mode (lanes_per_seq=1) and for the
tie-sensitive deterministic families; |Δ| <= 1e-12·max(1, |ref|) for split-lane modes
(the north star's bar is 1e-6 relative)."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests._golden import F
from tests._tiles import untile_y, untile_z

pytestmark = pytest.mark.gpu

SQ2 = math.sqrt(2)
PUBLISHED_GT = [6.034165981694009, 8.297032923590692, 10.446825985542404, 12.032218781087039,
                13.383600324774818, 14.946774913365687, 15.951320592930585, 17.196625822976216,
                18.087283038366593, 19.088517830594924]
TOL = 1e-12


@pytest.fixture(scope="module")
def ocx():
    from online_convex_optimization_amd import _lib, engine, exact_ftl, fast_algorithms
    assert _lib.device_count() >= 1
    return {"lib": _lib, "engine": engine, "fa": fast_algorithms, "ef": exact_ftl}


def close(a, b, tol=TOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


def close_closed(a, b, T):
    """Bar for the closed-form comparator (T/2 - ||theta_T||, OCX_ALG_CLIPPED_ROWS) against
    the reference's sequential sum of T terms: that sum's own rounding error grows like
    eps*T^1.5 (measured 3.3e-11 absolute, 7e-13 relative to the regret, at T = 1e4), so
    |diff| <= max(1e-12 * max(1, |ref|), 4 eps T^1.5).  North star: 1e-6 relative."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    tol = np.maximum(TOL * np.maximum(1.0, np.abs(b)), 4 * 2.22e-16 * float(T) ** 1.5)
    return np.all(np.abs(a - b) <= tol)


# ------------------------------------------------------------------ golden vectors
def test_simulate_alg_golden_bitexact(ocx, golden):
    fa = ocx["fa"]
    for name, z, y, rec in golden.explicit():
        for key, h in rec["alg"].items():
            flag, eta_h = key.split("_")
            got = fa.simulate_alg(z, y, int(flag), float.fromhex(eta_h))
            assert got == F(h), (name, key, got, F(h))


def test_smart_golden_bitexact(ocx, golden):
    fa = ocx["fa"]
    for name, z, y, rec in golden.explicit():
        if z.shape[0] > 600:
            continue  # O(T^2) prefix scans: keep the suite short
        for th_h, h in rec["smart"].items():
            got = fa.simulate_SMART_like(z, y, float.fromhex(th_h), SQ2)
            assert got == F(h), (name, th_h, got, F(h))
        assert fa.simulate_SMART(z, y) == F(rec["smart_default"])


def test_exact_ftl_golden(ocx, golden):
    ef = ocx["ef"]
    for name, z, y, rec in golden.explicit():
        if "run_ftrl" not in rec:
            continue
        a = golden.arr(f"{name}__comparator")
        rr = ef.run_ftrl(z, y, eta0=1.0, comparator_action=a)
        r = rec["run_ftrl"]
        assert rr.cum_loss == F(r["cum_loss"]), name
        assert np.array_equal(rr.x_last, np.array([F(v) for v in r["x_last"]])), name
        # comparator loss in the reference's order (dgemv_t rows, NumPy pairwise sum)
        assert rr.comp_loss == F(r["comp_loss"]), name
        assert rr.regret == F(r["regret"]), name
        acts = golden.arr(f"{name}__actions")
        rp = ef.replay_exact_ftl(z, y, acts)
        assert rp.cum_loss == F(rec["replay"]["cum_loss"]), name
        assert rp.comp_loss == F(rec["replay"]["comp_loss"]), name
        assert rp.regret == F(rec["replay"]["regret"]), name


def test_families_exact_ties(ocx, golden):
    fa = ocx["fa"]
    g_pub = dict(zip(range(100, 1100, 100), PUBLISHED_GT))
    for title, fn in (("Label flips", O.flip_sequence),
                      ("Switching leaders", O.switching_two_leaders_sequence)):
        for T_s, row in golden.j["families"][title].items():
            z, y, _ = fn(int(T_s))
            assert fa.simulate_alg(z, y, 0, SQ2) == F(row["FTRL"])
            assert fa.simulate_alg(z, y, 1, SQ2) == F(row["FTL"])
            assert fa.simulate_SMART(z, y) == F(row["SMART"])
            assert fa.simulate_empirical_g_SMART(z, y, g_pub[int(T_s)]) == F(row["EMP"])


def test_families_all_lane_splits_exact(ocx):
    """Single-nonzero-coordinate rows make every reduction exact: any lane split must
    reproduce the tie-sensitive trajectories bit-for-bit."""
    eng = ocx["engine"]
    for fn in (O.flip_sequence, O.switching_two_leaders_sequence):
        z, y, _ = fn(1000, d=64)
        ref = [O.simulate_alg(z, y, f, SQ2) for f in (0, 1)]
        Z = np.repeat(z[None].astype(np.float64), 3, axis=0)
        Y = np.repeat(y[None].astype(np.float64), 3, axis=0)
        for P in (1, -1, -8, 2, 4, 8, 16, 32, 64):
            for f in (0, 1):
                got = eng.simulate_alg_batch(Z, Y, f, SQ2, lanes_per_seq=P)
                assert np.all(got == ref[f]), (P, f, got, ref[f])


def test_seeded_gT_golden(ocx, golden):
    eng = ocx["engine"]
    by = {}
    for rec in golden.j["seeded_gT"]:
        by.setdefault((rec["base_seed"], rec["T"]), []).append(rec)
    for (seed, T), recs in by.items():
        runs = max(r["run"] for r in recs) + 1
        for P in (1, -1, -2, 0):
            got = eng.gT_regrets(T, runs, base_seed=seed, d=5, lanes_per_seq=P)
            for r in recs:
                if P != 0:
                    assert got[r["run"]] == F(r["regret"]), (seed, T, r["run"])
                else:
                    assert close(got[r["run"]], F(r["regret"])), (seed, T, r["run"])


def test_gT_small_sweep_golden(ocx, golden):
    fa = ocx["fa"]
    s = golden.j["gT_small"]
    g = fa.empirical_worst_case_thresholds(np.array(s["T_grid"]), runs=s["runs"],
                                           base_seed=s["base_seed"])
    assert {k: v for k, v in g.items()} == {int(k): F(v) for k, v in s["g"].items()}


def test_published_gT_curve(ocx):
    """End-to-end KAT: fast_driver.py's g(T) sweep (T=100..1000, runs=1000, d=5) ==
    the values behind the reference's published empirical_g_T_fast.png."""
    fa = ocx["fa"]
    g = fa.empirical_worst_case_thresholds(np.arange(100, 1100, 100), runs=1000)
    assert [g[T] for T in range(100, 1100, 100)] == PUBLISHED_GT


# ------------------------------------------------------------------ generator
@pytest.mark.parametrize("B,T,d,P", [(70, 50, 5, 1), (33, 20, 64, 4), (5, 8, 1024, 64),
                                     (40, 9, 129, 0), (3, 11, 2, 0), (9, 6, 64, -1),
                                     (17, 7, 100, -2), (192, 2000, 64, 1), (6, 40, 1024, 1),
                                     (4, 10, 1024, 0), (3, 5, 1024, -16), (70, 3, 1024, -32),
                                     (130, 301, 16, 8), (37, 700, 16, 1), (50, 123, 32, 8),
                                     (9, 77, 32, -4), (21, 50, 16, -2), (37, 257, 16, 8),
                                     (19, 33, 32, 8), (11, 65, 16, 8)])
def test_device_generator_matches_numpy(ocx, B, T, d, P):
    import torch
    eng = ocx["engine"]
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).generate_gT(base_seed=0, run0=10)
    torch.cuda.synchronize()
    z = untile_z(db.z.cpu().numpy(), db.L)
    y = untile_y(db.y.cpu().numpy(), db.L)
    # (192, 2000, 64): ~6700 ziggurat tail draws → the device log1p must equal libm's
    for b in range(B):
        zr, yr = O.gT_sample(0, T, 10 + b, d)
        assert np.array_equal(z[b], zr), (b, int((z[b] != zr).sum()))
        assert np.array_equal(y[b], yr), b
    # padding (coordinates >= d, sequences >= B) is zero
    zt = db.z.cpu().numpy()
    assert np.count_nonzero(zt) <= B * T * d


@pytest.mark.parametrize("B,T", [(33, 20), (192, 2000), (5000, 40)])
def test_generator_forms_agree(ocx, monkeypatch, B, T):
    """The d = 64 generator's two forms (8-row batches / 4 waves per SIMD, and the
    low-LDS 7-row form at 6 waves; ocx_gen_wave.hip launch_wave picks by makespan) write
    the same tiles bit for bit, equal to NumPy's streams."""
    import torch
    eng = ocx["engine"]
    out = {}
    monkeypatch.setenv("OCX_GEN_ROUNDS", "0")  # one launch of the form (not the rounds path)
    for form in ("default", "lr"):
        monkeypatch.setenv("OCX_GEN_FORM", form)
        db = eng.DeviceBatch(B, T, 64, lanes_per_seq=1).generate_gT(base_seed=3, run0=1)
        torch.cuda.synchronize()
        out[form] = (db.z.cpu().numpy(), db.y.cpu().numpy(), db.L)
        del db
    assert np.array_equal(out["default"][0], out["lr"][0])
    assert np.array_equal(out["default"][1], out["lr"][1])
    z = untile_z(out["lr"][0], out["lr"][2])
    for b in (0, B // 2, B - 1):
        zr, yr = O.gT_sample(3, T, 1 + b, 64)
        assert np.array_equal(z[b], zr), b


# ------------------------------------------------------------------ batched, all splits
@pytest.mark.parametrize("T,d", [(300, 64), (200, 16), (50, 5), (40, 1024), (0, 7), (25, 1),
                                 (64, 100)])
def test_batch_all_lane_splits(ocx, T, d):
    eng = ocx["engine"]
    rng = np.random.default_rng(T * 1000 + d)
    B = 37
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    cmp = rng.standard_normal((B, d)) / max(1.0, math.sqrt(d))
    for flag, eta0 in ((0, SQ2), (1, SQ2), (0, 0.3)):
        ref = O.simulate_alg_batch(z, y, flag, eta0, nthreads=4)
        refc = O.simulate_alg_batch(z, y, flag, eta0, comparator=cmp, nthreads=4)
        for P in (1, -1, -2, -4, -8, -16, -32, -64, 2, 4, 8, 16, 32, 64):
            if P != 1 and -(-d // abs(P)) > 64:
                continue
            reg, cum, comp, xl = eng.simulate_alg_batch(z, y, flag, eta0, lanes_per_seq=P,
                                                        return_all=True)
            if P == 1 or P < 0:  # exact modes (P = 1: auto lanes, -k: k chained lanes)
                assert np.array_equal(reg, ref[0]) and np.array_equal(cum, ref[1])
                assert np.array_equal(comp, ref[2]) and np.array_equal(xl, ref[3])
            else:
                assert close(reg, ref[0]) and close(cum, ref[1]) and close(comp, ref[2]), P
                assert close(xl, ref[3]), P
            regc, cumc, compc, _ = eng.simulate_alg_batch(z, y, flag, eta0, comparator=cmp,
                                                          lanes_per_seq=P, return_all=True)
            assert close(regc, refc[0]) and close(compc, refc[2]), P


@pytest.mark.parametrize("kernel", ["lanes", "wave"])
@pytest.mark.parametrize("B,T,d", [(19, 120, 12), (70, 200, 5), (5, 130, 64), (3, 0, 4),
                                   (9, 65, 1)])
def test_smart_batch_splits(ocx, monkeypatch, kernel, B, T, d):
    """Both re-scan SMART kernels (lane groups / one wave per sequence) in the bit-exact
    modes, and the O(T·d) kernel in the others, against the oracle, thresholds spread so
    that some sequences switch early, late or never."""
    eng = ocx["engine"]
    monkeypatch.setenv("OCX_SMART_KERNEL", kernel)
    rng = np.random.default_rng(5 + d)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    th = rng.uniform(-1.0, 6.0, size=B)
    ref, sw = O.simulate_smart_batch(z, y, th, SQ2, nthreads=4)
    assert T == 0 or len(set(sw.tolist())) > 1  # a mix of switch steps
    for P in (1, -1, -2, -4, -8, -16, 2, 4, 8, 64):
        if d > 64 * abs(P) or (P < -1 and -P > 64):
            continue
        got, gsw = eng.simulate_smart_batch(z, y, th, SQ2, lanes_per_seq=P, return_switch=True)
        if P == 1 or P < 0:  # bit-exact modes: the re-scan kernels, in order
            assert np.array_equal(got, ref) and np.array_equal(gsw, sw), P
        else:  # the O(T·d) kernel: butterfly sums, closed-form comparator
            assert close_closed(got, ref, T) and np.array_equal(gsw, sw), P


def test_replay_batch(ocx):
    eng = ocx["engine"]
    rng = np.random.default_rng(9)
    B, T, d = 9, 77, 6
    z = rng.standard_normal((B, T, d))
    y = rng.standard_normal((B, T))
    a = rng.standard_normal((B, T + 1, d))
    cum, comp = eng.replay_batch(z, y, a)
    for b in range(B):
        assert cum[b] == O.replay_cum_loss(z[b], y[b], a[b])
        assert close(comp[b], O.comparator_loss_blas(z[b], y[b], a[b, T]), 1e-13)


def test_errors_are_loud(ocx):
    fa = ocx["fa"]
    with pytest.raises(ValueError):
        fa.simulate_alg(np.zeros((4, 2)), np.zeros(3), 0, 1.0)
    with pytest.raises(NotImplementedError):   # labels 0: the general solver, d > 256
        ocx["ef"].run_ftrl(np.zeros((4, 257)), np.zeros(4))


# ------------------------------------------------------------------ full-size properties
def test_full_size_properties(ocx):
    """Bench-sized batch (d=64, T=1e4): determinism, split invariance (exact vs auto),
    and a sample of sequences against the oracle on the very same generated inputs."""
    import torch
    eng = ocx["engine"]
    B, T, d = 2048, 10000, 64
    exact = eng.DeviceBatch(B, T, d, lanes_per_seq=1).generate_gT(base_seed=0, run0=0)
    r1 = exact.simulate_alg().clone()
    r2 = exact.simulate_alg().clone()
    auto = eng.DeviceBatch(B, T, d, lanes_per_seq=0).generate_gT(base_seed=0, run0=0)
    ra = auto.simulate_alg().clone()  # butterfly sums + closed-form comparator
    ra2 = auto.simulate_alg(closed_comparator=False).clone()
    torch.cuda.synchronize()
    assert torch.equal(r1, r2)
    assert auto.L.P > 1
    assert torch.all((ra2 - r1).abs() <= TOL * torch.clamp(r1.abs(), min=1.0))
    assert close_closed(ra.cpu().numpy(), r1.cpu().numpy(), T)
    r1 = r1.cpu().numpy()
    for b in (0, 1, 777, B - 1):
        zr, yr = O.gT_sample(0, T, b, d)
        assert r1[b] == O.simulate_alg(zr, yr, 0, SQ2), b
    del exact, auto
    torch.cuda.empty_cache()


@pytest.mark.parametrize("B,T,d", [(65536, 1000, 16), (512, 10000, 1024)])
def test_config_shapes_full_size(ocx, B, T, d):
    """configs[1] (65 536 sequences, d=16, T=1e3) and configs[4]'s shape (d=1024, T=1e4) at
    full size: the default (BEST + closed-form comparator) and the bit-exact mode agree within
    the closed form's bar, and sampled sequences match the oracle (bit for bit in exact
    mode)."""
    import torch
    eng = ocx["engine"]
    ex = eng.DeviceBatch(B, T, d, lanes_per_seq=1).generate_gT(base_seed=2, run0=0)
    r_ex = ex.simulate_alg().clone()
    del ex
    best = eng.DeviceBatch(B, T, d).generate_gT(base_seed=2, run0=0)
    r_best = best.simulate_alg().clone()
    torch.cuda.synchronize()
    del best
    torch.cuda.empty_cache()
    r_ex, r_best = r_ex.cpu().numpy(), r_best.cpu().numpy()
    assert close_closed(r_best, r_ex, T)
    for b in (0, 1, B // 3, B - 1):
        z, y = O.gT_sample(2, T, b, d)
        assert r_ex[b] == O.simulate_alg(z, y, 0, SQ2), b


# ------------------------------------------------------------------ sequence families
@pytest.mark.parametrize("family,runs,reps,T", [("iid", 48, 16, 1000), ("massart", 48, 20, 300),
                                                ("iid", 3, 2, 100), ("massart", 2, 3, 1000)])
def test_device_families_match_numpy(ocx, family, runs, reps, T):
    """Device-generated random families == the reference's builders (fp32 rows, labels
    sign(z @ u) through this host's BLAS order, Massart flips) for every (run, rep)."""
    import torch
    eng = ocx["engine"]
    base = 0
    stream0 = 13 if family == "iid" else 23
    run_idx = np.repeat(np.arange(runs), reps)
    rep_idx = np.tile(np.arange(reps), runs)
    seeds = base + 2025 * (run_idx + 1)
    db = eng.DeviceBatch(runs * reps, T, 5, lanes_per_seq=1)
    db.generate_family(family, seeds, stream0 + rep_idx)
    torch.cuda.synchronize()
    z = untile_z(db.z.cpu().numpy(), db.L)
    y = untile_y(db.y.cpu().numpy(), db.L)
    bad_y = 0
    for b in range(runs * reps):
        if family == "iid":
            zr, yr, _ = O.random_iid_sample(int(seeds[b]), T, int(rep_idx[b]))
        else:
            zr, yr, _ = O.noisy_iid_sample(int(seeds[b]), T, int(rep_idx[b]))
        assert np.array_equal(z[b], zr.astype(np.float64)), b
        bad_y += int((y[b] != yr.astype(np.float64)).sum())
    assert bad_y == 0


def test_device_fixed_families(ocx):
    import torch
    eng = ocx["engine"]
    for name, fn in (("flip", O.flip_sequence), ("switching", O.switching_two_leaders_sequence)):
        for T, d, P in ((1000, 5, 1), (77, 64, 4), (40, 3, 0)):
            db = eng.DeviceBatch(3, T, d, lanes_per_seq=P).generate_family(name)
            torch.cuda.synchronize()
            z = untile_z(db.z.cpu().numpy(), db.L)
            y = untile_y(db.y.cpu().numpy(), db.L)
            zr, yr, _ = fn(T, d=d)
            for b in range(3):
                assert np.array_equal(z[b], zr.astype(np.float64)), (name, T, d)
                assert np.array_equal(y[b], yr.astype(np.float64)), (name, T, d)


def test_driver_stats_golden(ocx, golden):
    """fast_driver.evaluate_stream_with_stats on device == the reference driver's output."""
    from online_convex_optimization_amd import drivers
    drv = golden.j["driver"]
    g_emp = {int(k): F(v) for k, v in drv["g_emp"].items()}
    for title, rec in drv["cases"].items():
        st = drivers.evaluate_stream_with_stats(title, drv["T_grid"], g_emp, runs=rec["runs"],
                                                replicates=rec["replicates"])
        for k, (m, c) in rec["stats"].items():
            assert np.array_equal(st[k][0], np.array([F(v) for v in m])), (title, k)
            assert np.array_equal(st[k][1], np.array([F(v) for v in c])), (title, k)


# ------------------------------------------------------------------ long-horizon (chunked)
@pytest.mark.parametrize("T,d,runs,P", [(300, 5, 100, 1), (257, 64, 40, 0), (1000, 16, 70, -1),
                                         (130, 100, 20, 0), (37, 1024, 6, 0), (211, 64, 33, 1)])
def test_streamed_gT_matches_resident(ocx, monkeypatch, T, d, runs, P):
    """A tiny HBM budget forces the T-chunked path (seek → pass A → pass B with saved PCG
    states): regrets must equal the single-launch path bit for bit in the exact modes; in
    the butterfly mode (P = 0) the single launch runs the pipelined step (ocx_alg_pipe.hip)
    and the chunks the plain one, so they agree to the butterfly bar."""
    eng = ocx["engine"]
    whole = eng.gT_regrets(T, runs, base_seed=4, d=d, run0=7, lanes_per_seq=P)
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", str(200e3 / 2**30))  # ~200 KB → many chunks
    chunked = eng.gT_regrets(T, runs, base_seed=4, d=d, run0=7, lanes_per_seq=P)
    if P == 0:
        assert close(chunked, whole)
    else:
        assert np.array_equal(whole, chunked)
    for r in (0, runs - 1):
        z, y = O.gT_sample(4, T, 7 + r, d)
        ref = O.simulate_alg(z, y, 0, SQ2)
        if P == 0:
            assert close(chunked[r], ref)
        else:
            assert chunked[r] == ref


@pytest.mark.parametrize("T,d,runs,exact", [(200, 64, 700, False), (60, 64, 9000, False),
                                             (60, 32, 9000, True), (40, 1024, 40, False),
                                             (300, 5, 500, True), (50, 16, 5000, True),
                                             (40, 8, 3000, True)])
def test_best_mode_default(ocx, T, d, runs, exact):
    """The batched APIs' default (OCX_LANES_BEST): the exact layout's sums where its chains
    are short — d < 64 — and butterfly sums for d=64 batches (the pipelined kernel: few-wave
    and big ones alike) and d=1024, with the certified closed-form comparator in both cases
    (the g(T) entry points, which generate their batches, take butterfly lanes of two
    coordinates for 4 <= d < 64, ocx_capi.hip gT_run), so the
    default is held to close_closed against the oracle, never to bit equality (the
    bit-exact mode, lanes_per_seq=1, is checked bit for bit beside it)."""
    eng, lib = ocx["engine"], ocx["lib"]
    L = lib.layout(runs, T, d, eng.LANES_BEST)
    assert bool(L.P == 1 or L.chain) == exact
    reg = eng.gT_regrets(T, runs, base_seed=9, d=d)  # + the closed-form comparator
    assert np.array_equal(reg, eng.gT_regrets(T, runs, base_seed=9, d=d,
                                              lanes_per_seq=eng.LANES_BEST))
    ex = eng.gT_regrets(T, runs, base_seed=9, d=d, lanes_per_seq=1)
    for r in (0, runs // 3, runs - 1):
        z, y = O.gT_sample(9, T, r, d)
        ref = O.simulate_alg(z, y, 0, SQ2)
        assert close_closed(reg[r], ref, T), (r, reg[r], ref)
        assert ex[r] == ref
    assert close_closed(reg, ex, T)


@pytest.mark.parametrize("P", [1, 0])
def test_streamed_gT_ragged_last_batch(ocx, monkeypatch, P):
    """More runs than one streamed batch (131 072) with a short last batch: the last batch
    gets its own lane layout (d=5: 1 lane x 6 coordinates for the full batches, 4 x 2 for
    100 sequences), so theta must be zeroed with that batch's row width."""
    eng = ocx["engine"]
    T, d, runs = 40, 5, 131072 + 100
    whole = eng.gT_regrets(T, runs, base_seed=6, d=d, lanes_per_seq=P)
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", str(0.1))     # streamed, a few T-chunks
    monkeypatch.setenv("OCX_MIN_RESIDENT", str(1 << 30))
    chunked = eng.gT_regrets(T, runs, base_seed=6, d=d, lanes_per_seq=P)
    # butterfly sums follow each batch's lane split, so only exact mode is layout-invariant
    assert np.array_equal(whole, chunked) if P == 1 else close(chunked, whole)
    for r in (0, 131071, 131072, runs - 1):
        z, y = O.gT_sample(6, T, r, d)
        ref = O.simulate_alg(z, y, 0, SQ2)
        assert close(chunked[r], ref) if P == 0 else chunked[r] == ref


@pytest.mark.parametrize("T,d,runs", [(50, 64, 700), (2, 1024, 3000)])
def test_resident_batching_is_invisible(ocx, monkeypatch, T, d, runs):
    """Resident g(T) batches of any size (exact mode: lanes chosen per batch size; d=1024,
    3000 runs: 1500 waves, cut to one-round batches) give the same regrets bit for bit."""
    eng = ocx["engine"]
    whole = eng.gT_regrets(T, runs, base_seed=2, d=d, run0=5, lanes_per_seq=1)
    monkeypatch.setenv("OCX_MIN_RESIDENT", "1")
    per_seq = T * (8 * d + 8)
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", str(97 * per_seq / 2**30))  # batches of ~97
    small = eng.gT_regrets(T, runs, base_seed=2, d=d, run0=5, lanes_per_seq=1)
    assert np.array_equal(whole, small)
    for r in (0, runs // 2, runs - 1):
        z, y = O.gT_sample(2, T, 5 + r, d)
        assert small[r] == O.simulate_alg(z, y, 0, SQ2)


# ------------------------------------------------------------------ exact FTL (closed form)
def test_ftl_exact_matches_oracle(ocx):
    """exact_ftl run_ftl_exact / run_ftrl(no comparator) on the GPU == the oracle's closed
    form (the closed form itself is checked against scipy in test_exact_comparator_cpu)."""
    eng, ef = ocx["engine"], ocx["ef"]
    rng = np.random.default_rng(11)
    B, T, d = 21, 300, 7
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    for P in (1, -1, 4):
        cum, comp, act, ok = eng.ftl_exact_batch(z, y, lanes_per_seq=P)
        assert ok.all()
        for b in range(B):
            rc, rp, ra, rin = O.ftl_exact_closed_form(z[b], y[b])
            if P != 4:
                assert (cum[b], comp[b]) == (rc, rp) and np.array_equal(act[b], ra), (P, b)
            else:
                assert close([cum[b], comp[b]], [rc, rp]) and close(act[b], ra)
    res = ef.run_ftl_exact(z[0], y[0])
    rc, rp, ra, _ = O.ftl_exact_closed_form(z[0], y[0])
    cb = O.comparator_loss_blas_order(z[0], y[0], ra)  # the drop-in's comp_loss order
    assert (res.cum_loss, res.comp_loss) == (rc, cb) and np.array_equal(res.x_last, ra)
    assert close(cb, rp, 1e-13)
    rr = ef.run_ftrl(z[1], y[1], eta0=SQ2)
    _, _, a1, _ = O.ftl_exact_closed_form(z[1], y[1])
    ref = O.simulate_alg_full(z[1], y[1], 0, SQ2, comparator=a1)
    c1 = O.comparator_loss_blas_order(z[1], y[1], a1)
    assert (rr.regret, rr.cum_loss, rr.comp_loss) == (ref[1] - c1, ref[1], c1)
    # outside the regime: the general solver's actions, replayed (tests/test_gpu_exact_general.py)
    g = eng.exact_ball_solve(2.0 * z[:1], y[:1])
    r2 = ef.run_ftl_exact(2.0 * z[0], y[0])
    assert np.array_equal(r2.x_last, g["actions"][0, T])
    assert r2.cum_loss == np.cumsum(g["step_loss"][0, :T])[-1]


@pytest.mark.parametrize("B,T,d", [(21, 300, 7), (33, 257, 64), (5, 40, 1024), (4, 0, 3),
                                   (9, 100, 1)])
def test_ftrl_vs_exact_fused_matches_oracle(ocx, B, T, d):
    """One-pass FTRL + exact FTL (ocx_ftrl_vs_exact_batch) == the oracle's closed form and
    its FTRL run against that comparator; comp_ftl == FTRL's own FTL comparator loss."""
    eng = ocx["engine"]
    rng = np.random.default_rng(17 + d)
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    for P in (1, -1, 4):
        if P != 1 and d > 64 * abs(P):
            continue
        r = eng.ftrl_vs_exact_batch(z, y, SQ2, lanes_per_seq=P, with_ftl_comparator=True)
        assert r["in_regime"].all()
        for b in range(B):
            rc, rp, ra, _ = O.ftl_exact_closed_form(z[b], y[b])
            fr = O.simulate_alg_full(z[b], y[b], 0, SQ2, comparator=ra)
            ff = O.simulate_alg_full(z[b], y[b], 0, SQ2)
            got = [r["cum_exact"][b], r["comp"][b], r["cum_ftrl"][b], r["ftrl"][b],
                   r["comp_ftl"][b]]
            want = [rc, rp, fr[1], fr[0], ff[2]]
            if P != 4:
                assert got == want and np.array_equal(r["action"][b], ra), (P, b)
            else:  # butterfly sums + closed-form comparator losses
                assert close_closed(got, want, T) and close(r["action"][b], ra), (P, b)
    if B and T and d <= 10:   # outside the regime: the general solver's comparator
        r2 = eng.ftrl_vs_exact_batch(2.0 * z, y, SQ2)
        assert not r2["in_regime"].any()
        g = eng.exact_ball_solve(2.0 * z, y, all_prefixes=False)
        assert np.array_equal(r2["action"], g["actions"][:, 0])


def test_exact_driver_matches_oracle(ocx):
    from online_convex_optimization_amd import drivers
    runs, reps, T = 2, 3, 120
    st = drivers.exact_evaluate_stream_with_stats("Random i.i.d. (separable)", [T], runs=runs,
                                                  replicates=reps)
    ftrl, ftl = [], []
    for r in range(runs):
        fr, fl = [], []
        for rep in range(reps):
            z, y, _ = O.random_iid_sample(2025 * (r + 1), T, rep)
            c, p, a, ok = O.ftl_exact_closed_form(z, y)
            assert ok
            fl.append(c - p)
            fr.append(O.simulate_alg_full(z, y, 0, SQ2, comparator=a)[0])
        ftrl.append(float(np.mean(fr)))
        ftl.append(float(np.mean(fl)))
    assert st["FTRL"][0][0] == float(np.mean(ftrl))
    assert st["FTL (exact)"][0][0] == float(np.mean(ftl))


def test_release_buffers_then_regrow(ocx):
    """ocx_release_buffers frees the cached HBM; the next call regrows it, same results."""
    eng = ocx["engine"]
    a = eng.gT_regrets(300, 40, d=64, lanes_per_seq=1)
    eng.release_buffers()
    eng.release_buffers()  # idempotent
    b = eng.gT_regrets(300, 40, d=64, lanes_per_seq=1)
    assert np.array_equal(a, b)


# ------------------------------------------------------------------ closed-form comparator
@pytest.mark.parametrize("B,T,d,P", [(700, 300, 64, 128), (9000, 60, 64, 128), (300, 500, 5, 0),
                                     (40, 200, 1024, 128), (130, 1000, 16, 4), (64, 1, 3, 0)])
def test_closed_comparator_matches_two_pass(ocx, B, T, d, P):
    """OCX_ALG_CLIPPED_ROWS on g(T)-sampler rows: the loop is untouched (cum_loss bit for
    bit), the comparator loss T/2 - ||theta_T|| agrees with the streamed sum within the
    sum's own rounding, and so do the regrets (also against the oracle)."""
    import torch
    eng = ocx["engine"]
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).generate_gT(base_seed=5, run0=3)
    assert db.rows_clipped and not db.exact
    r_two = db.simulate_alg(closed_comparator=False).clone()
    cum_two, comp_two = db.cum.clone(), db.comp.clone()
    flag = torch.zeros(B, dtype=torch.int32, device=db.device)
    r_one = db.simulate_alg(closed_out=flag).clone()
    torch.cuda.synchronize()
    assert bool(torch.all(flag == 1))  # the sampler's sequences are all clean
    assert torch.equal(db.cum, cum_two)
    assert close_closed(db.comp.cpu().numpy(), comp_two.cpu().numpy(), T)
    assert close_closed(r_one.cpu().numpy(), r_two.cpu().numpy(), T)
    r_one = r_one.cpu().numpy()
    for b in (0, B // 2, B - 1):
        z, y = O.gT_sample(5, T, 3 + b, d)
        assert close_closed(r_one[b], O.simulate_alg(z, y, 0, SQ2), T), b
    # FTL (alg_flag 1) takes the same closed form
    f_two = db.simulate_alg(1, closed_comparator=False).clone()
    f_one = db.simulate_alg(1).clone()
    torch.cuda.synchronize()
    assert close_closed(f_one.cpu().numpy(), f_two.cpu().numpy(), T)


@pytest.mark.parametrize("P", [-1, 128, 0])
def test_closed_comparator_falls_back(ocx, P):
    """Sequences whose sub-gradients are not all -y_t/2 (a label of 0.5, a zero row with a
    zero label: an exact tie) or with a row outside the unit ball (1.5x, and one just
    outside, 1 + 1e-9: the kernel certifies ||z_t|| <= 1 itself, closed_comparator=True is
    only a request) take the second pass, bit-identical to the two-pass kernel; the clean
    sequences of the same waves keep the closed form."""
    import torch
    eng = ocx["engine"]
    rng = np.random.default_rng(3)
    B, T, d = 70, 120, 8
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    y[5, 17] = 0.5                       # not ±1
    z[9, 0] = 0.0
    y[9, 0] = 0.0                        # q - y == 0: the sub-gradient is 0, not -y/2
    y[40, T - 1] = 0.25
    z[12, 30] *= 1.5 / np.linalg.norm(z[12, 30])            # a row far outside the ball
    z[61, T - 1] *= (1.0 + 1e-9) / np.linalg.norm(z[61, T - 1])  # just outside it
    unclean = {5, 9, 12, 40, 61}
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).pack(z, y)
    assert not db.rows_clipped
    two = db.simulate_alg(closed_comparator=False).clone()
    flag = torch.full((B,), 7, dtype=torch.int32, device=db.device)
    one = db.simulate_alg(closed_comparator=True, closed_out=flag).clone()
    dflt = torch.full((B,), 7, dtype=torch.int32, device=db.device)
    auto = db.simulate_alg(closed_out=dflt).clone()  # default: the closed form outside exact modes
    torch.cuda.synchronize()
    two, one, flag = two.cpu().numpy(), one.cpu().numpy(), flag.cpu().numpy()
    assert set(np.nonzero(flag == 0)[0]) == unclean and np.all(flag[flag != 0] == 1)
    if db.exact:
        assert np.array_equal(auto.cpu().numpy(), two)
    else:
        assert np.array_equal(auto.cpu().numpy(), one)
        assert np.array_equal(dflt.cpu().numpy(), flag)
    for b in unclean:
        assert one[b] == two[b], b
    assert close_closed(one, two, T)
    for b in (0, 5, 9, 12, 40, 61, B - 1):
        assert close_closed(one[b], O.simulate_alg(z[b], y[b], 0, SQ2), T), b


def test_gT_sweep_c_entry(ocx):
    """ocx_gT_sweep (the C-level multi-device sweep, ngpus=1 here) and its device-list form
    against per-T gT_regrets calls."""
    import ctypes
    eng, lib = ocx["engine"], ocx["lib"]
    grid = np.array([30, 200, 1000], dtype=np.int64)
    runs = 50
    gmax = np.zeros(3)
    regs = np.zeros((3, runs))
    lib.call("ocx_gT_sweep", grid.ctypes.data_as(lib.c_i64p), 3, runs, 7, 16, SQ2, 1,
             lib.ptr(gmax), lib.ptr(regs))
    gmax2 = np.zeros(3)
    lib.call("ocx_gT_sweep", grid.ctypes.data_as(lib.c_i64p), 3, runs, 7, 16, SQ2, 0,
             lib.ptr(gmax2), None)
    assert np.array_equal(gmax, gmax2)
    for i, T in enumerate(grid):
        ref = eng.gT_regrets(int(T), runs, base_seed=7, d=16)
        assert np.array_equal(regs[i], ref)
        assert gmax[i] == eng.max_regret(ref)
    with pytest.raises(ValueError):
        lib.call("ocx_gT_sweep", grid.ctypes.data_as(lib.c_i64p), 3, runs, 7, 16, SQ2, 999,
                 lib.ptr(gmax), None)
    out = eng.gT_sweep(list(grid), runs, base_seed=7, d=16, devices=[0, 0, 0])
    for i, T in enumerate(grid):
        assert np.array_equal(out[int(T)][1], regs[i]) and out[int(T)][0] == gmax[i]


@pytest.mark.parametrize("P", [128, 0])
def test_ftrl_vs_exact_closed_form(ocx, P):
    """DeviceBatch.ftrl_vs_exact: closed-form comparator losses (OCX_ALG_CLOSED_COMPARATOR)
    vs the two-pass kernel on sampler rows (all in the regime: one pass), and on packed rows
    with a few sequences outside it (those stream pass 2, bit-identical to two-pass)."""
    import torch
    eng = ocx["engine"]
    B, T, d = 600, 400, 64
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=P).generate_gT(base_seed=8)
    cf2 = torch.zeros(B, dtype=torch.float64, device=db.device)
    cf1 = torch.zeros_like(cf2)
    db.ftrl_vs_exact(SQ2, comp_ftl=cf2, closed_comparator=False)
    two = [t.clone() for t in (db.cum, db.cum_exact, db.comp)]
    db.ftrl_vs_exact(SQ2, comp_ftl=cf1)
    one = [db.cum, db.cum_exact, db.comp]
    torch.cuda.synchronize()
    assert torch.equal(one[0], two[0]) and torch.equal(one[1], two[1])
    assert close_closed(one[2].cpu().numpy(), two[2].cpu().numpy(), T)
    assert close_closed(cf1.cpu().numpy(), cf2.cpu().numpy(), T)
    # rows outside the ball in a few sequences: those take the second pass
    rng = np.random.default_rng(2)
    z = rng.standard_normal((70, 120, 8))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((70, 120)) < 0.5, -1.0, 1.0)
    z[3, 10] *= 1.5
    z[50, 0] *= (1.0 + 1e-9) / np.linalg.norm(z[50, 0])  # just outside the ball
    pk = eng.DeviceBatch(70, 120, 8, lanes_per_seq=P).pack(z, y)
    pk.ftrl_vs_exact(SQ2, closed_comparator=False)
    a = pk.comp.clone()
    pk.ftrl_vs_exact(SQ2)
    torch.cuda.synchronize()
    a, bb = a.cpu().numpy(), pk.comp.cpu().numpy()
    assert a[3] == bb[3] and a[50] == bb[50]
    assert close_closed(bb, a, 120)


@pytest.mark.parametrize("P", [0, 128])
def test_streamed_closed_form_fallback(ocx, monkeypatch, P):
    """The streamed path's closed form (ocx_alg_chunk_kernel mode 2) and its fallback: with
    every third run marked as failing the check (ocx_test_gT_regrets_unclean, the test-only
    entry point of include/ocx_testing.h), those runs get the regenerated second pass,
    bit-identical to the resident two-pass kernel; the rest keep the closed form,
    bit-identical to the resident closed form."""
    import torch
    eng = ocx["engine"]
    T, d, runs = 257, 64, 40
    db = eng.DeviceBatch(runs, T, d, lanes_per_seq=P).generate_gT(base_seed=4, run0=7)
    closed = db.simulate_alg().clone()
    two = db.simulate_alg(closed_comparator=False).clone()
    torch.cuda.synchronize()
    closed, two = closed.cpu().numpy(), two.cpu().numpy()
    del db
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", str(200e3 / 2**30))  # ~200 KB → streamed
    monkeypatch.setenv("OCX_MIN_RESIDENT", str(1 << 30))
    plain = eng.gT_regrets(T, runs, base_seed=4, d=d, run0=7, lanes_per_seq=P)
    # butterfly layouts (both cases here): the resident launch is the pipelined kernel, the
    # chunks the plain one (test_streamed_gT_matches_resident): equal to the 1e-12 bar
    def same(a, b):
        return close(a, b)
    assert same(plain, closed)
    lib = ocx["lib"]
    mixed = np.zeros(runs)
    lib.call("ocx_test_gT_regrets_unclean", 4, T, 7, runs, d, SQ2, lib.ptr(mixed), P, 0, 3)
    marked = np.arange(runs) % 3 == 0
    assert same(mixed[marked], two[marked])
    assert same(mixed[~marked], closed[~marked])
    # the marked runs really took the streamed second pass: bit-equal to a two-pass run of
    # the same (chunked) kernel family, i.e. not the closed form
    assert not np.array_equal(mixed[marked], closed[marked])


@pytest.mark.parametrize("T,d", [(1, 3), (1, 20), (2, 8), (3, 5), (7, 13), (130, 5), (9000, 5),
                                 (65, 64), (12, 1024), (1, 32), (1, 77), (1, 1024), (2, 37),
                                 (6, 64), (7, 9), (11, 130), (130, 64)])
def test_comparator_loss_blas_order(ocx, T, d):
    """ocx_comparator_loss_blas_batch == the oracle's dgemv_t / pairwise order bit for bit
    (pinned on the goldens in test_oracle_golden), and == NumPy on this host to 1e-15."""
    from online_convex_optimization_amd import _lib
    from online_convex_optimization_amd._lib import ptr
    rng = np.random.default_rng(T * 7 + d)
    B = 3
    z = rng.standard_normal((B, T, d))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    x = rng.standard_normal((B, d))
    got = np.zeros(B)
    _lib.call("ocx_comparator_loss_blas_batch", ptr(z), ptr(y), ptr(x), B, T, d, ptr(got), 0)
    for b in range(B):
        if T * d <= 20000:
            assert got[b] == O.comparator_loss_blas_order(z[b], y[b], x[b]), (T, d, b)
        assert close(got[b], O.comparator_loss_blas(z[b], y[b], x[b]), 1e-15)

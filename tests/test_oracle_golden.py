"""Pin the CPU oracle against the reference's own outputs (bit-for-bit).

The fixtures were produced by running the reference (tests/golden/make_golden.py).
These tests run on CPU; they make the oracle trustworthy as the GPU checker.
"""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests._golden import F

PUBLISHED_GT = [6.034165981694009, 8.297032923590692, 10.446825985542404, 12.032218781087039,
                13.383600324774818, 14.946774913365687, 15.951320592930585, 17.196625822976216,
                18.087283038366593, 19.088517830594924]


def test_explicit_simulate_alg_bitexact(golden):
    n = 0
    for name, z, y, rec in golden.explicit():
        for key, h in rec["alg"].items():
            flag, eta_h = key.split("_")
            got = O.simulate_alg(z, y, int(flag), float.fromhex(eta_h))
            assert got == F(h), (name, key, got, F(h))
            n += 1
    assert n > 50


def test_explicit_smart_bitexact(golden):
    for name, z, y, rec in golden.explicit():
        for th_h, h in rec["smart"].items():
            got = O.simulate_SMART_like(z, y, float.fromhex(th_h), math.sqrt(2))
            assert got == F(h), (name, th_h, got, F(h))
        assert O.simulate_SMART(z, y) == F(rec["smart_default"]), name


def test_exact_ftl_run_ftrl_and_replay(golden):
    for name, z, y, rec in golden.explicit():
        if "run_ftrl" not in rec:
            continue
        a = golden.arr(f"{name}__comparator")
        reg, cum, comp, xl = O.simulate_alg_full(z, y, 0, 1.0, comparator=a)
        r = rec["run_ftrl"]
        # the FTRL trajectory is the same op sequence → bit-exact
        assert cum == F(r["cum_loss"]), name
        assert np.array_equal(xl, np.array([F(v) for v in r["x_last"]])), name
        # exact_ftl's comparator loss is BLAS dgemv + pairwise |r| sum; the explicit-order
        # restatement (what ocx_comp_blas.hip computes) reproduces it
        assert O.comparator_loss_blas(z, y, a) == F(r["comp_loss"]), name
        assert O.comparator_loss_blas_order(z, y, a) == F(r["comp_loss"]), name
        assert O.comparator_loss_blas_order(z, y, golden.arr(f"{name}__actions")[-1]) == \
            F(rec["replay"]["comp_loss"]), name
        # the sequential comparator sum agrees to rounding
        assert comp == pytest.approx(F(r["comp_loss"]), rel=1e-13, abs=1e-12)
        acts = golden.arr(f"{name}__actions")
        assert O.replay_cum_loss(z, y, acts) == F(rec["replay"]["cum_loss"]), name


def _openblas_arch():
    try:
        import threadpoolctl
        for i in threadpoolctl.threadpool_info():
            if i.get("internal_api") == "openblas":
                return i.get("architecture"), i.get("version")
    except Exception:  # pragma: no cover - threadpoolctl absent
        pass
    return None, None


@pytest.mark.skipif(_openblas_arch() != ("SkylakeX", "0.3.29"),
                    reason="the dgemv/ddot orders were probed on OpenBLAS 0.3.29's SkylakeX "
                           "kernels (this image, where the goldens were made)")
def test_comparator_blas_order_matches_numpy():
    """exact_ftl.py:224-227 `0.5 * np.abs(z @ x - y).sum()` in the oracle's explicit order
    equals NumPy on this image bit for bit, on every row kernel OpenBLAS's dgemv_t picks
    (4x4 groups, the 4x2 pair where T mod 4 >= 2, the 4x1 last row, one-row ddot with its
    8-lane blocks from d = 32) and every d mod 4 / d mod 16 / d mod 32 tail."""
    rng = np.random.default_rng(11)
    n = 0
    for T in (1, 2, 3, 5, 6, 7, 10, 11):
        for d in list(range(1, 41)) + [47, 63, 64, 65, 96, 127, 129, 200, 1024]:
            z = rng.standard_normal((T, d))
            y = np.where(rng.random(T) < 0.5, -1.0, 1.0)
            x = rng.standard_normal(d)
            want = 0.5 * float(np.abs(z @ x - y).sum())
            assert O.comparator_loss_blas_order(z, y, x) == want, (T, d)
            n += 1
    assert n == 8 * 49


def test_seeded_gT_sequences(golden):
    for rec in golden.j["seeded_gT"]:
        z, y = O.gT_sample(rec["base_seed"], rec["T"], rec["run"], rec["d"])
        assert float(z.sum()) == F(rec["z_sum"])
        assert float(y.sum()) == F(rec["y_sum"])
        assert O.simulate_alg(z, y, 0, math.sqrt(2)) == F(rec["regret"]), rec


def test_gT_small_sweep(golden):
    s = golden.j["gT_small"]
    g = O.empirical_worst_case_thresholds(s["T_grid"], runs=s["runs"], base_seed=s["base_seed"])
    for T in s["T_grid"]:
        assert g[T] == F(s["g"][str(T)])


def test_published_gT_values_recorded(golden):
    rec = golden.j["gT_published"]
    assert [F(h) for h in rec["g"]] == PUBLISHED_GT


def test_deterministic_families_exact_ties(golden):
    g_pub = dict(zip(range(100, 1100, 100), PUBLISHED_GT))
    for title, fn in (("Label flips", O.flip_sequence),
                      ("Switching leaders", O.switching_two_leaders_sequence)):
        for T_s, row in golden.j["families"][title].items():
            T = int(T_s)
            z, y, _ = fn(T)
            assert O.simulate_alg(z, y, 0, math.sqrt(2)) == F(row["FTRL"])
            assert O.simulate_alg(z, y, 1, math.sqrt(2)) == F(row["FTL"])
            assert O.simulate_SMART(z, y) == F(row["SMART"])
            assert O.simulate_SMART_like(z, y, g_pub[T], math.sqrt(2)) == F(row["EMP"])
    # BASELINE.md published values at T=1000
    fl = golden.j["families"]["Label flips"]["1000"]
    assert [F(fl[k]) for k in ("FTL", "SMART", "EMP", "FTRL")] == [
        250.0, 50.93691776310368, 27.057819971048957, 10.82084049854575]


def test_random_streams(golden):
    for rec in golden.j["streams"]:
        if rec["title"].startswith("Random"):
            z, y, u = O.random_iid_sample(rec["run_seed"], rec["T"], rec["rep"])
        else:
            z, y, u = O.noisy_iid_sample(rec["run_seed"], rec["T"], rec["rep"])
        assert float(z.astype(np.float64).sum()) == F(rec["z_sum"])
        assert float(y.astype(np.float64).sum()) == F(rec["y_sum"])
        assert O.simulate_alg(z, y, 0, math.sqrt(2)) == F(rec["FTRL"])
        assert O.simulate_alg(z, y, 1, math.sqrt(2)) == F(rec["FTL"])
        assert O.simulate_SMART(z, y) == F(rec["SMART"])


def test_batch_matches_scalar():
    rng = np.random.default_rng(1)
    B, T, d = 5, 40, 6
    z = rng.standard_normal((B, T, d))
    z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
    reg, cum, comp, xl = O.simulate_alg_batch(z, y, 0, math.sqrt(2), nthreads=2)
    for b in range(B):
        assert reg[b] == O.simulate_alg(z[b], y[b], 0, math.sqrt(2))
    regs, _ = O.simulate_smart_batch(z, y, 2.0, math.sqrt(2), nthreads=2)
    for b in range(B):
        assert regs[b] == O.simulate_SMART_like(z[b], y[b], 2.0, math.sqrt(2))

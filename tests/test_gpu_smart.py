"""GPU: SMART in O(T·d) (csrc/ocx_smart_closed.hip, ocx_dev_simulate_smart_ex).

The pre-switch prefix loss of fast_algorithms.py:157-160 has the closed form
(t+1)/2 − ½ s_t·S_t on clipped rows with ±1 labels; the kernel lets it decide the switch
only outside a rounding guard band and re-scans the prefix inside it, so its switch steps
must be the reference's: bit-identical regrets whenever the final comparator keeps the
reference's streamed sum (OCX_SMART_CLOSED_PREFIX alone), close_closed with the
closed-form comparator (the batched default outside the bit-exact modes)."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests._golden import F
from tests.test_gpu_parity import PUBLISHED_GT, close_closed

pytestmark = pytest.mark.gpu
SQ2 = math.sqrt(2)


@pytest.fixture(scope="module")
def eng():
    from online_convex_optimization_amd import _lib, engine
    assert _lib.device_count() >= 1
    return engine


def _smart(eng, z, y, th, *, lanes, prefix, comp):
    """simulate_smart on a packed batch: (regret, switch step, [re-scanned steps, closed])."""
    import torch
    B, T, d = z.shape
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=lanes).pack(z, y)
    sw = torch.full((B,), -7, dtype=torch.int64, device=db.device)
    st = torch.zeros(2, dtype=torch.int64, device=db.device)
    reg = db.simulate_smart(th, SQ2, switch_step=sw, closed_prefix=prefix,
                            closed_comparator=comp, stats=st)
    torch.cuda.synchronize()
    return reg.cpu().numpy()[:B].copy(), sw.cpu().numpy(), st.cpu().numpy()


def test_closed_prefix_golden_bitexact(eng, golden):
    """Every explicit golden (unclipped rows, real-valued labels, zero rows, d up to 1024,
    T up to 1000) with every golden threshold: the guarded closed prefix in the exact layout
    reproduces the reference's SMART regrets bit for bit (outside the regime every step
    re-scans)."""
    for name, z, y, rec in golden.explicit():
        T, d = z.shape
        ths = [float.fromhex(h) for h in rec["smart"]] + [math.sqrt(2 * T)]
        want = [F(h) for h in rec["smart"].values()] + [F(rec["smart_default"])]
        Z = np.repeat(z[None].astype(np.float64), len(ths), axis=0)
        Y = np.repeat(y[None].astype(np.float64), len(ths), axis=0)
        got, _, _ = _smart(eng, Z, Y, np.array(ths), lanes=1, prefix=True, comp=False)
        assert list(got) == want, name


def test_families_bitexact_default_mode(eng, golden):
    """Flip and switching families (exact arithmetic, exact ties) through the batched
    default (OCX_LANES_BEST: closed prefix + closed comparator): SMART and EMP regrets equal
    the reference's goldens bit for bit."""
    g_pub = dict(zip(range(100, 1100, 100), PUBLISHED_GT))
    for title, fn in (("Label flips", O.flip_sequence),
                      ("Switching leaders", O.switching_two_leaders_sequence)):
        for T_s, row in golden.j["families"][title].items():
            T = int(T_s)
            z, y, _ = fn(T)
            Z = np.repeat(z[None].astype(np.float64), 2, axis=0)
            Y = np.repeat(y[None].astype(np.float64), 2, axis=0)
            th = np.array([math.sqrt(2 * T), g_pub[T]])
            got, sw = eng.simulate_smart_batch(Z, Y, th, SQ2, return_switch=True)
            assert (got[0], got[1]) == (F(row["SMART"]), F(row["EMP"])), (title, T)
            for k in range(2):
                _, rsw = O.simulate_SMART_like(z, y, th[k], SQ2, return_switch=True)
                assert sw[k] == rsw, (title, T, k)


def test_closed_prefix_matches_rescan_on_sampler_rows(eng):
    """g(T)-sampler rows, thresholds spread over the range where switches happen: the
    closed prefix (exact layout) == the re-scan kernel bit for bit, switch steps included,
    with almost no re-scanned steps; with the closed comparator too, close_closed; sampled
    sequences against the oracle."""
    import torch
    B, T, d = 512, 1500, 8
    rng = np.random.default_rng(12)
    th = rng.uniform(-1.0, 30.0, size=B)
    th[::7] = 1e9  # never switches: the whole horizon stays pre-switch
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=1).generate_gT(base_seed=11)
    out = {}
    for key, (pf, cc) in {"rescan": (False, False), "prefix": (True, False),
                          "both": (True, True)}.items():
        sw = torch.full((B,), -7, dtype=torch.int64, device=db.device)
        st = torch.zeros(2, dtype=torch.int64, device=db.device)
        reg = db.simulate_smart(th, SQ2, switch_step=sw, closed_prefix=pf, closed_comparator=cc,
                                stats=st).clone()
        torch.cuda.synchronize()
        out[key] = (reg.cpu().numpy(), sw.cpu().numpy(), st.cpu().numpy())
    r0, s0, st0 = out["rescan"]
    r1, s1, st1 = out["prefix"]
    r2, s2, st2 = out["both"]
    assert len(set(s0.tolist())) > 10 and (s0 == -1).any() and (s0 >= 0).any()
    assert np.array_equal(r1, r0) and np.array_equal(s1, s0)
    assert np.array_equal(s2, s0) and close_closed(r2, r0, T)
    pre_switch_steps = int(np.where(s0 < 0, T, s0 + 1).sum())
    assert st0[0] == pre_switch_steps          # the re-scan kernel scans every step
    assert st1[0] <= pre_switch_steps // 1000  # the closed prefix almost never
    assert st2[1] == B                         # every sampler sequence is certified
    for b in (0, 1, B // 2, B - 1):
        z, y = O.gT_sample(11, T, b, d)
        ref, rsw = O.simulate_SMART_like(z, y, th[b], SQ2, return_switch=True)
        assert r1[b] == ref and s1[b] == rsw, b


def test_guard_band_sends_exact_ties_to_the_rescan(eng):
    """Flip sequences make ftl_loss − s_loss an exact half-integer at every step, so
    half-integer thresholds meet it EXACTLY (the reference's `>=` then fires): such steps
    fall inside the guard band and must re-scan, giving the reference's switch steps."""
    T = 400
    z, y, _ = O.flip_sequence(T)
    th = np.arange(-2.0, 40.0, 0.5)
    B = len(th)
    Z = np.repeat(z[None].astype(np.float64), B, axis=0)
    Y = np.repeat(y[None].astype(np.float64), B, axis=0)
    ref, rsw = O.simulate_smart_batch(Z, Y, th, SQ2, nthreads=4)
    for lanes in (1, eng.LANES_BEST):
        got, sw, st = _smart(eng, Z, Y, th, lanes=lanes, prefix=True, comp=lanes != 1)
        assert np.array_equal(got, ref) and np.array_equal(sw, rsw), lanes
        assert st[0] > 0  # some exact ties were caught by the band


@pytest.mark.parametrize("family,runs,reps", [("iid", 2, 2), ("massart", 2, 2)])
def test_random_families_T1e4(eng, family, runs, reps):
    """The driver families at T = 1e4 (fast_driver.py:100-111 calls SMART per replicate):
    the batched default (O(T·d)) against the oracle's O(T²) SMART within close_closed, the
    same switch steps, for SMART's sqrt(2T) and an early-switching threshold."""
    T, d = 10000, 5
    stream0 = 13 if family == "iid" else 23
    run_idx = np.repeat(np.arange(runs), reps)
    rep_idx = np.tile(np.arange(reps), runs)
    seeds = 2025 * (run_idx + 1)
    B = runs * reps
    import torch
    db = eng.DeviceBatch(2 * B, T, d)
    db.generate_family(family, np.concatenate([seeds, seeds]),
                       np.concatenate([stream0 + rep_idx, stream0 + rep_idx]))
    th = np.concatenate([np.full(B, math.sqrt(2 * T)), np.full(B, 2.0)])
    sw = torch.zeros(2 * B, dtype=torch.int64, device=db.device)
    reg = db.simulate_smart(th, SQ2, switch_step=sw).clone()
    torch.cuda.synchronize()
    reg, sw = reg.cpu().numpy(), sw.cpu().numpy()
    for b in range(2 * B):
        fn = O.random_iid_sample if family == "iid" else O.noisy_iid_sample
        z, y, _ = fn(int(seeds[b % B]), T, int(rep_idx[b % B]))
        ref, rsw = O.simulate_SMART_like(z, y, th[b], SQ2, return_switch=True)
        assert close_closed(reg[b], ref, T) and sw[b] == rsw, (family, b, reg[b], ref, sw[b], rsw)


def test_non_finite_thresholds_decide_without_rescan(eng):
    """thresh = +inf (never switch), -inf (switch at step 0), NaN (`>= NaN` is false: never)
    and a huge finite one: the closed-prefix kernel decides every step without re-scanning
    the prefix (an infinite threshold used to widen the rounding band to infinity and send
    every step to the O(t) re-scan), with the reference's switch steps and regrets."""
    import torch
    B, T, d = 4, 300, 8
    th = np.array([np.inf, -np.inf, np.nan, 1e300])
    db = eng.DeviceBatch(B, T, d, lanes_per_seq=1).generate_gT(base_seed=5)
    sw = torch.full((B,), -7, dtype=torch.int64, device=db.device)
    st = torch.zeros(2, dtype=torch.int64, device=db.device)
    reg = db.simulate_smart(th, SQ2, switch_step=sw, closed_prefix=True,
                            closed_comparator=False, stats=st).clone()
    torch.cuda.synchronize()
    reg, sw, st = reg.cpu().numpy(), sw.cpu().numpy(), st.cpu().numpy()
    assert st[0] == 0, st
    assert list(sw) == [-1, 0, -1, -1]
    for b in range(B):
        z, y = O.gT_sample(5, T, b, d)
        ref, rsw = O.simulate_SMART_like(z, y, float(th[b]), SQ2, return_switch=True)
        assert reg[b] == ref and sw[b] == rsw, (b, reg[b], ref, sw[b], rsw)

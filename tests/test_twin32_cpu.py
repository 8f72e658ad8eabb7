"""The float32 twin's oracle (oracle.t32_*, algorithms.py:10-171) pinned on the CPU.

tests/golden/twin32.npz holds the values of the twin's own NumPy calls on this image
(tests/golden/make_twin32.py).  The explicit-order restatement — the arithmetic the GPU
kernel ocx_twin32.hip implements — must reproduce every one of them bit for bit.  Where
the host's BLAS matches this image's (the probe below), the NumPy calls themselves are
also re-run against the fixtures.
"""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
F = np.float32


@pytest.fixture(scope="module")
def fx():
    with np.load(os.path.join(HERE, "golden", "twin32.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def _alg_keys(fx):
    return sorted({k[:-5] for k in fx if k.endswith("_runs")})


def test_alg_groups_bitexact(fx):
    n = 0
    for key in _alg_keys(fx):
        z, y = fx[key + "_z"], fx[key + "_y"]
        for i, (a, e) in enumerate(fx[key + "_runs"]):
            for b in range(z.shape[0]):
                r, c, p = O.t32_simulate_alg_full(z[b], y[b], int(a), float(e))
                assert type(r) is np.float32
                assert (r, c, p) == (fx[key + "_res"][i, b], fx[key + "_cum"][i, b],
                                     fx[key + "_comp"][i, b]), (key, a, e, b)
                n += 1
    assert n > 150


def test_smart_bitexact(fx):
    z, y = fx["smart_z"], fx["smart_y"]
    switches = set()
    for i, th in enumerate(fx["smart_thresh"]):
        for b in range(z.shape[0]):
            got = O.t32_simulate_smart_full(z[b], y[b], float(th), math.sqrt(2))
            want = (fx["smart_res"][i, b], fx["smart_cum"][i, b], fx["smart_comp"][i, b],
                    fx["smart_sw"][i, b])
            assert got == want, (th, b)
            switches.add(got[3])
    assert -1 in switches and len(switches) > 4  # early, late and no switch all covered


def test_gT_sampler_and_thresholds(fx):
    for T in (10, 100):
        regs = [O.t32_simulate_alg_full(*O.t32_gT_sample(0, T, r), 0, math.sqrt(2))[0]
                for r in range(16)]
        assert np.array_equal(np.array(regs, F), fx[f"gT_T{T}_regrets"]), T
    g = O.t32_empirical_worst_case_thresholds(fx["gT_grid"], runs=8)
    assert [g[int(T)] for T in fx["gT_grid"]] == list(fx["gT_grid_g"])


def test_pairwise_sum_and_row_norms_match_numpy():
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 8, 9, 127, 128, 129, 1000, 8192, 8193, 20000):
        a = rng.random(n).astype(F)
        assert O.t32_sum(a) == np.sum(a), n
    for d in (1, 5, 8, 13, 31):
        z = rng.standard_normal((200, d)).astype(F)
        assert np.array_equal(O.t32_row_norms(z), np.linalg.norm(z, axis=1)), d


def _host_blas_like_this_image() -> bool:
    rng = np.random.default_rng(11)
    for _ in range(200):
        a = rng.standard_normal(5).astype(F)
        b = rng.standard_normal(5).astype(F)
        if np.dot(a, b) != O.t32_sdot(a, b):
            return False
    z = rng.standard_normal((13, 5)).astype(F)
    x = rng.standard_normal(5).astype(F)
    return bool(np.array_equal(z @ x, O.t32_gemv(z, x)))


def test_numpy_calls_reproduce_fixtures(fx):
    if not _host_blas_like_this_image():
        pytest.skip("host BLAS orders sdot/sgemv differently from the image the fixtures came from")
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_twin32",
                                                  os.path.join(HERE, "golden", "make_twin32.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    for key in ("alg_T100", "fam", "dim8"):
        z, y = fx[key + "_z"], fx[key + "_y"]
        for i, (a, e) in enumerate(fx[key + "_runs"]):
            for b in range(z.shape[0]):
                assert mk.np_simulate_alg(z[b], y[b], int(a), float(e))[0] == fx[key + "_res"][i, b]
    z, y = fx["smart_z"], fx["smart_y"]
    for i, th in enumerate(fx["smart_thresh"][:3]):
        assert mk.np_simulate_smart(z[0], y[0], float(th), math.sqrt(2))[0] == fx["smart_res"][i, 0]

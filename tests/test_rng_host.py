"""CPU check of the device RNG source (csrc/ocx_rng.h) against NumPy itself.

The header is compiled for the host with g++ (it is __host__ __device__ code) and
compared with NumPy 2.x's SeedSequence / PCG64 / ziggurat / choice — the
third-party code that owns the reference's RNG arithmetic (fast_algorithms.py:254).
The GPU build of the same header is checked in tests/test_gpu_parity.py.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "rng_host.cpp")
OUT = os.path.join(ROOT, "build", "tests", "librng_host.so")


@pytest.fixture(scope="module")
def lib():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hdr = os.path.join(ROOT, "online_convex_optimization_amd", "csrc", "ocx_rng.h")
    if (not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC),
                                                               os.path.getmtime(hdr))):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                        SRC, "-o", OUT, "-lm"], check=True)
    L = ctypes.CDLL(OUT)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    dp = ctypes.POINTER(ctypes.c_double)
    L.h_seedseq_state4.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, u64p]
    L.h_raw.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_int64, u64p]
    L.h_normals.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_int64, dp]
    L.h_gT.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, dp, dp]
    L.h_log1p.argtypes = [dp, ctypes.c_int64, dp]
    return L


def _u64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


@pytest.mark.parametrize("entropy", [[0, 100, 0], [0, 1000, 999], [3, 7, 123456],
                                     [2**32 + 5, 10, 1], [0, 0, 0], [1, 2, 3, 4, 5, 6]])
def test_seedsequence(lib, entropy):
    ss = np.random.SeedSequence(entropy)
    words = np.concatenate([np.array([v & 0xFFFFFFFF] + ([v >> 32] if v >> 32 else []),
                                     dtype=np.uint32) for v in entropy])
    out = np.zeros(4, dtype=np.uint64)
    lib.h_seedseq_state4(words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(words),
                         _u64p(out))
    assert np.array_equal(out, ss.generate_state(4, np.uint64))


@pytest.mark.parametrize("seed", [(0, 100, 0), (0, 10000, 77), (5, 3, 2**40)])
def test_pcg64_raw(lib, seed):
    out = np.zeros(1000, dtype=np.uint64)
    lib.h_raw(*seed, 1000, _u64p(out))
    ref = np.random.PCG64(np.random.SeedSequence(list(seed))).random_raw(1000)
    assert np.array_equal(out, ref)


def test_ziggurat_normals(lib):
    n = 200000  # ~50 tail / rejection events
    out = np.zeros(n)
    lib.h_normals(0, 1000, 3, n, _dp(out))
    ref = np.random.Generator(np.random.PCG64(np.random.SeedSequence([0, 1000, 3]))
                              ).standard_normal(n)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("T,d,run", [(100, 5, 0), (57, 5, 3), (33, 1, 2), (20, 8, 1),
                                     (10, 64, 4), (5, 129, 0), (4, 300, 1), (3, 1024, 7)])
def test_gT_sampler(lib, T, d, run):
    z = np.zeros((T, d))
    y = np.zeros(T)
    lib.h_gT(0, T, run, d, _dp(z), _dp(y))
    gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence([0, T, run])))
    zr = gen.standard_normal((T, d))
    nr = np.linalg.norm(zr, axis=1, keepdims=True)
    zr *= (1.0 / np.maximum(nr, 1.0))
    yr = gen.choice([-1.0, 1.0], size=T)
    assert np.array_equal(z, zr)
    assert np.array_equal(y, yr)


def test_log1p_matches_libm(lib):
    """The ziggurat tail uses log1p(-u), u in [0, 1): the restatement must equal the host
    libm (what NumPy calls) bit for bit, not just to 1 ulp."""
    import math
    rng = np.random.default_rng(3)
    x = np.concatenate([-rng.random(400000), -rng.random(50000) * 1e-3,
                        -np.ldexp(rng.random(50000), -rng.integers(20, 60, 50000)),
                        rng.random(50000) * 3.0, [0.0, -0.0, -0.5, -1e-300, 1e300, -1.0]])
    out = np.zeros_like(x)
    lib.h_log1p(_dp(x), len(x), _dp(out))
    ref = np.array([math.log1p(v) if v > -1.0 else (-math.inf) for v in x])
    assert np.array_equal(out, ref)

"""Sequence families and stream builders (reference: sequence_generation.py).

Same names, signatures and outputs (float32 arrays, NumPy streams via ``_rng``) as
the reference module, so ``fast_driver.py``-style code can import either.  These
build one sequence at a time on the host, as the reference does.  The batched drivers
do not use them: the g(T) adversary (``engine.DeviceBatch.generate_gT``) and the four
families below (``engine.DeviceBatch.generate_family``, ``ocx_dev_gen_family``) are
generated on device, bit-identical to these builders (tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import numpy as np

from .fast_algorithms import _rng

Sample = Tuple[np.ndarray, np.ndarray, np.ndarray]


def flip_sequence(T: int, d: int = 5) -> Sample:
    """sequence_generation.py:24-28: z = e1, labels alternate -1, +1, -1, ..."""
    z = np.zeros((T, d), dtype=np.float32)
    z[:, 0] = 1.0
    y = np.where(np.arange(1, T + 1) % 2 == 1, 1.0, -1.0).astype(np.float32)
    return z, y, np.zeros(d, dtype=np.float32)


def switching_two_leaders_sequence(T: int, *, block_len: int = 20, d: int = 5) -> Sample:
    """sequence_generation.py:36-47: z = e1, labels in blocks of +1 / -1 of block_len."""
    blocks = np.arange(T) // max(int(block_len), 1)
    y = np.where(blocks % 2 == 0, 1.0, -1.0).astype(np.float32)
    z = np.zeros((T, d), dtype=np.float32)
    z[:, 0] = 1.0
    return z, y, np.zeros(d, dtype=np.float32)


def _unit(run_seed: int, stream: int, d: int) -> np.ndarray:
    u = _rng(run_seed, 0, stream).standard_normal(d).astype(np.float32, copy=False)
    n = float(np.linalg.norm(u))
    if n > 0:
        u /= n
    return u


def _clipped_rows(gen: np.random.Generator, T: int, d: int) -> np.ndarray:
    z = gen.standard_normal((T, d)).astype(np.float32, copy=False)
    norms = np.linalg.norm(z, axis=1, keepdims=True).astype(np.float32, copy=False)
    np.maximum(norms, 1.0, out=norms)
    z *= (1.0 / norms)
    return z


def _labels(z: np.ndarray, u: np.ndarray) -> np.ndarray:
    y = np.sign(z @ u).astype(np.float32, copy=False)
    y[y == 0.0] = 1.0
    return y


def make_random_iid_stream(*, d: int = 5, run_seed: int = 0) -> Callable[[int, int], Sample]:
    """sequence_generation.py:54-69: separable i.i.d. rows, y = sign(z.u)."""
    u = _unit(run_seed, 11, d)

    def sample(T: int, rep: int = 0) -> Sample:
        z = _clipped_rows(_rng(run_seed, T, 13 + rep), T, d)
        return z, _labels(z, u), u
    return sample


def make_noisy_iid_stream(*, p: float, d: int = 5, run_seed: int = 0
                          ) -> Callable[[int, int], Sample]:
    """sequence_generation.py:72-89: as above with Massart label noise rate p."""
    u = _unit(run_seed, 21, d)

    def sample(T: int, rep: int = 0) -> Sample:
        gen = _rng(run_seed, T, 23 + rep)
        z = _clipped_rows(gen, T, d)
        y = _labels(z, u)
        y[gen.random(T) < p] *= -1.0
        return z, y, u
    return sample


def make_flip_stream(*, d: int = 5, run_seed: int = 0) -> Callable[[int, int], Sample]:
    """sequence_generation.py:91-94."""
    return lambda T, rep=0: flip_sequence(T, d=d)


def make_switching_two_leaders_stream(*, block_len: int = 20, d: int = 5, run_seed: int = 0
                                      ) -> Callable[[int, int], Sample]:
    """sequence_generation.py:96-99."""
    return lambda T, rep=0: switching_two_leaders_sequence(T, block_len=block_len, d=d)


CASES: Dict[str, Callable[..., Callable[[int, int], Sample]]] = {
    "Random i.i.d. (separable)": lambda *, run_seed: make_random_iid_stream(d=5, run_seed=run_seed),
    "Massart noise 10%": lambda *, run_seed: make_noisy_iid_stream(p=0.10, d=5, run_seed=run_seed),
    "Label flips": lambda *, run_seed: make_flip_stream(d=5, run_seed=run_seed),
    "Switching leaders": lambda *, run_seed: make_switching_two_leaders_stream(
        block_len=20, d=5, run_seed=run_seed),
}

RUNS_BY_TITLE = {"Random i.i.d. (separable)": 48, "Massart noise 10%": 48,
                 "Label flips": 1, "Switching leaders": 1}
REPLICATES_BY_TITLE = {"Random i.i.d. (separable)": 16, "Massart noise 10%": 20,
                       "Label flips": 1, "Switching leaders": 1}

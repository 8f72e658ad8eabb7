"""Multi-GPU sharding of independent sequences: one process per GPU, torch.distributed.

The sequences of a sweep are independent streams ``_rng(base_seed, T, run)``
(fast_algorithms.py:254-257), so ranks take disjoint contiguous run ranges and
regenerate and simulate them on their own GPU with no data-path collective.  The
path's only exchange is the result collection at the end: one all-gather of the
per-run regrets (RCCL over xGMI with the "nccl" backend; gloo in CPU tests) from which
every rank gets the full regret vector and g(T) = max(0, max regrets).
"""
from __future__ import annotations

from typing import Callable, Dict, Sequence, Tuple

import numpy as np


def shard(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, start+count) share of ``total`` items for ``rank``."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def all_gather_ragged(local, world: int, total: int, device=None):
    """All-gather 1-D float64 shards made by ``shard(total, ., world)`` into [total]."""
    import torch
    import torch.distributed as dist
    width = -(-int(total) // int(world))
    buf = torch.zeros(width, dtype=torch.float64, device=device)
    buf[: local.numel()] = local
    out = torch.zeros(width * world, dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(out, buf)
    parts = []
    for r in range(world):
        _, cnt = shard(total, r, world)
        parts.append(out[r * width: r * width + cnt])
    return torch.cat(parts)


def max_regret(regrets) -> float:
    """fast_algorithms.py:228, :242-243 (max over runs, starting from 0.0)."""
    r = np.asarray(regrets, dtype=np.float64)
    pos = r[r > 0.0]
    return float(pos.max()) if pos.size else 0.0


def gT_sweep_distributed(T_grid: Sequence[int], runs: int, *, base_seed: int = 0, d: int = 5,
                         compute: Callable[[int, int, int], np.ndarray] = None,
                         device=None, lanes_per_seq: int = 128
                         ) -> Dict[int, Tuple[float, np.ndarray]]:
    """empirical_worst_case_thresholds across the ranks of the default process group.

    ``compute(T, run0, count)`` returns this rank's regrets (default: regenerate and
    simulate on the local GPU through engine.gT_regrets).  ``device`` is where the gather
    runs: the rank's current GPU under the "nccl" (RCCL) backend, host memory otherwise.
    ``lanes_per_seq`` as engine.gT_regrets (default OCX_LANES_BEST; 1 = bit-exact).
    Returns, on every rank, {T: (g(T), regrets[runs] in run order)}."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if device is None and dist.get_backend() == "nccl":
        # RCCL gathers device tensors only: collect on this rank's GPU
        device = torch.device("cuda", torch.cuda.current_device())
    if compute is None:
        from . import engine
        dev_index = torch.cuda.current_device()

        def compute(T, run0, count):
            return engine.gT_regrets(T, count, base_seed=base_seed, d=d, run0=run0,
                                     lanes_per_seq=lanes_per_seq, device=dev_index)
    out = {}
    for T in T_grid:
        T = int(T)
        run0, cnt = shard(runs, rank, world)
        local = torch.as_tensor(np.asarray(compute(T, run0, cnt), dtype=np.float64))
        if device is not None:
            local = local.to(device)
        full = all_gather_ragged(local, world, runs, device=local.device).cpu().numpy()
        out[T] = (max_regret(full), full)
    return out

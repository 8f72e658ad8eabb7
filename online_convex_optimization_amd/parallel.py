"""Multi-GPU sharding of independent sequences: one process per GPU, torch.distributed.

The sequences of a sweep are independent streams ``_rng(base_seed, T, run)``
(fast_algorithms.py:254-257), so ranks take disjoint contiguous run ranges and
regenerate and simulate them on their own GPU with no data-path collective.  The
path's only exchange is the result collection at the end, and it never leaves HBM under
RCCL: for g(T) alone one all_reduce(MAX) of one double per T (each rank's max reduced on
its GPU); for the regret curves one all-gather of the device-resident per-run regrets
(RCCL over xGMI with the "nccl" backend; gloo in CPU tests).
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
                         compute_max: Callable[[int, int, int], float] = None,
                         device=None, lanes_per_seq: int = 128, return_regrets: bool = True,
                         as_tensor: bool = False) -> Dict[int, Tuple[float, object]]:
    """empirical_worst_case_thresholds (fast_algorithms.py:211-247) across the ranks of the
    default process group; rank r takes the contiguous run shard ``shard(runs, r, world)``.

    ``return_regrets=False`` (what the reference's function returns, g(T) only): each rank
    reduces its shard's max on its own GPU (engine.gT_max → ocx_gT_max; no regret leaves
    the GPU) and one all_reduce(MAX) of one double per T combines the ranks:
    max_r max(0, shard max) == max(0, max over all runs), bit for bit.

    ``return_regrets=True``: the regret curves too.  Each rank's regrets stay in HBM
    (engine.gT_regrets_device → ocx_gT_regrets_dev) and are all-gathered device to device
    (RCCL over xGMI under the "nccl" backend; a host-memory gather under gloo, whose
    collectives are host-side); g(T) is then reduced from the gathered tensor.

    ``compute(T, run0, count)`` / ``compute_max(T, run0, count)`` replace the GPU work (CPU
    tests: the oracle).  ``device``: where the gather runs (default: this rank's GPU under
    nccl, host memory otherwise).  ``lanes_per_seq`` as engine.gT_regrets (default
    OCX_LANES_BEST; 1 = bit-exact).  Returns, on every rank, {T: (g(T), regrets)} with
    regrets [runs] in run order — a numpy array, a torch tensor on the gather device with
    ``as_tensor``, or None without ``return_regrets``."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    if device is None and nccl:
        # RCCL reduces and gathers device tensors only: collect on this rank's GPU
        device = torch.device("cuda", torch.cuda.current_device())
    if device is None:
        device = torch.device("cpu")
    gpu_compute = compute is None
    if gpu_compute:
        from . import engine
        dev_index = torch.cuda.current_device()
    out = {}
    for T in T_grid:
        T = int(T)
        run0, cnt = shard(runs, rank, world)
        if not return_regrets:
            if compute_max is not None:
                m = float(compute_max(T, run0, cnt))
            elif gpu_compute:
                m = engine.gT_max(T, cnt, base_seed=base_seed, d=d, run0=run0,
                                  lanes_per_seq=lanes_per_seq, device=dev_index)
            else:
                m = max_regret(compute(T, run0, cnt))
            g = torch.tensor([m], dtype=torch.float64, device=device)
            dist.all_reduce(g, op=dist.ReduceOp.MAX)
            out[T] = (float(g.item()), None)
            continue
        if gpu_compute:
            local = engine.gT_regrets_device(T, cnt, base_seed=base_seed, d=d, run0=run0,
                                             lanes_per_seq=lanes_per_seq, device=dev_index)
            if local.device != device:
                local = local.to(device)
        else:
            local = torch.as_tensor(np.asarray(compute(T, run0, cnt), dtype=np.float64)).to(device)
        full = all_gather_ragged(local, world, runs, device=device)
        # fast_algorithms.py:228, :242-243: max over runs starting from 0.0 (NaN never wins)
        pos = full[full > 0.0]
        g = float(pos.max().item()) if pos.numel() else 0.0
        out[T] = (g, full if as_tensor else full.cpu().numpy())
    return out

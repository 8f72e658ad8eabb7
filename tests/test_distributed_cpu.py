"""World-size-2 gloo tests of the multi-rank path (CPU only, no GPU needed).

Each rank computes its shard of runs with the CPU oracle standing in for its GPU
(tests may use the oracle as the checker); the sharding, the ragged all-gather and
the g(T) reduction are the product code in online_convex_optimization_amd.parallel.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from online_convex_optimization_amd.parallel import max_regret, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, T_grid, runs, q):
    import torch.distributed as dist
    from oracle import oracle as O
    from online_convex_optimization_amd.parallel import gT_sweep_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def compute(T, run0, count):
        return np.array([O.simulate_alg(*O.gT_sample(0, T, r, 5), 0, math.sqrt(2))
                         for r in range(run0, run0 + count)])
    res = gT_sweep_distributed(T_grid, runs, compute=compute)
    # g(T) alone: each rank's shard max, one all_reduce(MAX) of one double per T
    gonly = gT_sweep_distributed(T_grid, runs, compute=compute,
                                 compute_max=lambda T, r0, n: max(0.0, float(np.max(
                                     compute(T, r0, n), initial=0.0))),
                                 return_regrets=False)
    q.put((rank, {T: (g, regs.tolist(), gonly[T]) for T, (g, regs) in res.items()}))
    dist.destroy_process_group()


def _bench_report_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 5
    regrets = np.random.default_rng(rank).standard_normal(B)
    gathered = torch.zeros(world * B, dtype=torch.float64)
    dist.all_gather_into_tensor(gathered, torch.from_numpy(regrets))
    ident = {"device_index": rank, "name": "cpu-stand-in", "pci": f"0000:{rank + 0x10:02x}:00",
             "uuid": None}
    rep = bench.rank_report(dist, rank, world, ident, 0.25 + rank, 1.5, regrets,
                            gathered.numpy())
    bad = gathered.numpy().copy()
    bad[-1] += 1.0  # the last rank's block corrupted
    rep_bad = bench.rank_report(dist, rank, world, ident, 0.25, 1.5, regrets, bad)
    q.put((rank, rep, rep_bad["gathered_check"], rep_bad["gathered_blocks_ok"]))
    dist.destroy_process_group()


def test_bench_rank_report_world2():
    """bench.py's multi-rank self-check (what the 8-GPU SCALE run prints): world size,
    every rank's device identity, wall time and kernel time, and a gathered_check that
    compares every rank's block of the gathered regrets with that rank's own checksum."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_bench_report_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, rep, bad_ok, bad_blocks = q.get(timeout=300)
        res[r] = (rep, bad_ok, bad_blocks)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rep, bad_ok, bad_blocks = res[0]
    assert rep["world_size"] == 2 and rep["distinct_devices"] == 2
    assert rep["gathered_check"] is True and rep["gathered_blocks_ok"] == [True, True]
    assert [r["rank"] for r in rep["ranks"]] == [0, 1]
    assert [r["device_index"] for r in rep["ranks"]] == [0, 1]
    assert [r["elapsed_ms"] for r in rep["ranks"]] == [250.0, 1250.0]
    assert all(r["kernel_ms"] == 1.5 and r["n_regrets"] == 5 for r in rep["ranks"])
    assert bad_ok is False and bad_blocks == [True, False]


def test_shard_covers_exactly():
    for total in (0, 1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard(total, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c


def test_max_regret_semantics():
    assert max_regret([-1.0, -2.0]) == 0.0
    assert max_regret([0.5, float("nan"), 2.0]) == 2.0


@pytest.mark.parametrize("world", [2])
def test_gT_sweep_world2_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    T_grid, runs = [30, 100], 7  # odd run count: ragged shards
    procs = [ctx.Process(target=_worker, args=(r, world, port, T_grid, runs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import oracle as O
    ref = O.empirical_worst_case_thresholds(T_grid, runs=runs)
    for rank in range(world):
        for T in T_grid:
            g, regs, (g_only, none) = results[rank][T]
            assert g == ref[T] and g_only == ref[T] and none is None
            assert len(regs) == runs
            assert regs == results[0][T][1]

"""GPU: the product's multi-device code paths on a one-GPU box.

* parallel.gT_sweep_distributed with its DEFAULT compute (device-resident regrets from
  engine.gT_regrets_device on the rank's GPU, or ocx_gT_max + one all_reduce(MAX) for g(T)
  alone), world_size 2 over gloo, both ranks on device 0, ragged shards;
* the same over the "nccl" backend (RCCL) with world_size 1: RCCL initialisation and the
  device all-gather run for real (two ranks cannot share one GPU under RCCL);
* engine.gT_sweep(devices=[0, 0]): one process driving a device list from threads.

Each is compared with one engine.gT_regrets call over all runs and with the oracle on
sampled runs.  The sequences are independent streams _rng(seed, T, run)
(fast_algorithms.py:254-257), so sharding must be bit-invisible."""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle as O

pytestmark = pytest.mark.gpu
SQ2 = math.sqrt(2)
T_GRID, RUNS, D = [40, 257], 37, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, backend, q):
    import torch
    import torch.distributed as dist
    from online_convex_optimization_amd.parallel import gT_sweep_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = gT_sweep_distributed(T_GRID, RUNS, base_seed=3, d=D)
        # regret curves gathered device to device, kept as tensors
        tens = gT_sweep_distributed(T_GRID, RUNS, base_seed=3, d=D, as_tensor=True)
        dev_ok = all(isinstance(v, torch.Tensor) and v.dtype == torch.float64 and
                     v.device.type == ("cuda" if backend == "nccl" else "cpu")
                     for _, v in tens.values())
        same = all(np.array_equal(tens[T][1].cpu().numpy(), res[T][1]) and
                   tens[T][0] == res[T][0] for T in T_GRID)
        # g(T) alone: ocx_gT_max per rank + one all_reduce(MAX)
        gonly = gT_sweep_distributed(T_GRID, RUNS, base_seed=3, d=D, return_regrets=False)
        q.put((rank, {T: (g, regs.tolist(), gonly[T][0], gonly[T][1] is None, dev_ok and same)
                      for T, (g, regs) in res.items()}))
    finally:
        dist.destroy_process_group()


def _run(world, backend):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=90) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return results


@pytest.fixture(scope="module")
def reference():
    from online_convex_optimization_amd import engine
    ref = {T: engine.gT_regrets(T, RUNS, base_seed=3, d=D) for T in T_GRID}
    for T in T_GRID:
        for r in (0, RUNS // 2, RUNS - 1):
            z, y = O.gT_sample(3, T, r, D)
            # default mode: closed-form comparator (tests/test_gpu_parity.py close_closed)
            want = O.simulate_alg(z, y, 0, SQ2)
            assert abs(ref[T][r] - want) <= max(1e-12 * max(1.0, abs(want)), 9e-16 * T ** 1.5)
    return ref


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (1, "nccl")])
def test_gT_sweep_distributed_default_compute(reference, world, backend):
    results = _run(world, backend)
    for rank in range(world):
        for T in T_GRID:
            g, regs, g_only, none, tens_ok = results[rank][T]
            assert np.array_equal(np.array(regs), reference[T]), (backend, rank, T)
            assert g == max(0.0, float(reference[T].max()))
            assert g_only == g and none and tens_ok, (backend, rank, T)


def test_gT_sweep_device_list(reference):
    from online_convex_optimization_amd import engine
    out = engine.gT_sweep(T_GRID, RUNS, base_seed=3, d=D, devices=[0, 0])
    for T in T_GRID:
        g, regs = out[T]
        assert np.array_equal(regs, reference[T])
        assert g == max(0.0, float(reference[T].max()))


def test_gT_max_on_device(reference):
    """ocx_gT_max / gT_sweep(return_regrets=False): the max reduced on device (an atomic max
    over bit patterns) equals the max of the regrets the host receives, bit for bit, on one
    device, on a device list, and through the streamed (T-chunked) path."""
    from online_convex_optimization_amd import engine
    for T in T_GRID:
        want = max(0.0, float(reference[T].max()))
        assert engine.gT_max(T, RUNS, base_seed=3, d=D) == want
        # ragged shards of one run range
        assert max(engine.gT_max(T, 20, base_seed=3, d=D),
                   engine.gT_max(T, RUNS - 20, base_seed=3, d=D, run0=20)) == want
    out = engine.gT_sweep(T_GRID, RUNS, base_seed=3, d=D, devices=[0, 0], return_regrets=False)
    for T in T_GRID:
        g, regs = out[T]
        assert regs is None and g == max(0.0, float(reference[T].max()))
    os.environ["OCX_HBM_BUDGET_GB"] = "0.0004"  # forces the streamed path (T-chunks)
    try:
        for T in T_GRID:
            assert engine.gT_max(T, RUNS, base_seed=3, d=D) == max(0.0, float(reference[T].max()))
    finally:
        del os.environ["OCX_HBM_BUDGET_GB"]
    assert engine.gT_max(T_GRID[0], 0, base_seed=3, d=D) == 0.0


def test_gT_regrets_device(reference, monkeypatch):
    """engine.gT_regrets_device (ocx_gT_regrets_dev): the regrets land in a device tensor,
    bit-identical to the host-array entry point, on the resident and the streamed path."""
    import torch
    from online_convex_optimization_amd import engine
    for T in T_GRID:
        t = engine.gT_regrets_device(T, RUNS, base_seed=3, d=D)
        assert t.is_cuda and np.array_equal(t.cpu().numpy(), reference[T])
        sub = torch.full((RUNS - 5,), -7.0, dtype=torch.float64, device="cuda")
        engine.gT_regrets_device(T, RUNS - 5, base_seed=3, d=D, run0=5, out=sub)
        assert np.array_equal(sub.cpu().numpy(), reference[T][5:])
    monkeypatch.setenv("OCX_HBM_BUDGET_GB", "0.0004")  # streamed path (T-chunks)
    t = engine.gT_regrets_device(T_GRID[1], RUNS, base_seed=3, d=D)
    assert np.array_equal(t.cpu().numpy(), reference[T_GRID[1]])
    with pytest.raises(ValueError):
        engine.gT_regrets_device(40, 3, out=torch.zeros(4, dtype=torch.float64, device="cuda"))

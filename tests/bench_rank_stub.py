"""Rank body for tests/test_bench_launcher.py: what `bench.py --gpus N` runs per rank, with
the GPU work stubbed out.  The launcher (bench.launch_ranks) starts this file as N ranks;
each takes its place from bench.rank_env exactly as bench.main does, joins a gloo group and
rank 0 prints one JSON line with the world size and every rank's identity.  Rank 0 then runs
bench.cpu_leg — the CPU baseline and the parity check the bench line carries at every world
size — on its own shard's regrets (here computed by the oracle in place of the GPU kernel, so
the check must come out bit-exact)."""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse()
    world, rank, local, gpu, dist_on = bench.rank_env(a, 0)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rows = [None] * world
    dist.all_gather_object(rows, {"rank": rank, "local_rank": local, "gpu": gpu,
                                  "pid": os.getpid(), "dist_on": dist_on})
    cpu = parity = None
    if rank == 0 and a.cpu_seconds > 0:
        from oracle import oracle as O
        regrets = np.array([O.simulate_alg(*O.gT_sample(0, a.T, r, a.d), 0, math.sqrt(2))
                            for r in range(a.B)])
        cpu, parity = bench.cpu_leg(a, a.T, a.d, a.B, regrets)
    if rank == 0:
        print(json.dumps({"world_size": dist.get_world_size(), "ranks": rows,
                          "cpu_baseline": cpu, "parity": parity}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

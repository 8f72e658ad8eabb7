"""FTRL kernel timing probe (round 3): the resident batches the g(T) sweeps and configs run,
default layout (OCX_LANES_BEST), closed-form comparator.  One JSON line per batch.  Run it
twice, with and without OCX_ALG_NO_PIPE=1, to compare the pipelined butterfly kernel with
the plain one (the switch is read once per process)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def main():
    shapes = [(4900, 100000, 64, engine.LANES_BEST), (4900, 100000, 64, 16),
              (3328, 100000, 64, engine.LANES_BEST), (3400, 10000, 1024, engine.LANES_BEST),
              (2048, 10000, 1024, engine.LANES_BEST), (32768, 10000, 64, engine.LANES_BEST)]
    if os.environ.get("OCX_PROBE_SHORT"):
        shapes = shapes[:3]
    pipe = not os.environ.get("OCX_ALG_NO_PIPE")
    for B, T, d, lanes in shapes:
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes).generate_gT(base_seed=0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for closed, algo in ((True, 0), (False, 0), (True, 1)):
            db.simulate_alg(algo, math.sqrt(2), closed_comparator=closed)
            torch.cuda.synchronize()
            ev[0].record()
            reps = 3
            for _ in range(reps):
                db.simulate_alg(algo, math.sqrt(2), closed_comparator=closed)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / reps
            passes = 1 if closed else 2
            gbs = B * T * (8 * d + 8) * passes / (ms * 1e-3) / 1e9
            print(json.dumps({"B": B, "T": T, "d": d, "layout": [db.L.P, db.L.C, db.L.chain],
                              "pipe": pipe, "closed": closed, "algo": algo, "kernel_ms": ms,
                              "GBps": gbs, "frac": gbs / 8000.0,
                              "regret0": float(db.regret[0].item())}), flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

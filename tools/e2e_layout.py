"""End-to-end layout probe (round 3; rerun by tools/evidence.sh): generation + FTRL (closed-form comparator) of one
resident d = 64 batch under several lane layouts.  One JSON line per layout: generator ms,
FTRL ms, timesteps/s of the pair.
    python tools/e2e_layout.py [B] [T] [lanes,...]   (lanes 128 = OCX_LANES_BEST)"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    lanes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [128, 8, 16]
    d = 64
    for lp in lanes:
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=lp)
        g_ms = timed(lambda: db.generate_gT(base_seed=0))
        a_ms = timed(lambda: db.simulate_alg(0, math.sqrt(2), closed_comparator=True))
        print(json.dumps({"B": B, "T": T, "d": d, "lanes_per_seq": lp,
                          "layout": [db.L.P, db.L.C, db.L.chain], "gen_ms": g_ms, "ftrl_ms": a_ms,
                          "timesteps_per_s": B * T / ((g_ms + a_ms) * 1e-3),
                          "ftrl_frac": B * T * (8 * d + 8) / (a_ms * 1e-3) / 8e12}), flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

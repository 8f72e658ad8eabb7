"""BASELINE configs[3] and configs[4] at their full trial counts on one GPU (the 8-GPU runs shard
the same runs over ranks): g(T) = max(0, max over runs of the FTRL regret) on the g(T) adversary,
generation included, through engine.gT_max.  One JSON line per (d, T).
    python tools/full_configs.py [--runs3 1000000] [--runs4 100000] [--T3 100,1000,10000,100000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs3", type=int, default=1000000)
    ap.add_argument("--runs4", type=int, default=100000)
    ap.add_argument("--T3", default="100,1000,10000,100000")
    a = ap.parse_args()
    from online_convex_optimization_amd import engine
    jobs = [(64, int(T), a.runs3, "configs[3]") for T in a.T3.split(",")]
    jobs.append((1024, 10000, a.runs4, "configs[4]"))
    for d, T, runs, name in jobs:
        # warm: kernels, library streams and the HBM buffers at the batch size this call takes
        # (a run count that fills the budget-sized batch; the first call of a process pays the
        # allocation, reported as cold_seconds)
        warm = min(runs, max(4096, (240 << 30) // (T * (8 * d + 8)) + 1))  # a budget-sized batch
        t0 = time.perf_counter()
        engine.gT_max(T, warm, d=d)
        cold = time.perf_counter() - t0
        t0 = time.perf_counter()
        g = engine.gT_max(T, runs, d=d)
        dt = time.perf_counter() - t0
        print(json.dumps({"what": "full_config", "config": name, "d": d, "T": T, "runs": runs,
                          "seconds": dt, "timesteps_per_s": T * runs / dt, "g": g,
                          "warm_runs": warm, "cold_seconds": cold}), flush=True)


if __name__ == "__main__":
    main()

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
        engine.gT_max(T, min(runs, 4096), d=d)  # warm: kernels and library streams
        t0 = time.perf_counter()
        g = engine.gT_max(T, runs, d=d)
        dt = time.perf_counter() - t0
        print(json.dumps({"what": "full_config", "config": name, "d": d, "T": T, "runs": runs,
                          "seconds": dt, "timesteps_per_s": T * runs / dt, "g": g}), flush=True)
        engine.release_buffers()


if __name__ == "__main__":
    main()

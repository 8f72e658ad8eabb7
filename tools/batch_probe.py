"""g(T) calls whose runs span one, two or three budget-sized batches (d = 64): where the
multi-batch path's time goes.  Each shape warmed with itself.  One JSON line per (T, runs).
    python tools/batch_probe.py [--T 1000] [--runs 495574,495575,600000,1000000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--runs", default="495574,495575,600000,1000000")
    ap.add_argument("--fn", default="gT_max")
    a = ap.parse_args()
    from online_convex_optimization_amd import engine
    fn = getattr(engine, a.fn)
    for runs in (int(x) for x in a.runs.split(",")):
        t0 = time.perf_counter()
        fn(a.T, runs, d=64)
        first = time.perf_counter() - t0
        best = 1e9
        for _ in range(2):
            t0 = time.perf_counter()
            fn(a.T, runs, d=64)
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"what": "batch_probe", "fn": a.fn, "T": a.T, "runs": runs, "seconds": best, "first_call_seconds": first,
                          "timesteps_per_s": a.T * runs / best}), flush=True)


if __name__ == "__main__":
    main()

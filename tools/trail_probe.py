"""The trailing pipeline (ocx_pipeline.hip ocx_run_gen_sim_trailing) against the sequential
generate-then-simulate loop on the capacity-limited g(T) batches: configs[4] (d = 1024,
T = 1e4) and configs[3]'s T = 1e5 point (d = 64).  One JSON line per (case, mode): seconds and
timesteps/s of engine.gT_max (what empirical_worst_case_thresholds runs per T), after a warm
call of the same shape, and whether the regrets equal the sequential loop's bit for bit.

    python tools/trail_probe.py [--cases c4,t1e5] [--chunks 8,4,16] [--runs-c4 32768] [--runs-t5 131072]
                                [--check 0] [--only-trailing] [--ramps 4,0]

--ramps: the trailing modes are run for every (chunks, ramp) pair; ramp = OCX_TRAIL_RAMP, the
first chunk of the doubling ramp in 64-step blocks (0 = equal chunks, as before round 6).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {"c4": (10000, 1024), "t1e5": (100000, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c4,t1e5")
    ap.add_argument("--chunks", default="12")
    ap.add_argument("--runs-c4", type=int, default=32768)
    ap.add_argument("--runs-t5", type=int, default=131072)
    ap.add_argument("--check", type=int, default=1, help="compare regrets with the sequential loop")
    ap.add_argument("--only-trailing", action="store_true", help="skip the sequential mode (PMC passes)")
    ap.add_argument("--ramps", default="", help="OCX_TRAIL_RAMP values per trailing mode ('' = the default)")
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    for case in a.cases.split(","):
        T, d = CASES[case]
        runs = a.runs_c4 if case == "c4" else a.runs_t5
        ref = None
        modes = [] if a.only_trailing else [("sequential", "0", None)]
        ramps = a.ramps.split(",") if a.ramps else [None]
        modes += [("trailing", "1", c, r) for c in a.chunks.split(",") for r in ramps]
        modes = [m if len(m) == 4 else (*m, None) for m in modes]
        for name, trail, chunks, ramp in modes:
            os.environ["OCX_TRAILING"] = trail
            if chunks:
                os.environ["OCX_TRAIL_CHUNKS"] = chunks
            if ramp is not None:
                os.environ["OCX_TRAIL_RAMP"] = ramp
            else:
                os.environ.pop("OCX_TRAIL_RAMP", None)
            engine.gT_max(T, runs, d=d)  # warm: HBM buffers, kernels
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g = engine.gT_max(T, runs, d=d)
            dt = time.perf_counter() - t0
            same = None
            if a.check:
                r = engine.gT_regrets(T, runs, d=d)
                if ref is None:
                    ref = r
                same = bool(np.array_equal(r, ref))
            print(json.dumps({"what": "trail_probe", "case": case, "T": T, "d": d, "runs": runs,
                              "mode": name, "chunks": int(chunks) if chunks else None,
                              "ramp": None if ramp is None else int(ramp),
                              "seconds": dt, "timesteps_per_s": T * runs / dt,
                              "frac_of_16400B" if d == 1024 else "frac_of_1040B":
                                  T * runs / dt * 2 * (8 * d + 8) / 8e12,
                              "g": g, "regrets_equal_sequential": same}), flush=True)
        os.environ.pop("OCX_TRAIL_CHUNKS", None)
        os.environ.pop("OCX_TRAIL_RAMP", None)
        os.environ.pop("OCX_TRAILING", None)
        engine.release_buffers()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

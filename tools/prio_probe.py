"""Generator wave priority (OCX_GEN_PRIO, s_setprio; a round-6 experiment build — the knob is not
in the product library) where generation shares the SIMDs with an FTRL pass: the sub-batch pipeline at the bench shape (DeviceBatch.generate_simulate, 32 768 x 1e4
x 64, `steps` batches) and the trailing pipeline at T = 1e5 (engine.gT_max over 131 072 runs).
Regrets are compared with priority 0's.  One JSON line per (priority, case).
    python tools/prio_probe.py [--prios 0,1,2,3] [--cases pipe,t1e5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prios", default="0,1,2,3")
    ap.add_argument("--cases", default="pipe,t1e5")
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    prios = a.prios.split(",")
    ref = {}
    for case in a.cases.split(","):
        if case == "pipe":
            B, T, d = 32768, 10000, 64
            X = engine.DeviceBatch(B, T, d)
            for p in prios:
                os.environ["OCX_GEN_PRIO"] = p
                X.generate_simulate(0, 0, 1)  # warm
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(2):
                    t0 = time.perf_counter()
                    X.generate_simulate(0, 0, a.steps)
                    torch.cuda.synchronize()
                    best = min(best, time.perf_counter() - t0)
                reg = X.regret[:B].cpu().numpy().copy()
                r0 = ref.setdefault(case, reg)
                print(json.dumps({"what": "prio", "case": case, "prio": int(p), "B": B, "T": T, "d": d,
                                  "batches": a.steps, "ms_per_batch": best / a.steps * 1e3,
                                  "timesteps_per_s": B * T * a.steps / best,
                                  "regrets_equal_prio0": bool(np.array_equal(reg, r0))}), flush=True)
            del X
            torch.cuda.empty_cache()
        elif case == "t1e5":
            T, d, runs = 100000, 64, 131072
            for p in prios:
                os.environ["OCX_GEN_PRIO"] = p
                engine.gT_max(T, runs, d=d)  # warm: HBM buffers, kernels
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g = engine.gT_max(T, runs, d=d)
                dt = time.perf_counter() - t0
                r0 = ref.setdefault(case, g)
                print(json.dumps({"what": "prio", "case": case, "prio": int(p), "T": T, "d": d,
                                  "runs": runs, "seconds": dt, "timesteps_per_s": T * runs / dt,
                                  "g": g, "g_equal_prio0": g == r0}), flush=True)
            engine.release_buffers()
            torch.cuda.empty_cache()
    os.environ.pop("OCX_GEN_PRIO", None)


if __name__ == "__main__":
    main()

"""g(T) (on-device max) at several HBM budgets: how the resident batch size moves the
sweep (OCX_HBM_BUDGET_GB sets the batch; 0 = the default rule).  One JSON line each."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from online_convex_optimization_amd import engine
    cases = [(10000, 131072, b) for b in ("0", "160", "125", "200")] + \
            [(1000, 1000000, b) for b in ("0", "175", "130")]
    for T, runs, b in cases:
        if b == "0":
            os.environ.pop("OCX_HBM_BUDGET_GB", None)
        else:
            os.environ["OCX_HBM_BUDGET_GB"] = b
        engine.gT_max(T, runs, d=64)
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            g = engine.gT_max(T, runs, d=64)
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"T": T, "runs": runs, "budget_gb": b, "seconds": best,
                          "timesteps_per_s": T * runs / best, "g": g}), flush=True)


if __name__ == "__main__":
    main()

"""Timing of the float32 twin on the GPU: driver.py's workloads.

    python tools/twin32_probe.py > gpurun_out/twin32_probe.jsonl
"""
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import algorithms as A  # noqa: E402
from online_convex_optimization_amd import engine  # noqa: E402


def timed(fn, reps=3):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


def main():
    out = []
    grid = np.arange(100, 1100, 100)
    s = timed(lambda: A.empirical_worst_case_thresholds(grid, runs=1000), reps=1)
    out.append({"what": "empirical_worst_case_thresholds(T=100..1000, runs=1000)", "s": s})
    rng = np.random.default_rng(0)
    for T in (100, 1000):
        z = (rng.standard_normal((T, 5)) * 0.5).astype(np.float32)
        y = np.where(rng.random(T) < 0.5, -1.0, 1.0).astype(np.float32)
        out.append({"what": f"simulate_alg single call T={T}", "s": timed(lambda: A.simulate_alg(z, y, 0, math.sqrt(2)), 20)})
        out.append({"what": f"simulate_SMART single call T={T} (no switch)",
                    "s": timed(lambda: A.simulate_SMART_like(z, y, 1e9, math.sqrt(2)), 3)})
        for B in (1000, 16384):
            zb = (rng.standard_normal((B, T, 5)) * 0.5).astype(np.float32)
            yb = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0).astype(np.float32)
            out.append({"what": f"twin32_batch FTRL B={B} T={T}",
                        "s": timed(lambda: engine.twin32_batch(zb, yb, 0, math.sqrt(2)), 3)})
            out.append({"what": f"twin32_batch SMART B={B} T={T} (no switch)",
                        "s": timed(lambda: engine.twin32_batch(zb, yb, 2, math.sqrt(2), thresh=1e9), 1)})
    from online_convex_optimization_amd import drivers
    s = timed(lambda: drivers.driver_main(), reps=1)
    out.append({"what": "drivers.driver_main() (driver.py:204-226 without figures, defaults)", "s": s})
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

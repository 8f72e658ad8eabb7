"""g(T) regrets through the C entry point (generation + FTRL per resident batch) at small d:
OCX_LANES_BEST (butterfly lanes of two coordinates for 8 <= d < 64) against the exact layout
(lanes_per_seq=1).  One JSON line per (d, mode)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from online_convex_optimization_amd import engine
    T, runs = 1000, 65536
    for d in (5, 8, 16, 32):
        ref = None
        for name, lanes in (("best", engine.LANES_BEST), ("exact", 1)):
            engine.gT_regrets(T, 4096, base_seed=0, d=d, lanes_per_seq=lanes)  # warm up
            t0 = time.perf_counter()
            reg = engine.gT_regrets(T, runs, base_seed=0, d=d, lanes_per_seq=lanes)
            dt = time.perf_counter() - t0
            if ref is None:
                ref = reg
            print(json.dumps({"what": "gT_regrets", "d": d, "T": T, "runs": runs, "mode": name,
                              "seconds": dt, "timesteps_per_s": runs * T / dt,
                              "max_rel_vs_best": float(np.max(np.abs(reg - ref) / np.maximum(1, np.abs(ref))))}),
                  flush=True)


if __name__ == "__main__":
    main()

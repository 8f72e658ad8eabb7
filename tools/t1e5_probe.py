"""T = 1e5, d = 64 g(T) batch policy with the closed-form comparator: resident few-wave
batches (default) vs the streamed path (seek + generate chunk + FTRL chunk, no pass B),
and a few HBM budgets.  One JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from online_convex_optimization_amd import engine
    T, d = 100000, 64
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    cases = [("resident", {}), ("streamed", {"OCX_MIN_RESIDENT": str(1 << 30)}),
             ("streamed_120G", {"OCX_MIN_RESIDENT": str(1 << 30), "OCX_HBM_BUDGET_GB": "120"})]
    ref = None
    for name, env in cases:
        for k in ("OCX_MIN_RESIDENT", "OCX_HBM_BUDGET_GB"):
            os.environ.pop(k, None)
        os.environ.update(env)
        engine.release_buffers()
        engine.gT_regrets(T, 4096, d=d)  # warm kernels and buffers
        t0 = time.perf_counter()
        regs = engine.gT_regrets(T, runs, d=d)
        dt = time.perf_counter() - t0
        if ref is None:
            ref = regs
        import numpy as np
        print(json.dumps({"case": name, "T": T, "runs": runs, "d": d, "seconds": dt,
                          "timesteps_per_s": T * runs / dt, "frac_1040B": T * runs / dt * 1040 / 8e12,
                          "max_rel_vs_resident": float((np.abs(regs - ref) / np.maximum(1, np.abs(ref))).max())}),
              flush=True)


if __name__ == "__main__":
    main()

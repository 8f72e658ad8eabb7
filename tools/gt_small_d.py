"""g(T) regrets through the C entry point (generation + FTRL per resident batch) at small d:
OCX_LANES_BEST (butterfly lanes of two coordinates for 8 <= d < 64) against the exact layout
(lanes_per_seq=1).  One JSON line per (d, mode).  Then generation and FTRL apart per (d, lanes)
of --split (d:lanes, default the layouts gT_regrets takes).
    python tools/gt_small_d.py [--no-gt] [--split 8:4,16:8,32:8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-gt", action="store_true")
    ap.add_argument("--split", default="8:4,16:8,32:8")
    a = ap.parse_args()
    import numpy as np
    from online_convex_optimization_amd import engine
    T, runs = 1000, 65536
    for d in (() if a.no_gt else (5, 8, 16, 32)):
        ref = None
        for name, lanes in (("best", engine.LANES_BEST), ("exact", 1)):
            engine.gT_regrets(T, runs, base_seed=0, d=d, lanes_per_seq=lanes)  # warm: same shape
            t0 = time.perf_counter()
            reg = engine.gT_regrets(T, runs, base_seed=0, d=d, lanes_per_seq=lanes)
            dt = time.perf_counter() - t0
            if ref is None:
                ref = reg
            print(json.dumps({"what": "gT_regrets", "d": d, "T": T, "runs": runs, "mode": name,
                              "seconds": dt, "timesteps_per_s": runs * T / dt,
                              "max_rel_vs_best": float(np.max(np.abs(reg - ref) / np.maximum(1, np.abs(ref))))}),
                  flush=True)
    # generation and the FTRL pass apart, on the resident batch in the layout gT_regrets takes
    # (OCX_LANES_BEST: lanes of two coordinates, up to 8)
    import torch
    for d, lanes in ((int(x.split(":")[0]), int(x.split(":")[1])) for x in a.split.split(",")):
        X = engine.DeviceBatch(runs, T, d, lanes_per_seq=lanes)
        tg = tf = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            X.generate_gT(0, 0)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            X.simulate_alg(closed_comparator=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            tg, tf = min(tg, t1 - t0), min(tf, t2 - t1)
        print(json.dumps({"what": "split", "d": d, "T": T, "runs": runs, "lanes": lanes,
                          "P": int(X.L.P), "C": int(X.L.C), "gen_ms": tg * 1e3, "ftrl_ms": tf * 1e3,
                          "normals_per_s": runs * T * d / tg,
                          "ftrl_frac_8tbs": runs * T * (8 * d + 8) / tf / 8e12}), flush=True)
        del X
        engine.release_buffers()


if __name__ == "__main__":
    main()

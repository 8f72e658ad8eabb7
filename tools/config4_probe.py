"""configs[4] (d = 1024, T = 1e4): where a batch's time goes and how the batch size sets it.

Prints the free HBM, then engine.gT_regrets over `runs` runs with batches of whole generator
waves per SIMD (the default since round 6) and with equal batches (OCX_BATCH_WAVES=0), then per
resident batch size B the generator and the FTRL pass apart (DeviceBatch, OCX_LANES_BEST =
32 x 32).  One JSON line each.  (The engine sizes its batches by the free HBM: the g(T) calls
come first, before any DeviceBatch has grown torch's cache.)

    python tools/config4_probe.py [--runs 32768] [--sizes 2048,2731,2979,3072]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=32768)
    ap.add_argument("--sizes", default="2048,2731,2979,3072")
    ap.add_argument("--T", type=int, default=10000)
    ap.add_argument("--modes", default="32:0:1,32:0:0",
                    help="lanes:trailing:whole-wave-batches per g(T) call (64 / trailing 1: the "
                         "round-6 64 x 16 trailing experiment, whose code git history keeps)")
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    T, d = a.T, 1024
    free, total = torch.cuda.mem_get_info()
    print(json.dumps({"what": "hbm", "free_GiB": free / 2**30, "total_GiB": total / 2**30}), flush=True)
    engine.release_buffers()
    import numpy as np
    refs = {}
    # (layout lanes, trailing, whole-wave batches): 32 x 32 sequential (the default), the same
    # with equal batches, 64 x 16 sequential, 64 x 16 through the trailing pipeline
    for lanes, trail, bw in [m.split(":") for m in a.modes.split(",")]:
        os.environ["OCX_GT_1K_LANES"] = lanes
        os.environ["OCX_TRAILING"] = trail
        os.environ["OCX_BATCH_WAVES"] = bw
        engine.gT_regrets(T, a.runs, d=d)  # warm: the same shape (grows the library's HBM buffers)
        t0 = time.perf_counter()
        reg = engine.gT_regrets(T, a.runs, d=d)
        dt = time.perf_counter() - t0
        ref = refs.setdefault(lanes, reg)
        print(json.dumps({"what": "config4_gT", "T": T, "runs": a.runs, "d": d, "lanes": int(lanes),
                          "trailing": trail == "1", "batch_waves": bw == "1", "seconds": dt,
                          "free_GiB_after": torch.cuda.mem_get_info()[0] / 2**30,
                          "timesteps_per_s": T * a.runs / dt,
                          "same_regrets_as_first_of_layout": bool(np.array_equal(reg, ref)),
                          "g": engine.max_regret(reg)}), flush=True)
    engine.release_buffers()
    for k in ("OCX_BATCH_WAVES", "OCX_GT_1K_LANES", "OCX_TRAILING"):
        os.environ.pop(k, None)
    for B in (int(x) for x in a.sizes.split(",") if x):
        try:
            X = engine.DeviceBatch(B, T, d)
        except Exception as e:  # too large for this device
            print(json.dumps({"what": "batch", "B": B, "error": str(e)[:160]}), flush=True)
            torch.cuda.empty_cache()
            continue
        tg = tf = 1e9
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            X.generate_gT(0, 0)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            X.simulate_alg(closed_comparator=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            tg, tf = min(tg, t1 - t0), min(tf, t2 - t1)
        print(json.dumps({"what": "batch", "B": B, "T": T, "d": d, "P": int(X.L.P), "C": int(X.L.C),
                          "gen_ms": tg * 1e3, "ftrl_ms": tf * 1e3,
                          "ftrl_TBps": B * T * (8 * d + 8) / tf / 1e12,
                          "ns_per_stream_step": (tg + tf) / (B * T) * 1e9}), flush=True)
        del X
        import gc
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

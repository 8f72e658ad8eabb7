"""d = 1024 generator time against the streams it runs per SIMD (1 024 / 2 048 / 2 688 streams
= about 1 / 2 / 3 waves per SIMD), and the FTRL pass over the same batch in the 32 x 32 layout
(OCX_LANES_BEST) and the 64 x 16 one (lanes 64) — the measurements behind the d = 1024
trailing pipeline's pairing.  One JSON line per batch size.

    python tools/genscale_probe.py [--T 5000]
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
    ap.add_argument("--T", type=int, default=5000)
    ap.add_argument("--sizes", default="1024,2048,2688")
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    T, d = a.T, 1024

    def timed(fn, reps=2):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        return best

    for B in (int(x) for x in a.sizes.split(",")):
        X = engine.DeviceBatch(B, T, d)
        g = timed(lambda: X.generate_gT(0, 0))
        f = timed(lambda: X.simulate_alg())
        Y = engine.DeviceBatch(B, T, d, lanes_per_seq=64)
        g64 = timed(lambda: Y.generate_gT(0, 0))
        f64 = timed(lambda: Y.simulate_alg())
        rel = float((X.regret - Y.regret).abs().max() / X.regret.abs().max())
        print(json.dumps({"B": B, "T": T, "d": d, "gen_ms": g, "ftrl_ms_32x32": f,
                          "gen_ms_64x16": g64, "ftrl_ms_64x16": f64, "gen_streams_per_s": B / g * 1e3,
                          "maxrel_64x16_vs_32x32": rel}), flush=True)
        del X, Y
        engine.release_buffers()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

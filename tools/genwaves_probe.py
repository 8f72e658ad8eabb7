"""Generator time against the resident waves per SIMD, for the d = 1024 form and the d = 64
few-stream form (OCX_GEN_FORM=lr, single launch: OCX_GEN_ROUNDS=0), both in four-wave blocks, one
wave per stream: B = 1 024·w streams put w waves on every SIMD (256 CUs).  One JSON line per
(d, B): the launch time (best of `reps`), 64-normal rows per second, and the cycles per
64-draw round per wave at the nominal 2.4 GHz (rows ≈ rounds).  Run under rocprofv3 --pmc for
the counters of the same launches (tools/pmc_summary.py --by-grid).

    python tools/genwaves_probe.py [--cases 1024:1024:5000,...] [--reps 2]
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
    ap.add_argument("--cases", default="1024:1024:5000,1024:2048:5000,1024:3072:5000,"
                                        "64:1024:50000,64:2048:50000,64:3072:50000,64:4096:50000,"
                                        "64:6144:50000")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    os.environ["OCX_GEN_ROUNDS"] = "0"
    os.environ["OCX_GEN_FORM"] = "lr"
    import torch
    from online_convex_optimization_amd import engine
    for c in a.cases.split(","):
        d, B, T = (int(v) for v in c.split(":"))
        X = engine.DeviceBatch(B, T, d)
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            X.generate_gT(0, 0)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        rows = B * T * d / 64
        simds = 1024
        wps = B / simds
        cyc = best * 2.4e9 / (rows / B)  # cycles per row per wave
        print(json.dumps({"d": d, "B": B, "T": T, "waves_per_simd": wps, "ms": best * 1e3,
                          "rows_per_s": rows / best, "rows_per_s_per_simd": rows / best / simds,
                          "cycles_per_row_per_wave": cyc,
                          "cycles_per_row_per_simd": cyc / wps}), flush=True)
        del X
        engine.release_buffers()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

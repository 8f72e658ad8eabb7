"""configs[1]'s g(T) batch (65 536 runs x T = 1 000) at d = 16 / 32 through engine.gT_regrets:
the sequential generate-then-simulate loop (OCX_PIPELINE=0) against the sub-batch pipeline
(round 6 for these d) at several sub-batch sizes (OCX_PIPE_SUB_ROUNDS generator rounds per
sub-batch) and generator waves per SIMD (OCX_PIPE_WPS; `def`: the library's own choice).  One JSON line per setting, with a
bit-for-bit check against the sequential loop.

    python tools/small_pipe_probe.py [--d 16,32] [--runs 65536] [--T 1000]
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
    ap.add_argument("--d", default="16,32")
    ap.add_argument("--runs", type=int, default=65536)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--settings", default="seq,1:4,2:4,4:4,1:3,2:3,1:5")
    a = ap.parse_args()
    import numpy as np
    from online_convex_optimization_amd import engine
    for d in (int(x) for x in a.d.split(",")):
        ref = None
        for st in a.settings.split(","):
            for k in ("OCX_PIPELINE", "OCX_PIPE_SUB_ROUNDS", "OCX_PIPE_WPS"):
                os.environ.pop(k, None)
            if st == "seq":
                os.environ["OCX_PIPELINE"] = "0"
            elif st == "def":  # the library's own choice
                pass
            else:
                r, w = st.split(":")
                os.environ["OCX_PIPE_SUB_ROUNDS"] = r
                os.environ["OCX_PIPE_WPS"] = w
            engine.gT_regrets(a.T, a.runs, d=d)  # warm: same shape, streams, events
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                reg = engine.gT_regrets(a.T, a.runs, d=d)
                best = min(best, time.perf_counter() - t0)
            if ref is None:
                ref = reg
            print(json.dumps({"what": "small_pipe", "d": d, "T": a.T, "runs": a.runs, "setting": st,
                              "ms": best * 1e3, "timesteps_per_s": a.runs * a.T / best,
                              "frac_of_2x(8d+8)": a.runs * a.T / best * 2 * (8 * d + 8) / 8e12,
                              "bitidentical_to_seq": bool(np.array_equal(reg, ref))}), flush=True)
    for k in ("OCX_PIPELINE", "OCX_PIPE_SUB_ROUNDS", "OCX_PIPE_WPS"):
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()

"""General exact-FTL solver timing probe (round 3; rerun by tools/evidence.sh): ocx_dev_exact_ball_solve_tiled on the
exact driver's shapes (d = 5, every prefix of T = 100..1000, the linf ball, on the i.i.d.
family's clipped rows), and the exact g(T) comparator (final prefix only, 200 runs).  One
JSON line per shape: kernel ms, problems/s, mean Newton steps, max certified gap.

    python tools/exact_probe.py [--shapes B:T:d:norm:allp,...]   (allp 1 / 0; e.g. 4:200:256:linf:0)"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def time_solve(db, norm, all_prefixes, reps=3):
    g = db.exact_general(norm, all_prefixes)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(db.stream)
    for _ in range(reps):
        g = db.exact_general(norm, all_prefixes)
    ev[1].record(db.stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, g


SHAPES = ((48, 100, 5, "linf", True), (48, 1000, 5, "linf", True), (48, 1000, 5, "l1", True),
          (48, 1000, 5, "l2", True), (200, 1000, 5, "linf", False), (1024, 1000, 10, "linf", True))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    shapes = SHAPES
    if a.shapes:
        shapes = [(int(B), int(T), int(d), nm, ap_ == "1") for B, T, d, nm, ap_ in
                  (x.split(":") for x in a.shapes.split(","))]
    rng = np.random.default_rng(0)
    for B, T, d, norm, allp in shapes:
        z = rng.standard_normal((B, T, d))
        z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
        y = np.where(rng.random((B, T)) < 0.5, -1.0, 1.0)
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=1 if d <= 64 else engine.LANES_BEST).pack(z, y)
        t0 = time.perf_counter()
        ms, g = time_solve(db, norm, allp, a.reps)
        info = g["info"][:B].cpu().numpy()
        gap = g["gap"][:B].cpu().numpy()
        obj = g["obj"][:B].cpu().numpy()
        nprob = info.size
        wb, wn = np.unravel_index(int(np.argmax(gap)), gap.shape)
        worst = {"b": int(wb), "slot": int(wn), "gap": float(gap[wb, wn]), "obj": float(obj[wb, wn]),
                 "info": int(info[wb, wn]),
                 "x": g["actions"][wb, wn].cpu().numpy().tolist(),
                 "n_gap_over_1e-8": int((gap > 1e-8 * (1 + obj)).sum())}
        print(json.dumps({"B": B, "T": T, "d": d, "norm": norm, "all_prefixes": allp,
                          "problems": int(nprob), "kernel_ms": ms,
                          "problems_per_s": nprob / (ms * 1e-3),
                          "newton_mean": float(np.abs(info).mean()),
                          "capped": int((info < 0).sum()), "gap_max": float(gap.max()), "worst": worst,
                          "wall_s": time.perf_counter() - t0}), flush=True)
        del db, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Newton-step counts of the general exact solver per prefix (debugging aid for d > 64):
the data of tests/test_gpu_exact_general.py::test_big_lp_matches_highs, and the same rows cut
to fewer coordinates.  One JSON line per (d, norm)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def data(seed, B, T, d, clip=True, labels="pm1"):
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((B, T, d))
    if clip:
        z /= np.maximum(1.0, np.linalg.norm(z, axis=2, keepdims=True))
    y = (np.where(rng.random((B, T)) < 0.5, -1.0, 1.0) if labels == "pm1"
         else rng.standard_normal((B, T)))
    return z, y


def main():
    shapes = ((100, "l1", 100), (100, "l1", 64), (100, "l1", 48), (100, "linf", 100),
              (100, "linf", 64), (70, "l1", 70), (128, "l1", 128), (256, "l1", 256), (256, "linf", 256),
              (256, "l2", 256), (100, "l2", 100))
    if len(sys.argv) > 1:
        shapes = [(int(a), b, int(c)) for a, b, c in (x.split(":") for x in sys.argv[1].split(","))]
    for d, norm, cut in shapes:
        z, y = data(5 * d + (norm == "l1"), 2, 130, d)
        z = np.ascontiguousarray(z[..., :cut])
        res = engine.exact_ball_solve(z, y, norm=norm, all_prefixes=True)
        info = res["info"]
        steps = np.abs(info) & 0xFFFFF
        print(json.dumps({"d": cut, "norm": norm, "capped": int((info < 0).sum()),
                          "capped_prefixes": np.argwhere(info < 0)[:, 1].tolist()[:40],
                          "steps_mean": float(steps.mean()), "steps_max": int(steps.max()),
                          "gap_max": float(res["gap"].max()),
                          "uncertified": [[int(b), int(n), float(res["gap"][b, n]), float(res["obj"][b, n]),
                                           int(info[b, n])] for b, n in
                                          np.argwhere(res["gap"] > 1e-8 * (1 + np.abs(res["obj"])))[:12]]}),
              flush=True)


if __name__ == "__main__":
    main()

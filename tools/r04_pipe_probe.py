"""Round 4: the pipelined butterfly kernel with and without one of its step forms (the knob
OCX_PROBE_KNOB names: OCX_PIPE_CAND, the candidate-select step, by default; OCX_PIPE_SPEC,
the speculative sub-gradient step; csrc/ocx_alg_pipe.hip) on the few-wave batches and the
bench batch.  One JSON line per (batch, algorithm, form): kernel ms, fraction of 8 TB/s, and
whether the regrets of the two forms are bit-identical (they must be)."""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


KNOB = os.environ.get("OCX_PROBE_KNOB", "OCX_PIPE_CAND")


def timed(db, algo, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    db.simulate_alg(algo, math.sqrt(2))
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        db.simulate_alg(algo, math.sqrt(2))
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, db.regret[:db.L.B].cpu().numpy().copy()


def main():
    shapes = [(4900, 100000, 64), (3328, 100000, 64), (2048, 10000, 1024), (32768, 10000, 64)]
    if os.environ.get("OCX_PROBE_SHAPES"):
        shapes = [shapes[int(i)] for i in os.environ["OCX_PROBE_SHAPES"].split(",")]
    for B, T, d in shapes:
        db = engine.DeviceBatch(B, T, d).generate_gT(base_seed=0)
        for algo in (0, 1):
            res = {}
            for cand in ("0", "1"):
                os.environ[KNOB] = cand
                res[cand] = timed(db, algo, 3)
            same = bool(np.array_equal(res["0"][1], res["1"][1]))
            for cand, (ms, _) in res.items():
                gbs = B * T * (8 * d + 8) / (ms * 1e-3) / 1e9
                print(json.dumps({"B": B, "T": T, "d": d, "layout": [db.L.P, db.L.C],
                                  "algo": "FTL" if algo else "FTRL", "knob": KNOB, "on": cand == "1",
                                  "kernel_ms": ms, "frac": gbs / 8000.0,
                                  "bitidentical_forms": same}), flush=True)
        del db
        torch.cuda.empty_cache()
    os.environ.pop(KNOB, None)


if __name__ == "__main__":
    main()

"""Generation alone in rounds (ocx_run_gen_rounds) by round form (OCX_GEN_ROUNDS_FORM: ov4,
ov5, lr6) and against the single launch (OCX_GEN_ROUNDS=0), on the bench's resident batch
(32 768 x 1e4 x 64, OCX_LANES_BEST): min ms over repeats (HIP events) and whether the tiles
equal the single launch's bit for bit (wrapping int64 sums of z and y).
    python tools/gen_rounds_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def sums(db):
    zs, ys = db.z.view(torch.int64), db.y.view(torch.int64)
    return (int(zs.sum().item()), int(zs[::7].sum().item()), int(ys.sum().item()),
            int(ys[::5].sum().item()))


def main():
    B = int(os.environ.get("OCX_PROBE_B", 32768))
    T = int(os.environ.get("OCX_PROBE_T", 10000))
    db = engine.DeviceBatch(B, T, 64, lanes_per_seq=engine.LANES_BEST)
    forms = [("single", {"OCX_GEN_ROUNDS": "0"}), ("ov4", {"OCX_GEN_ROUNDS_FORM": "ov4"}),
             ("ov5", {"OCX_GEN_ROUNDS_FORM": "ov5"}), ("lr6", {"OCX_GEN_ROUNDS_FORM": "lr6"})]
    ref = None
    for name, env in forms:
        for k in ("OCX_GEN_ROUNDS", "OCX_GEN_ROUNDS_FORM"):
            os.environ.pop(k, None)
        os.environ.update(env)
        db.generate_gT(0, 0)  # warm
        torch.cuda.synchronize()
        got = sums(db)
        ref = ref or got
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(db.stream)
            db.generate_gT(0, 0)
            e1.record(db.stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"form": name, "B": B, "T": T, "ms_min": min(ts),
                          "bitidentical_to_single": got == ref}), flush=True)


if __name__ == "__main__":
    main()

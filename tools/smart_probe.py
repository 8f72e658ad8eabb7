"""SMART timing probe (round 3; rerun by tools/evidence.sh): the O(T²·d) re-scan kernels vs the O(T·d) closed-prefix
kernel on g(T)-sampler batches, next to the FTL kernel on the same batch.  One JSON line per
configuration."""
import json
import math
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from online_convex_optimization_amd import engine  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    for B, T, d in [(32768, 1000, 5), (768, 1000, 5), (32768, 10000, 5), (4096, 10000, 64)]:
        th = math.sqrt(2 * T)
        rec = {"B": B, "T": T, "d": d, "thresh": "sqrt(2T)"}
        ex = engine.DeviceBatch(B, T, d, lanes_per_seq=1).generate_gT(base_seed=0)
        sw = torch.zeros(B, dtype=torch.int64, device="cuda")
        st = torch.zeros(2, dtype=torch.int64, device="cuda")
        if T <= 1000:
            rec["rescan_ms"] = timed(lambda: ex.simulate_smart(th, closed_prefix=False,
                                                               closed_comparator=False), 1)
            r0 = ex.regret.clone()
        rec["prefix_exact_layout_ms"] = timed(lambda: ex.simulate_smart(
            th, switch_step=sw, closed_prefix=True, closed_comparator=False))
        r1 = ex.regret.clone()
        if T <= 1000:
            rec["prefix_bitexact_vs_rescan"] = bool(torch.equal(r0, r1))
        del ex
        torch.cuda.empty_cache()
        db = engine.DeviceBatch(B, T, d).generate_gT(base_seed=0)
        st.zero_()
        rec["best_ms"] = timed(lambda: db.simulate_smart(th, switch_step=sw, stats=st), 3)
        torch.cuda.synchronize()
        rec["best_stats_per_call"] = (st.cpu().numpy() / 4).tolist()
        rec["switched"] = int((sw >= 0).sum().item())
        rec["ftl_ms"] = timed(lambda: db.simulate_alg(1))
        rec["ftrl_ms"] = timed(lambda: db.simulate_alg(0))
        rec["layout"] = [db.L.P, db.L.C, db.L.chain]
        del db
        torch.cuda.empty_cache()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

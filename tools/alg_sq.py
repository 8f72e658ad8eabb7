"""One FTRL and one FTL launch of the pipelined kernel on a few-wave resident batch (default
4 900 x 1e5 x 64, OCX_LANES_BEST: the 8 x 8 butterfly), for SQ counter passes
(tools/evidence.sh algsq): rocprofv3 --pmc tells the two launches apart by the FTL template
argument.  python tools/alg_sq.py [B T d]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def main():
    B, T, d = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (4900, 100000, 64)))
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=engine.LANES_BEST).generate_gT(base_seed=0)
    for algo in (0, 1):
        db.simulate_alg(algo, math.sqrt(2), closed_comparator=True)
    torch.cuda.synchronize()
    print("layout", db.L.P, db.L.C, "ok", flush=True)


if __name__ == "__main__":
    main()

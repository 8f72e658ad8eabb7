"""Small-d generator check on the GPU: the DF = 16 / 32 form (default) against the generic loop
(OCX_GEN_SMALL=0) and NumPy's streams, per sequence; prints the first mismatch per case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from online_convex_optimization_amd import engine
    from oracle import oracle as O
    from tests._tiles import untile_y, untile_z
    for (B, T, d, P) in [(37, 257, 16, 8), (37, 40, 16, 8), (19, 33, 32, 8), (11, 65, 16, 8), (130, 301, 16, 8), (9, 77, 32, -4),
                         (50, 123, 32, 8), (37, 700, 16, 1)]:
        out = {}
        for mode in ("1", "0"):
            os.environ["OCX_GEN_SMALL"] = mode
            db = engine.DeviceBatch(B, T, d, lanes_per_seq=P).generate_gT(base_seed=3, run0=0)
            torch.cuda.synchronize()
            out[mode] = (untile_z(db.z.cpu().numpy(), db.L), untile_y(db.y.cpu().numpy(), db.L))
        bad = []
        for b in range(B):
            zr, yr = O.gT_sample(3, T, b, d)
            for mode in ("1", "0"):
                z, y = out[mode][0][b], out[mode][1][b]
                if not (np.array_equal(z, zr) and np.array_equal(y, yr)):
                    wz = np.argwhere(z != zr)
                    bad.append((mode, b, wz[:3].tolist(), int((z != zr).sum()), int((y != yr).sum())))
        print(B, T, d, P, "bad:", len(bad), bad[:6], flush=True)
    os.environ.pop("OCX_GEN_SMALL", None)


if __name__ == "__main__":
    main()

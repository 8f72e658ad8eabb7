"""One few-wave resident batch for counter runs: d=64, T=1e5, 4 900 sequences (the g(T)
sweep's T=1e5 batch), default layout (8 x 8 butterfly), closed-form comparator; the FTRL
kernel is launched twice after one generation."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from online_convex_optimization_amd import engine
    db = engine.DeviceBatch(4900, 100000, 64, lanes_per_seq=128)
    db.generate_gT(0, 0)
    for _ in range(2):
        db.simulate_alg(closed_comparator=True)
    torch.cuda.synchronize()
    print("ok", int(db.L.P), int(db.L.C), int(db.L.G))


if __name__ == "__main__":
    main()

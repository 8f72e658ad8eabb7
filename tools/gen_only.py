"""Launch only the g(T) generator on one resident batch (for rocprofv3 counter passes):
    python tools/gen_only.py B T d [launches] [lanes_per_seq]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from online_convex_optimization_amd import engine
    B, T, d = (int(v) for v in sys.argv[1:4])
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    kw = {"lanes_per_seq": int(sys.argv[5])} if len(sys.argv) > 5 else {}
    db = engine.DeviceBatch(B, T, d, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        db.generate_gT(0, 0)
    torch.cuda.synchronize()
    print(f"gen {B}x{T}x{d}: {(time.perf_counter() - t0) / n * 1e3:.2f} ms per launch", flush=True)


if __name__ == "__main__":
    main()

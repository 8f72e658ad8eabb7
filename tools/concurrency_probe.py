"""Probe: do two independent kernels on two HIP streams run concurrently?  Generator on
buffer 0 (stream A) and FTRL on buffer 1 (stream B), no events between them; compared
with each alone.  Streams from torch's pool and from hipStreamCreate directly."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from online_convex_optimization_amd import engine
    B, T, d = 16384, 10000, 64
    b0 = engine.DeviceBatch(B, T, d)
    b1 = engine.DeviceBatch(B, T, d)
    b0.generate_gT(0, 0)
    b1.generate_gT(0, B)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")

    def raw_stream():
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0  # non-blocking
        return torch.cuda.ExternalStream(h.value)

    pairs = {"torch_pool": (torch.cuda.Stream(), torch.cuda.Stream()),
             "hip_nonblocking": (raw_stream(), raw_stream())}
    for name, (sa, sb) in pairs.items():
        def gen():
            b0.stream = sa
            b0.generate_gT(0, 0)

        def sim():
            b1.stream = sb
            b1.simulate_alg()

        res = {"streams": name, "sa": hex(sa.cuda_stream), "sb": hex(sb.cuda_stream)}
        for label, fns in (("gen", [gen]), ("sim", [sim]), ("both", [gen, sim]), ("both_rev", [sim, gen])):
            for f in fns:
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                for f in fns:
                    f()
            torch.cuda.synchronize()
            res[label + "_ms"] = 1e3 * (time.perf_counter() - t0) / 3
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

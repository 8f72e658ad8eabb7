"""Probe: can the d = 1024 g(T) batch (configs[4]) overlap generation and FTRL by splitting
the CUs between them (hipExtStreamCreateWithCUMask) instead of sharing SIMDs?  The lean-FTRL
co-residency of the d = 64 pipelines does not fit at d = 1024.

For each split (FTRL on n CUs, chosen contiguous or strided over the CU index, the generator
on the rest): the generator alone, FTRL alone, and both at once on two unrelated batches
(X generated while Y, generated beforehand, is simulated).  One JSON line per measurement.

    python tools/cumask_probe.py [--B 0] [--T 5000] [--splits 32c,40c,48c,64c]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hip_lib():
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def cu_stream(torch, hip, bits, ncu):
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for i in bits:
        words[i // 32] |= (1 << (i % 32))
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=0, help="streams per batch (0: three per SIMD of the generator's CUs)")
    ap.add_argument("--T", type=int, default=5000)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--splits", default="32c,40c,48c,64c")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    hip = hip_lib()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    dflt = torch.cuda.current_stream()

    def timed(fn):
        best = None
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            best = dt if best is None else min(best, dt)
        return best

    for sp in a.splits.split(","):
        n, kind = int(sp[:-1]), sp[-1]
        if kind == "c":  # contiguous mask bits: spread evenly over the XCDs (r05_cumask_map.txt)
            fb = list(range(n))
        else:  # strided: every (ncu // n)-th CU
            step = ncu // n
            fb = [i * step for i in range(n)]
        gb = [i for i in range(ncu) if i not in set(fb)]
        B = a.B or 12 * len(gb)
        X = engine.DeviceBatch(B, a.T, a.d)
        Y = engine.DeviceBatch(B, a.T, a.d)
        X.stream = dflt
        Y.stream = dflt
        Y.generate_gT(0, 0)
        torch.cuda.synchronize()
        ref = Y.simulate_alg().clone()
        g_all = timed(lambda: X.generate_gT(0, B))
        f_all = timed(lambda: Y.simulate_alg())
        sf = cu_stream(torch, hip, fb, ncu)
        sg = cu_stream(torch, hip, gb, ncu)
        os.environ["OCX_GEN_CUS"] = str(len(gb))
        X.stream = sg
        Y.stream = sf
        g_ms = timed(lambda: X.generate_gT(0, B))
        f_ms = timed(lambda: Y.simulate_alg())

        def both():
            X.generate_gT(0, B)
            Y.simulate_alg()

        def both_rev():
            Y.simulate_alg()
            X.generate_gT(0, B)
        b_ms = timed(both)
        br_ms = timed(both_rev)
        same = bool(torch.equal(Y.regret, ref))
        seq = g_all + f_all
        print(json.dumps({"B": B, "T": a.T, "d": a.d, "P": X.L.P, "C": X.L.C, "cus": ncu,
                          "split": sp, "ftrl_cus": n, "gen_cus": len(gb), "gen_all_ms": g_all,
                          "ftrl_all_ms": f_all, "sequential_ms": seq, "gen_ms": g_ms,
                          "ftrl_ms": f_ms, "both_ms": b_ms, "both_rev_ms": br_ms,
                          "regrets_equal": same,
                          "both_vs_sequential": min(b_ms, br_ms) / seq}), flush=True)
        os.environ.pop("OCX_GEN_CUS", None)
        X.stream = dflt
        Y.stream = dflt
        del X, Y
        engine.release_buffers()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

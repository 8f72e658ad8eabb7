"""Diagnostics on one MI355X: HBM read ceilings and the FTRL kernel across lane splits.

    python tools/tune.py [--B 32768 --T 10000 --d 64] [--lanes 1,2,4,8,16]

Prints one JSON line per measurement.  Not part of the product path."""
import argparse
import ctypes
import json
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_probe():
    out = os.path.join(ROOT, "build", "libhbm_probe.so")
    src = os.path.join(ROOT, "tools", "hbm_probe.hip")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", src, "-o", out],
                       check=True)
    return out


def timeit(fn, stream, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32768)
    ap.add_argument("--T", type=int, default=10000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--lanes", default="1,2,4,8,16")
    ap.add_argument("--probe", type=int, default=1)
    ap.add_argument("--variants", default="", help="tune_build/libocx_<name>.so to A/B")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import _lib, engine
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    B, T, d = a.B, a.T, a.d
    alg = B * T * 2 * (8 * d + 8)
    db = None
    for P in [int(x) for x in a.lanes.split(",")]:
        db = None
        torch.cuda.empty_cache()
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=P)
        db.generate_gT(0, 0)
        torch.cuda.synchronize()
        libs = [("base", None)]
        for v in [x for x in a.variants.split(",") if x]:
            L = ctypes.CDLL(os.path.join(ROOT, "tune_build", f"libocx_{v}.so"))
            L.ocx_dev_simulate_alg.argtypes = _lib.SIGNATURES["ocx_dev_simulate_alg"][1]
            libs.append((v, L))

        def run(L):
            if L is None:
                return lambda: db.simulate_alg(0, math.sqrt(2))
            return lambda: L.ocx_dev_simulate_alg(ctypes.byref(db.L), db.z.data_ptr(),
                                                  db.y.data_ptr(), 0, math.sqrt(2), None,
                                                  db.regret.data_ptr(), None, None, None,
                                                  ctypes.c_void_p(st.cuda_stream))
        res = {n: [] for n, _ in libs}
        for _ in range(a.rounds):
            for n, L in libs:
                res[n].append(timeit(run(L), st, reps=3))
        for n, _ in libs:
            ms = min(res[n])
            print(json.dumps({"what": "alg", "lib": n, "lanes": P, "P": db.L.P, "C": db.L.C,
                              "chain": db.L.chain, "ms_min": ms,
                              "ms_med": sorted(res[n])[len(res[n]) // 2],
                              "GBs": alg / ms / 1e6, "frac": alg / ms / 1e6 / 8000}), flush=True)
    if a.probe and db is not None:
        lib = ctypes.CDLL(build_probe())
        out = torch.zeros(1 << 20, dtype=torch.float64, device="cuda")
        nbytes = db.z_bytes
        for kind, nw in ((0, 2048), (0, 4096), (0, 8192), (0, 16384), (1, 0), (2, 2048),
                         (2, 4096), (2, 8192), (3, 2048), (3, 4096), (4, 4096), (4, 8192)):
            ms = timeit(lambda: lib.probe_run(kind, ctypes.c_void_p(db.z.data_ptr()),
                                              ctypes.c_int64(nbytes), ctypes.c_int64(nw),
                                              ctypes.c_void_p(out.data_ptr()),
                                              ctypes.c_void_p(st.cuda_stream)), st)
            print(json.dumps({"what": "probe", "kind": ["region8", "stride", "region16", "region32",
                                                        "region16plain"][kind], "waves": nw,
                              "bytes": nbytes, "ms": ms, "GBs": nbytes / ms / 1e6}), flush=True)


if __name__ == "__main__":
    main()

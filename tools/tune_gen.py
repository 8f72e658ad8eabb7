"""A/B timing of the g(T) generator (ocx_dev_gen_gT) across tuning builds.

    python tools/tune_gen.py --variants nostore,nonorm,noparse [--B 32768 --T 10000 --d 64]

Each variant is tune_build/libocx_<name>.so (online_convex_optimization_amd._build.
build_variant).  Prints one JSON line per library.  Diagnostic only."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32768)
    ap.add_argument("--T", type=int, default=10000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dir", default="tune_build", help="where the variant libraries are")
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import _lib, engine
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    db = engine.DeviceBatch(a.B, a.T, a.d, lanes_per_seq=a.lanes)
    libs = [("base", _lib.load())]
    for v in [x for x in a.variants.split(",") if x]:
        L = ctypes.CDLL(os.path.join(ROOT, a.dir, f"libocx_{v}.so"))
        L.ocx_dev_gen_gT.argtypes = _lib.SIGNATURES["ocx_dev_gen_gT"][1]
        libs.append((v, L))
    res = {n: [] for n, _ in libs}
    for _ in range(a.rounds):
        for n, L in libs:
            def run():
                rc = L.ocx_dev_gen_gT(ctypes.byref(db.L), 0, 0, db.z.data_ptr(), db.y.data_ptr(),
                                      ctypes.c_void_p(st.cuda_stream))
                assert rc == 0
            run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            for _ in range(3):
                run()
            e.record(st)
            torch.cuda.synchronize()
            res[n].append(s.elapsed_time(e) / 3)
    for n, _ in libs:
        ms = min(res[n])
        print(json.dumps({"what": "gen", "lib": n, "B": a.B, "T": a.T, "d": a.d, "P": db.L.P,
                          "ms_min": ms, "timesteps_per_s": a.B * a.T / ms * 1e3,
                          "normals_per_s": a.B * a.T * a.d / ms * 1e3}), flush=True)


if __name__ == "__main__":
    main()

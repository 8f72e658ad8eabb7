"""Generator A/B between the tuning libraries (OCX_TUNE_DIR, default tune_r04) named on the command line, the first
the reference: checks their outputs agree (wrapping int64 sums of z and y, full and strided)
on three shapes, then times ocx_dev_gen_gT for each (min over rounds, HIP events).
    python tools/gen_lib_ab.py rej0,rej1"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from online_convex_optimization_amd import _lib, engine  # noqa: E402


def lib(name):
    # "main": the product library itself (the reference of the comparison)
    path = (os.path.join(ROOT, "online_convex_optimization_amd", "libocx.so") if name == "main" else
            os.path.join(ROOT, os.environ.get("OCX_TUNE_DIR", "tune_r04"), f"libocx_{name}.so"))
    L = ctypes.CDLL(path)
    L.ocx_dev_gen_gT.argtypes = _lib.SIGNATURES["ocx_dev_gen_gT"][1]
    return L


def main():
    st = torch.cuda.current_stream()
    libs = [(n, lib(n)) for n in sys.argv[1].split(",")]
    shapes = ((3000, 1000, 64), (32768, 10000, 64), (4900, 100000, 64), (2048, 10000, 1024))
    if os.environ.get("GENAB_SHAPES"):  # "B:T:d,..."
        shapes = tuple(tuple(int(v) for v in c.split(":")) for c in os.environ["GENAB_SHAPES"].split(","))
    for B, T, d in shapes:
        db = engine.DeviceBatch(B, T, d, lanes_per_seq=engine.LANES_BEST)
        sums = []
        for n, L in libs:  # one buffer (the big shapes fill HBM): compare wrapping sums
            assert L.ocx_dev_gen_gT(ctypes.byref(db.L), 0, 0, db.z.data_ptr(), db.y.data_ptr(),
                                    ctypes.c_void_p(st.cuda_stream)) == 0
            zs = db.z.view(torch.int64)
            ys = db.y.view(torch.int64)
            sums.append((int(zs.sum().item()), int(zs[::7].sum().item()),
                         int(ys.sum().item()), int(ys[::7].sum().item()),
                         int(ys[::13].sum().item())))
        del zs, ys  # views of db.z: it would keep the batch alive into the next shape
        same = all(x == sums[0] for x in sums)
        print(json.dumps({"B": B, "T": T, "d": d, "bit_identical": bool(same)}), flush=True)
        if not same:
            sys.exit(3)
        res = {n: [] for n, _ in libs}
        for _ in range(3):
            for n, L in libs:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(st)
                for _ in range(3):
                    L.ocx_dev_gen_gT(ctypes.byref(db.L), 0, 0, db.z.data_ptr(), db.y.data_ptr(),
                                     ctypes.c_void_p(st.cuda_stream))
                e.record(st)
                torch.cuda.synchronize()
                res[n].append(s.elapsed_time(e) / 3)
        for n in res:
            print(json.dumps({"what": "gen", "lib": n, "B": B, "T": T, "d": d, "ms_min": min(res[n])}),
                  flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

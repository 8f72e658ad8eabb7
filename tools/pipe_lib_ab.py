"""FTRL / FTL kernel A/B between tuning builds of ocx_alg_pipe.hip (OCX_TUNE_DIR, default
tune_r04; _build.build_variant), the first the reference: whether the regrets of every build
are bit-identical to the first's (and the largest relative difference, for the fast-action
builds), then each build's kernel time (min over rounds, HIP events) on the few-wave batches
and the bench batch.  The batches are g(T) rows (OCX_ALG_CLIPPED_ROWS), as in the sweeps.
    python tools/pipe_lib_ab.py p0,pys,pftl"""
import ctypes
import json
import math
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
    L.ocx_dev_simulate_alg_ex.argtypes = _lib.SIGNATURES["ocx_dev_simulate_alg_ex"][1]
    return L


def main():
    st = torch.cuda.current_stream()
    libs = [(n, lib(n)) for n in sys.argv[1].split(",")]
    shapes = [(4900, 100000, 64), (3328, 100000, 64), (32768, 10000, 64), (2048, 10000, 1024)]
    for B, T, d in shapes:
        db = engine.DeviceBatch(B, T, d).generate_gT(base_seed=0)
        for algo in (0, 1):
            regs, res = [], {n: [] for n, _ in libs}

            def launch(L):
                rc = L.ocx_dev_simulate_alg_ex(ctypes.byref(db.L), db.z.data_ptr(), db.y.data_ptr(),
                                               algo, math.sqrt(2), None, db.regret.data_ptr(), None,
                                               None, None, _lib.OCX_ALG_CLIPPED_ROWS, None,
                                               ctypes.c_void_p(st.cuda_stream))
                assert rc == 0
            for n, L in libs:
                launch(L)
                torch.cuda.synchronize()
                regs.append(db.regret[:B].clone())
            same = all(torch.equal(r, regs[0]) for r in regs)
            rel = {n: float(((r - regs[0]).abs() / regs[0].abs().clamp(min=1.0)).max())
                   for (n, _), r in zip(libs, regs)}
            for _ in range(3):
                for n, L in libs:
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record(st)
                    launch(L)
                    e.record(st)
                    torch.cuda.synchronize()
                    res[n].append(s.elapsed_time(e))
            for n in res:
                ms = min(res[n])
                print(json.dumps({"lib": n, "B": B, "T": T, "d": d, "layout": [db.L.P, db.L.C],
                                  "algo": "FTL" if algo else "FTRL", "kernel_ms": ms,
                                  "frac": B * T * (8 * d + 8) / (ms * 1e-3) / 8e12,
                                  "bitidentical": same, "max_rel_vs_first": rel[n]}), flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

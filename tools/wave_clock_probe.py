"""Where the few-wave FTRL / FTL launches spend their time, wave by wave: the diagnostic
build of ocx_alg_pipe.hip (OCX_PIPE_WAVE_CLOCK=1, tuning library libocx_wclk.so under
OCX_TUNE_DIR, default tune_r04; made here on the CPU by `python tools/wave_clock_probe.py
--build`) writes each wave's duration and start (100 MHz real-time clock) and its HW_ID /
XCC_ID instead of the loss sums.  One JSON line per algorithm: the launch's time (events),
the waves' duration spread, and the mean duration by how many of the launch's waves shared
the wave's SIMD and CU, and by XCD.
    python tools/wave_clock_probe.py [B T d]"""
import ctypes
import json
import math
import os
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TUNE = os.path.join(ROOT, os.environ.get("OCX_TUNE_DIR", "tune_r04"))


def build():
    from online_convex_optimization_amd import _build
    print(_build.build_variant("wclk", ["OCX_PIPE_WAVE_CLOCK=1"], source="ocx_alg_pipe.hip",
                               out_dir=TUNE))


def main():
    import numpy as np
    import torch
    from online_convex_optimization_amd import _lib, engine
    B, T, d = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (4900, 100000, 64)))
    L = ctypes.CDLL(os.path.join(TUNE, "libocx_wclk.so"))
    L.ocx_dev_simulate_alg_ex.argtypes = _lib.SIGNATURES["ocx_dev_simulate_alg_ex"][1]
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=engine.LANES_BEST).generate_gT(base_seed=0)
    S = 64 // db.L.P
    st = torch.cuda.current_stream()
    dur = torch.zeros(db.L.G * S, dtype=torch.float64, device=db.device)
    t0 = torch.zeros_like(dur)
    hw = torch.zeros(db.L.G * S, dtype=torch.int32, device=db.device)
    for algo in (0, 1):
        def launch():
            rc = L.ocx_dev_simulate_alg_ex(ctypes.byref(db.L), db.z.data_ptr(), db.y.data_ptr(),
                                           algo, math.sqrt(2), None, db.regret.data_ptr(),
                                           dur.data_ptr(), t0.data_ptr(), None,
                                           _lib.OCX_ALG_CLIPPED_ROWS, hw.data_ptr(),
                                           ctypes.c_void_p(st.cuda_stream))
            assert rc == 0
        launch()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(st)
        launch()
        ev[1].record(st)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1])
        w_dur = dur[:B:S].cpu().numpy() * 1e-5  # 100 MHz ticks -> ms
        w_t0 = t0[:B:S].cpu().numpy()
        w_hw = hw[:B:S].cpu().numpy().astype(np.int64)
        xcc = (w_hw >> 16) & 0xF
        cu_key = [(int(x), int((h >> 13) & 7), int((h >> 12) & 1), int((h >> 8) & 15))
                  for x, h in zip(xcc, w_hw)]
        simd_key = [k + (int((h >> 4) & 3),) for k, h in zip(cu_key, w_hw)]
        per_cu, per_simd = Counter(cu_key), Counter(simd_key)
        by = {"simd": defaultdict(list), "cu": defaultdict(list), "xcd": defaultdict(list)}
        for i in range(len(w_dur)):
            by["simd"][per_simd[simd_key[i]]].append(w_dur[i])
            by["cu"][per_cu[cu_key[i]]].append(w_dur[i])
            by["xcd"][int(xcc[i])].append(w_dur[i])
        out = {"B": B, "T": T, "d": d, "layout": [db.L.P, db.L.C], "algo": "FTL" if algo else "FTRL",
               "kernel_ms": ms, "waves": int(len(w_dur)), "cus_used": len(per_cu),
               "wave_ms": {q: float(np.percentile(w_dur, p)) for q, p in
                           (("min", 0), ("p10", 10), ("median", 50), ("p90", 90), ("max", 100))},
               "start_spread_ms": float((w_t0.max() - w_t0.min()) * 1e-5)}
        for k, grp in by.items():
            out[f"mean_wave_ms_by_waves_per_{k}" if k != "xcd" else "mean_wave_ms_by_xcd"] = {
                str(n): [round(float(np.mean(v)), 3), len(v)] for n, v in sorted(grp.items())}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    build() if "--build" in sys.argv else main()

"""Generation overlapped with FTRL in sub-batches (ocx_dev_gen_simulate, csrc/ocx_pipeline.hip)
against the sequential gen-then-FTRL loop, on the bench's resident batch (32 768 x 1e4 x 64,
OCX_LANES_BEST).  One JSON line per configuration: ms per batch, timesteps/s, fraction of
2*(8d+8) B/step, and whether the regrets and g(T) are bit-identical to the sequential path.
Knobs per configuration (OCX_PROBE_CONFIGS="wps:sub:gs:ss,..."): OCX_PIPE_WPS (generator waves
per SIMD), sub_seqs (sequences per sub-batch; 0 = one generator round), OCX_PIPE_GEN_STREAMS /
OCX_PIPE_SIM_STREAMS (sub-batches alternating over one or two streams per side).
OCX_PROBE_SIDES=1 also times each side alone through OCX_PIPE_SKIP, which only a tuning build
compiled with -DOCX_PIPE_TUNE_SKIP honours (OCX_LIB)."""
import json
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from online_convex_optimization_amd import engine  # noqa: E402


def run(db, nb, pipelined, sub=0):
    g = torch.zeros(1, dtype=torch.float64, device=db.device)
    db.generate_simulate(0, 0, 1, gmax=g, pipelined=pipelined, sub_seqs=sub)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    db.generate_simulate(0, 0, nb, gmax=g, pipelined=pipelined, sub_seqs=sub)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return dt / nb * 1e3, db.regret[:db.L.B].cpu().numpy().copy(), float(g.item())


def _configs():
    # (generator waves per SIMD, sub-batch sequences, generator streams, FTRL streams)
    configs = [("4", 0, "2", "2"), ("4", 0, "1", "1"), ("3", 0, "2", "2"), ("4", 2 * 1024, "2", "2")]
    if os.environ.get("OCX_PROBE_CONFIGS"):
        configs = []
        for c in os.environ["OCX_PROBE_CONFIGS"].split(","):
            f = c.split(":") + ["2", "2"]
            configs.append((f[0], int(f[1]), f[2], f[3]))
    return configs


def _env(wps, gs, ss):
    os.environ["OCX_PIPE_WPS"] = wps
    os.environ["OCX_PIPE_GEN_STREAMS"] = gs
    os.environ["OCX_PIPE_SIM_STREAMS"] = ss


def main():
    B = int(os.environ.get("OCX_PROBE_B", 32768))
    T = int(os.environ.get("OCX_PROBE_T", 10000))
    d = 64
    nb = int(os.environ.get("OCX_PROBE_NB", 4))
    lanes = int(os.environ.get("OCX_PROBE_LANES", engine.LANES_BEST))
    db = engine.DeviceBatch(B, T, d, lanes_per_seq=lanes)
    # OCX_PROBE_SEQ=0 (the PMC traffic step): the pipelined runs alone
    seq = os.environ.get("OCX_PROBE_SEQ", "1") != "0"
    configs = _configs()
    if not seq:
        for wps, sub, gs, ss in configs:
            _env(wps, gs, ss)
            ms, r, g = run(db, nb, True, sub)
            print(json.dumps({"B": B, "T": T, "mode": "pipelined", "ms_per_batch": ms}), flush=True)
        return
    ms0, r0, g0 = run(db, nb, False)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    db.generate_gT(0, 0)
    ev[1].record()
    db.simulate_alg(0, math.sqrt(2))
    ev[2].record()
    torch.cuda.synchronize()
    parts = {"gen_default_ms": ev[0].elapsed_time(ev[1]), "sim_default_ms": ev[1].elapsed_time(ev[2])}
    rate = lambda ms: B * T / (ms * 1e-3)
    print(json.dumps({"B": B, "T": T, "layout": [db.L.P, db.L.C], "mode": "sequential",
                      "ms_per_batch": ms0, "timesteps_per_s": rate(ms0),
                      "frac_1040": rate(ms0) * 1040 / 8e12, "gmax": g0, **parts}), flush=True)
    for wps, sub, gs, ss in configs:
        _env(wps, gs, ss)
        # each side alone (OCX_PIPE_SKIP, tuning builds only: outputs wrong, times only)
        side = {}
        for skip in (("sim", "gen") if os.environ.get("OCX_PROBE_SIDES", "0") == "1" else ()):
            os.environ["OCX_PIPE_SKIP"] = skip
            side["gen_only_ms" if skip == "sim" else "sim_only_ms"] = run(db, nb, True, sub)[0]
        os.environ.pop("OCX_PIPE_SKIP", None)
        ms, r, g = run(db, nb, True, sub)
        print(json.dumps({"B": B, "T": T, "layout": [db.L.P, db.L.C], "mode": "pipelined",
                          "wps": int(wps), "sub_seqs": sub,
                          "gen_streams": int(gs), "sim_streams": int(ss),
                          "ms_per_batch": ms, "timesteps_per_s": rate(ms),
                          "frac_1040": rate(ms) * 1040 / 8e12, "gmax": g, **side,
                          "bitidentical": bool(np.array_equal(r, r0)) and g == g0}), flush=True)


if __name__ == "__main__":
    main()

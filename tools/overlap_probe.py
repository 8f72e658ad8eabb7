"""Probe: does generation of batch k+1 overlap with simulation of batch k on two HIP
streams?  Serial = gen, sim, gen, sim on one stream; pipelined = gen on stream 1,
sim on stream 2, double-buffered with events.  One JSON line per (B, T, d)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(B, T, d, nbatch, lanes):
    import torch
    from online_convex_optimization_amd import engine
    s_gen = torch.cuda.Stream()
    s_sim = torch.cuda.Stream()
    bufs = [engine.DeviceBatch(B, T, d, lanes_per_seq=lanes) for _ in range(2)]

    def serial():
        for k in range(nbatch):
            db = bufs[k % 2]
            db.stream = torch.cuda.current_stream()
            db.generate_gT(0, k * B)
            db.simulate_alg()
        torch.cuda.synchronize()

    def pipelined():
        gen_done = [torch.cuda.Event() for _ in range(2)]
        sim_done = [torch.cuda.Event() for _ in range(2)]
        for k in range(nbatch):
            i = k % 2
            db = bufs[i]
            if k >= 2:
                s_gen.wait_event(sim_done[i])
            db.stream = s_gen
            db.generate_gT(0, k * B)
            gen_done[i].record(s_gen)
            s_sim.wait_event(gen_done[i])
            db.stream = s_sim
            db.simulate_alg()
            sim_done[i].record(s_sim)
        torch.cuda.synchronize()

    out = {"B": B, "T": T, "d": d, "nbatch": nbatch, "lanes": lanes}
    for name, fn in (("serial", serial), ("pipelined", pipelined), ("serial2", serial),
                     ("pipelined2", pipelined)):
        fn()  # warm
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        out[name + "_s"] = dt
        out[name + "_timesteps_per_s"] = nbatch * B * T / dt
    # separate component times
    db = bufs[0]
    db.stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    db.generate_gT(0, 0)
    torch.cuda.synchronize()
    out["gen_only_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    db.simulate_alg()
    torch.cuda.synchronize()
    out["sim_only_s"] = time.perf_counter() - t0
    print(json.dumps(out), flush=True)
    del bufs
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="16384x10000x64,131072x1000x64,1024x10000x1024")
    ap.add_argument("--nbatch", type=int, default=6)
    ap.add_argument("--lanes", type=int, default=1)
    a = ap.parse_args()
    for c in a.cases.split(","):
        B, T, d = (int(v) for v in c.split("x"))
        run(B, T, d, a.nbatch, a.lanes)


if __name__ == "__main__":
    main()

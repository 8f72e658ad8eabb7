"""Probe: generation of batch k+1 beside simulation of batch k, double-buffered, on
(a) one stream (serial), (b) two plain streams, (c) two streams restricted to disjoint
CU masks (hipExtStreamCreateWithCUMask), FTRL on `f` CUs and the generator on the rest.
One JSON line per variant.  Run the FTRL priority build with OCX_LIB set."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cu_stream(torch, bits):
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)()
    for i in bits:
        words[i // 32] |= (1 << (i % 32))
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(8), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16384)
    ap.add_argument("--T", type=int, default=10000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--nbatch", type=int, default=6)
    ap.add_argument("--lanes", type=int, default=128)
    ap.add_argument("--splits", default="32:8,64:4,96:8,128:2")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    from online_convex_optimization_amd import engine
    B, T, d = a.B, a.T, a.d
    bufs = [engine.DeviceBatch(B, T, d, lanes_per_seq=a.lanes) for _ in range(2)]

    def serial():
        for k in range(a.nbatch):
            db = bufs[k % 2]
            db.stream = torch.cuda.current_stream()
            db.generate_gT(0, k * B)
            db.simulate_alg()
        torch.cuda.synchronize()

    def pipelined(s_gen, s_sim):
        gen_done = [torch.cuda.Event() for _ in range(2)]
        sim_done = [torch.cuda.Event() for _ in range(2)]
        for k in range(a.nbatch):
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

    def timed(fn, *args):
        fn(*args)
        best = 1e9
        for _ in range(2):
            t0 = time.perf_counter()
            fn(*args)
            best = min(best, time.perf_counter() - t0)
        return best

    ref = None
    variants = [("serial", serial, ())]
    variants.append(("pipe", pipelined, (torch.cuda.Stream(), torch.cuda.Stream())))
    for sp in [x for x in a.splits.split(",") if x]:
        f, mod = (int(v) for v in sp.split(":"))
        # FTRL on CUs i with i % mod < f*mod/256, generator on the rest
        take = f * mod // 256
        fb = [i for i in range(256) if i % mod < take]
        gb = [i for i in range(256) if i % mod >= take]
        variants.append((f"mask{len(fb)}m{mod}", pipelined, (cu_stream(torch, gb), cu_stream(torch, fb)),
                         len(gb)))
    for v in variants:
        name, fn, args = v[0], v[1], v[2]
        if len(v) > 3:
            os.environ["OCX_GEN_CUS"] = str(v[3])
        else:
            os.environ.pop("OCX_GEN_CUS", None)
        dt = timed(fn, *args)
        solo = {}
        if len(v) > 3:  # each half alone on its CU-masked stream
            s_gen, s_sim = args
            db = bufs[0]
            for nm, st, call in (("gen_ms", s_gen, lambda: db.generate_gT(0, 0)),
                                 ("sim_ms", s_sim, db.simulate_alg)):
                db.stream = st
                call()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(2):
                    call()
                torch.cuda.synchronize()
                solo[nm] = 1e3 * (time.perf_counter() - t0) / 2
            serial()  # restore the buffers' contents
        regs = torch.cat([b.regret for b in bufs]).cpu()
        if ref is None:
            ref = regs
        same = bool(torch.equal(regs, ref))
        print(json.dumps({"tag": a.tag, "variant": name, "B": B, "T": T, "d": d, "nbatch": a.nbatch,
                          "lanes": a.lanes, "s": dt, "ms_per_batch": 1e3 * dt / a.nbatch,
                          "timesteps_per_s": a.nbatch * B * T / dt, "same_regrets": same, **solo}),
              flush=True)
    os.environ.pop("OCX_GEN_CUS", None)
    # components alone
    db = bufs[0]
    db.stream = torch.cuda.current_stream()
    for name, fn in (("gen_only", lambda: db.generate_gT(0, 0)), ("sim_only", db.simulate_alg)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(json.dumps({"tag": a.tag, "variant": name, "B": B, "ms": 1e3 * (time.perf_counter() - t0) / 3}),
              flush=True)


if __name__ == "__main__":
    main()

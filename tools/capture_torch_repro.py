"""Does torch.cuda.graph crash capturing a multi-stream fork/join WITHOUT libocx?

The second half of tools/capture_repro.hip's question (see there): the same schedule as
ocx_pipeline.hip — the capturing stream forks to three side streams through one event,
sub-batches ordered by per-sub-batch events, one join event per side stream — written with
torch streams, events and elementwise kernels only, captured with torch.cuda.graph after an
eager warm-up, replayed twice against the eager result.

    timeout -k 10 120 python tools/capture_torch_repro.py
"""
import sys

import torch


def enqueue(st, side, ev_fork, ev_gen, ev_sim, ev_join, buf, out, nb, ns):
    gen2, sim, sim2 = side
    ev_fork.record(st)
    for s in side:
        s.wait_event(ev_fork)
    rec = [False] * ns
    j = 0
    for k in range(nb):
        for i in range(ns):
            gs = gen2 if j & 1 else st
            ss = sim2 if j & 1 else sim
            if rec[i]:
                gs.wait_event(ev_sim[i])
            with torch.cuda.stream(gs):
                buf[i].fill_(float(k)).add_(torch.arange(buf.shape[1], device=buf.device,
                                                         dtype=buf.dtype))
            ev_gen[i].record(gs)
            ss.wait_event(ev_gen[i])
            with torch.cuda.stream(ss):
                torch.mul(buf[i], 2.0, out=out[i])
            ev_sim[i].record(ss)
            rec[i] = True
            j += 1
    for s, e in zip(side, ev_join):
        e.record(s)
        st.wait_event(e)


def main():
    dev = torch.device("cuda", 0)
    nb, ns, per = 2, 6, 1 << 16
    st = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(3)]
    ev_fork = torch.cuda.Event()
    ev_gen = [torch.cuda.Event() for _ in range(ns)]
    ev_sim = [torch.cuda.Event() for _ in range(ns)]
    ev_join = [torch.cuda.Event() for _ in range(3)]
    with torch.cuda.stream(st):
        buf = torch.zeros((ns, per), dtype=torch.float64, device=dev)
        out = torch.zeros_like(buf)
    torch.cuda.synchronize()
    print("eager warm-up", flush=True)
    with torch.cuda.stream(st):
        enqueue(st, side, ev_fork, ev_gen, ev_sim, ev_join, buf, out, nb, ns)
    torch.cuda.synchronize()
    ref = out.clone()
    print("capture (torch.cuda.graph, default error mode)", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        enqueue(st, side, ev_fork, ev_gen, ev_sim, ev_join, buf, out, nb, ns)
    print("captured", flush=True)
    for r in range(2):
        out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        if not torch.equal(out, ref):
            print(f"replay {r}: WRONG output", flush=True)
            return 1
    print("ok: torch-only fork/join captured and replayed twice, output equal", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

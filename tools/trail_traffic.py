"""HBM bytes of the trailing pipeline (tools/evidence.sh trailtraffic): sums FETCH_SIZE and
WRITE_SIZE over the generator's row-range launches (ocx_gen_wave_kernel, d = 64 forms) and
the chunked lean FTRL launches (ocx_alg_pipe_kernel, MINW = 4, CHUNK) of
`trail_probe.py --cases t1e5 --only-trailing --check 0` (a warm call and a timed call of
engine.gT_max), and prices them against the algorithmic 8(d+1) B per timestep each way (the
generator's write of z and y, the FTRL pass's one read).  gfx950's streaming reads count
FETCH_SIZE at half the bytes (MI355X_MICROARCH.md, HBM section): read = 2 x FETCH_SIZE x 1024.

    python tools/trail_traffic.py FETCH_DIR WRITE_DIR RUNS T [d]"""
import csv
import glob
import json
import os
import sys


def side_of(k):
    if k.startswith("void ocx_gen_wave_kernel<0, 64,"):  # either d = 64 form (the launcher picks)
        return "gen"
    if "ocx_alg_pipe_kernel<" in k:
        args = [x.strip() for x in k.split("<", 1)[1].split(">", 1)[0].split(",")]
        if args[4:6] == ["4", "true"]:
            return "ftrl"
    return None


def per_side(d, counter):
    out = {"gen": [0.0, set()], "ftrl": [0.0, set()]}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            side = side_of(r["Kernel_Name"])
            if side is None:
                continue
            out[side][0] += float(r["Counter_Value"])
            out[side][1].add((f, r["Dispatch_Id"]))
    return {s: (v[0], len(v[1])) for s, v in out.items()}


def main():
    fetch = per_side(sys.argv[1], "FETCH_SIZE")
    write = per_side(sys.argv[2], "WRITE_SIZE")
    runs, T = int(sys.argv[3]), int(sys.argv[4])
    d = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    calls = 2  # trail_probe: a warm call and the timed one
    alg = calls * runs * T * (8 * d + 8)
    res = {"runs": runs, "T": T, "d": d, "calls": calls, "alg_bytes_each_way": alg}
    for side in ("gen", "ftrl"):
        rd = 2.0 * fetch[side][0] * 1024.0
        wr = write[side][0] * 1024.0
        res[side] = {"dispatches": fetch[side][1], "read_bytes": rd, "write_bytes": wr,
                     "read_over_alg": rd / alg, "write_over_alg": wr / alg}
    tot = sum(res[s]["read_bytes"] + res[s]["write_bytes"] for s in ("gen", "ftrl"))
    res["total_over_2x_alg"] = tot / (2 * alg)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

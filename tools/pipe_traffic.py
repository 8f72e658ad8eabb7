"""HBM bytes of the overlapped pipeline (tools/evidence.sh pipetraffic): sums FETCH_SIZE and
WRITE_SIZE over the generator's range launches (ocx_gen_wave_kernel, OV form) and the lean
FTRL launches (ocx_alg_pipe_kernel, MINW = 4) of the probe's pipelined batches, and prices
them against the algorithmic 8(d+1) B per timestep each way (the generator's write of z and
y, the FTRL pass's one read).  gfx950's streaming reads count FETCH_SIZE at half the bytes
(MI355X_MICROARCH.md, HBM section): read = 2 x FETCH_SIZE x 1024.

    python tools/pipe_traffic.py FETCH_DIR WRITE_DIR"""
import csv
import glob
import json
import os
import sys

B, T, D = 32768, 10000, 64


def per_kernel(d, counter):
    out = {"gen": [0.0, set()], "ftrl": [0.0, set()]}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"]
            if "ocx_gen_wave_kernel<0, 64, false, false, 5>" in k:
                side = "gen"
            elif "ocx_alg_pipe_kernel<" in k and [x.strip() for x in k.split("<", 1)[1].split(">", 1)[0].split(",")][5:6] == ["4"]:
                side = "ftrl"
            else:
                continue
            out[side][0] += float(r["Counter_Value"])
            out[side][1].add((f, r["Dispatch_Id"]))
    return {s: (v[0], len(v[1])) for s, v in out.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    # the probe runs a warm-up call of one batch and the timed call of OCX_PROBE_NB batches
    nb = int(os.environ.get("OCX_PROBE_NB", 2)) + 1
    alg = B * T * (8 * D + 8)
    res = {"batches": nb, "B": B, "T": T, "d": D, "alg_bytes_per_batch_each_way": alg}
    for side in ("gen", "ftrl"):
        rd = 2.0 * fetch[side][0] * 1024.0 / nb
        wr = write[side][0] * 1024.0 / nb
        res[side] = {"dispatches": fetch[side][1], "read_bytes_per_batch": rd,
                     "write_bytes_per_batch": wr,
                     "read_over_alg": rd / alg, "write_over_alg": wr / alg}
    tot = sum(res[s]["read_bytes_per_batch"] + res[s]["write_bytes_per_batch"] for s in ("gen", "ftrl"))
    res["total_over_2x_alg"] = tot / (2 * alg)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

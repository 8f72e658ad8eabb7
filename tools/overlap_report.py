"""Concurrency of the overlapped pipeline from a rocprofv3 --kernel-trace directory
(tools/evidence.sh overlaptrace): the generator's range launches (ocx_gen_wave_kernel, OV
form) and the lean FTRL launches (ocx_alg_pipe_kernel, MINW = 4) — how much of the FTRL
kernels' time ran while a generator launch was running, and the wall time of the pipelined
batches against the sum of their kernels' times.

    python tools/overlap_report.py DIR"""
import csv
import glob
import json
import os
import sys


def intervals(rows, pred):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if pred(r["Kernel_Name"]))


def union(iv):
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    """Total length of the intersection of two sorted, disjoint interval lists."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s = max(a[i][0], b[j][0])
        e = min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    # the pipelined launches: the generator's four-wave OV form and the 4-waves-per-SIMD FTRL
    gen = intervals(rows, lambda k: "ocx_gen_wave_kernel<0, 64, false, false, 4>" in k or
                    "ocx_gen_wave_kernel<0, 64, false, false, 5>" in k)
    # the lean FTRL form: MINW = 4 (template argument 6; a seventh, FQ, may follow)
    ftrl = intervals(rows, lambda k: "ocx_alg_pipe_kernel<" in k and
                     [x.strip() for x in k.split("<", 1)[1].split(">", 1)[0].split(",")][5:6] == ["4"])
    gu, fu = union([list(x) for x in gen]), union([list(x) for x in ftrl])
    ov = overlap(gu, fu)
    ftrl_busy = sum(e - s for s, e in fu)
    gen_busy = sum(e - s for s, e in gu)
    span = (max(gu[-1][1], fu[-1][1]) - min(gu[0][0], fu[0][0])) if gu and fu else 0
    print(json.dumps({
        "gen_launches": len(gen), "ftrl_launches": len(ftrl),
        "gen_busy_ms": gen_busy / 1e6, "ftrl_busy_ms": ftrl_busy / 1e6,
        "ftrl_time_overlapped_with_gen_ms": ov / 1e6,
        "ftrl_overlapped_frac": ov / ftrl_busy if ftrl_busy else None,
        "span_ms": span / 1e6,
        "span_vs_sum_of_kernels": span / (gen_busy + ftrl_busy) if gen_busy + ftrl_busy else None,
        "source": os.path.relpath(files[0]) if files else None}))


if __name__ == "__main__":
    main()

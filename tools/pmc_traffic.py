"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs into HBM bytes per kernel launch.

    python tools/pmc_traffic.py --fetch DIR_OR_CSV --write DIR_OR_CSV --kernel ocx_alg_kernel \
        --B 32768 --T 10000 --d 64 --P 4 [--out profiles/traffic.json]

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  * FETCH_SIZE / WRITE_SIZE are in KiB;
  * FETCH_SIZE reads exactly 1/2 of the bytes of a wide (16 B/lane) coalesced streaming
    read, so the read side is 2 × FETCH_SIZE × 1024 (the kernel's z tiles are 16-B
    dwordx4 loads);
  * WRITE_SIZE is exact for 16-B stores; this kernel writes only B doubles.
Counters are collected in separate passes (one counter per pass) on the same command.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def _csv(path: str) -> str:
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
        if not c:
            raise SystemExit(f"no counter_collection.csv under {path}")
        return c[0]
    return path


def per_dispatch(path: str, counter: str, kernel: str):
    vals = {}
    with open(_csv(path)) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="ocx_alg_kernel",
                    help="substring of the kernel's name the dispatches must contain")
    ap.add_argument("--label", default=None,
                    help="kernel name recorded in the output (default: --kernel); bench.py "
                         "matches it against the kernel family its layout runs")
    ap.add_argument("--B", type=int, required=True)
    ap.add_argument("--T", type=int, required=True)
    ap.add_argument("--d", type=int, required=True)
    ap.add_argument("--P", type=int, required=True)
    ap.add_argument("--passes", type=int, default=2,
                    help="passes over z per launch: 2 = streamed comparator, 1 = closed form")
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit("kernel not found in the counter CSVs")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    read_bytes = 2.0 * f_kib * 1024.0
    write_bytes = w_kib * 1024.0
    alg = a.B * a.T * a.passes * (8 * a.d + 8)
    out = {"kernel": a.label or a.kernel, "kernel_match": a.kernel, "B": a.B, "T": a.T, "d": a.d, "P": a.P,
           "comparator": "closed" if a.passes == 1 else "two-pass",
           "dispatches": len(fetch), "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
           "hbm_read_bytes_per_launch": read_bytes, "hbm_write_bytes_per_launch": write_bytes,
           "hbm_bytes_per_launch": read_bytes + write_bytes,
           "alg_bytes_per_launch": alg, "traffic_over_alg": (read_bytes + write_bytes) / alg,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 16-B streaming read), "
                         "write = WRITE_SIZE x 1024"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

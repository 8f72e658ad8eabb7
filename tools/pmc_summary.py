"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches and XCDs).

    python tools/pmc_summary.py DIR [DIR ...] [--kernel SUBSTR]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--by-grid", action="store_true",
                    help="one group per (kernel, grid size): launches of one kernel at several sizes")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if a.kernel not in k:
                    continue
                k = k[:70]
                if a.by_grid:
                    k = f"{k} grid={r.get('Grid_Size', '?')}"
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((f, r["Dispatch_Id"]))
    for k, v in agg.items():
        print(f"{k}  (dispatches: {len(disp[k])})")
        for c, x in sorted(v.items()):
            print(f"    {c:24s} {x:.4e}")


if __name__ == "__main__":
    main()

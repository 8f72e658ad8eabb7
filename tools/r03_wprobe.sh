#!/bin/bash
# Round 3: WRITE_SIZE calibration of the generator's 8-B-per-lane store shapes (tools/wprobe.hip).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/wp
export TMPDIR=/tmp
for m in ${MODES:-0 1 2}; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/wp/m$m" -o run -- "$R/tune_r03/wprobe" $m > gpurun_out/wp/m$m.log 2>&1 || { echo "probe $m failed"; tail -5 gpurun_out/wp/m$m.log; exit 4; }
  grep "bytes per launch" gpurun_out/wp/m$m.log
done
python3 - <<'PY'
import csv, glob, json
import os
for m in [int(x) for x in os.environ.get("MODES", "0 1 2").split()]:
    f = glob.glob(f"gpurun_out/wp/m{m}/**/*counter_collection.csv", recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "WRITE_SIZE":
            v[r["Dispatch_Id"]] = v.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    n = 8 * 2048 * 1000 * 128 * 8
    print(json.dumps({"mode": m, "bytes": n, "write_size_bytes": [x * 1024 for x in v.values()],
                      "ratio": [x * 1024 / n for x in v.values()]}))
PY

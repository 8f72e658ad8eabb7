#!/bin/bash
# Exact-mode lane splits for the bench shape, then the sweep perf lines.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/bench_lanes.log
for L in -2 -8 -16 1; do
  timeout -k 10 600 python bench.py --lanes $L --steps 6 --warmup 1 --cpu-seconds 1 > gpurun_out/bench_l.log 2>&1 || { echo "bench lanes=$L failed"; tail -5 gpurun_out/bench_l.log; exit 3; }
  grep '^{' gpurun_out/bench_l.log >> gpurun_out/bench_lanes.log
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_lanes.log"):
    r = json.loads(l)
    print(r["config"]["lanes_per_seq"], r["config"]["coords_per_lane"], round(r["value"] / 1e9, 3), r["roofline"]["frac"], r["parity"]["bitexact"])
PY
timeout -k 10 600 python tools/perf_extra.py sweep > gpurun_out/perf_sweep.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_sweep.log | cut -c1-200
exit $rc

#!/bin/bash
# configs[4] shape (d=1024, T=1e4): exact-mode lane splits vs tree mode.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/bench_d1024.log
for L in -64 -32 -16 0; do
  timeout -k 10 600 python bench.py --d 1024 --B 2048 --lanes $L --steps 3 --warmup 1 --cpu-seconds 1 > gpurun_out/bench_l.log 2>&1 || { echo "bench lanes=$L failed"; tail -5 gpurun_out/bench_l.log; exit 3; }
  grep '^{' gpurun_out/bench_l.log >> gpurun_out/bench_d1024.log
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_d1024.log"):
    r = json.loads(l)
    c = r["config"]
    print(c["lanes_per_seq"], c["coords_per_lane"], c["sums"], round(r["value"] / 1e9, 3), round(r["roofline"]["frac"], 3), r["parity"])
PY

#!/bin/bash
# configs[3] g(T) sweep (d=64) and configs[4] (d=1024) at the default lanes (OCX_LANES_BEST)
# and in exact mode; then the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_best.jsonl || { echo "sweep best failed"; exit 2; }
cut -c1-250 gpurun_out/sweep_best.jsonl
timeout -k 10 600 python tools/perf_extra.py --lanes 1 sweep > gpurun_out/sweep_exact.jsonl || { echo "sweep exact failed"; exit 3; }
cut -c1-250 gpurun_out/sweep_exact.jsonl
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 5; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json; cut -c1-300 gpurun_out/bench_default.json

#!/bin/bash
# Where the T=100 / T=1e3 sweep points spend their time: per-dispatch kernel trace.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/perf_extra.py --Ts 100,1000 sweep > gpurun_out/t100_sweep.log 2>&1 || { tail -20 gpurun_out/t100_sweep.log; exit 2; }
cat gpurun_out/t100_sweep.log
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_t100"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_t100" -o t100 --output-format csv -- python3 "$R/tools/perf_extra.py" --Ts 100,1000 sweep > "$R/gpurun_out/prof_t100.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_t100.log"; exit 3; }
find "$R/gpurun_out/prof_t100" -name '*.csv' | head

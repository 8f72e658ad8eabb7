#!/bin/bash
# Parity suite, the d=64 g(T) sweep points (configs[3]) and kernel-trace stats of prof_long.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/perf_extra.py sweep > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 3; }
grep '^{' gpurun_out/sweep.log
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_long"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_long" -o long --output-format csv -- python3 "$R/tools/perf_extra.py" prof_long > "$R/gpurun_out/prof_long.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_long.log"; exit 5; }
grep '^{' "$R/gpurun_out/prof_long.log"
cut -c1-60,150-230 "$R/gpurun_out/prof_long/long_kernel_stats.csv" | head -8

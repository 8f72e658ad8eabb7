#!/bin/bash
# T=100 sweep point: HIP runtime API trace (where the host time between kernels goes)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/rt_t100"
timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d "$R/gpurun_out/rt_t100" -o rt -- python3 "$R/tools/perf_extra.py" --Ts 100 sweep > "$R/gpurun_out/rt_t100.log" 2>&1 || { tail -20 "$R/gpurun_out/rt_t100.log"; exit 3; }
grep '^{' "$R/gpurun_out/rt_t100.log"
find "$R/gpurun_out/rt_t100" -name '*.csv'

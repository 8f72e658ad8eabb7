#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_driver"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_driver" -o drv --output-format csv -- python3 "$R/tools/perf_extra.py" driver > "$R/gpurun_out/prof_driver.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_driver.log"; exit 5; }
grep -v amdgpu "$R/gpurun_out/prof_driver.log" | grep '^{' | cut -c1-200
head -12 "$R"/gpurun_out/prof_driver/drv_kernel_stats.csv | cut -c1-220

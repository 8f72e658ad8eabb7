#!/bin/bash
# Closed-form comparators: GPU suite, configs[2] (fused exact), the d=64 g(T) sweep and
# configs[4] with the closed-form default.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 500 python tools/perf_extra.py config3 > gpurun_out/c3.log 2>&1 || { tail -20 gpurun_out/c3.log; exit 3; }
grep '^{' gpurun_out/c3.log
timeout -k 10 500 python tools/perf_extra.py sweep > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 4; }
grep '^{' gpurun_out/sweep.log
timeout -k 10 500 python tools/perf_extra.py config4 > gpurun_out/c4.log 2>&1 || { tail -20 gpurun_out/c4.log; exit 5; }
grep '^{' gpurun_out/c4.log

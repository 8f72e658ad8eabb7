#!/bin/bash
# BEST butterfly rule retuned for the one-pass kernel: GPU suite, few-wave probes, sweep,
# configs[4].
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python tools/batch_probe.py 3328x100000x64x128,1024x10000x64x128,2048x10000x64x128,2926x10000x1024x128 > gpurun_out/bp_best2.jsonl 2>/dev/null || exit 3
cat gpurun_out/bp_best2.jsonl
timeout -k 10 500 python tools/perf_extra.py sweep config4 > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 4; }
grep '^{' gpurun_out/sweep.log

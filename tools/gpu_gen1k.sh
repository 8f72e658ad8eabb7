#!/bin/bash
# d=1024 generator with full rounds (row spill to the ring's front): the GPU suite, then
# the d=1024 batch times and configs[4]'s g(T).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/batch_probe.py 3400x10000x1024x128,2048x10000x1024x128,32768x10000x64x128 > gpurun_out/bp_1k.jsonl 2>/dev/null || exit 3
cat gpurun_out/bp_1k.jsonl
timeout -k 10 500 python tools/perf_extra.py config4 > gpurun_out/config4.log 2>&1 || { tail -20 gpurun_out/config4.log; exit 4; }
grep '^{' gpurun_out/config4.log

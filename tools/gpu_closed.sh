#!/bin/bash
# Closed-form comparator: GPU suite, default bench (closed) and the two-pass bench.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench_closed.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_closed.log; exit 5; }
grep '^{' gpurun_out/bench_closed.log > gpurun_out/bench_closed.json; cat gpurun_out/bench_closed.json

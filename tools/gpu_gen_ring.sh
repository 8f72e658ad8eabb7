#!/bin/bash
# Generator low-LDS form (few-stream batches): parity of the generator and g(T) tests,
# then per-kernel batch times.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -k "generator or gT or families or full_size or closed or streamed or best_mode or resident" > gpurun_out/pytest_gen.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
timeout -k 10 300 python tools/batch_probe.py 32768x10000x64x128,4900x100000x64x128,5000x2000x64x0,3328x100000x64x128 > gpurun_out/bp_lr.jsonl 2>/dev/null || exit 3
cat gpurun_out/bp_lr.jsonl
timeout -k 10 500 python tools/perf_extra.py sweep > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 4; }
grep '^{' gpurun_out/sweep.log

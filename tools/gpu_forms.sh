#!/bin/bash
# Generator form selection: tests, then the d=64 sweep.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -k "generator or gT or closed or streamed or best_mode or resident" > gpurun_out/pytest_gen.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
timeout -k 10 500 python tools/perf_extra.py sweep > gpurun_out/sweep_forms.log 2>&1 || { tail -20 gpurun_out/sweep_forms.log; exit 4; }
grep '^{' gpurun_out/sweep_forms.log | cut -c1-200

#!/bin/bash
# GPU pass: parity suite, then an optional tuning sweep (TUNE_LANES).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
  grep -v amdgpu.ids gpurun_out/bench.log
fi
if [ -n "${TUNE_LANES:-}" ]; then
  timeout -k 10 800 python tools/tune.py --lanes "$TUNE_LANES" --probe 0 > gpurun_out/tune.log 2>&1; rc2=$?
  grep -v amdgpu.ids gpurun_out/tune.log; exit $rc2
fi
exit $rc

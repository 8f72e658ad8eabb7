#!/bin/bash
# Full GPU pass: parity suite, perf lines (generator, sweep, drivers), default bench.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/perf_extra.py ${PERF:-gen sweep driver config3 exact_driver} > gpurun_out/perf_full.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_default.log
exit $rc

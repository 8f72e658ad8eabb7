#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/perf_extra.py config3 exact_driver > gpurun_out/perf_fused.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_fused.log | cut -c1-330
exit $rc

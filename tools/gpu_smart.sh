#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "smart or driver" > gpurun_out/pytest_smart.log 2>&1
rc=$?; echo "pytest(smart) rc=$rc"; tail -15 gpurun_out/pytest_smart.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/perf_extra.py smart driver > gpurun_out/perf_smart.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_smart.log | cut -c1-250
exit $rc

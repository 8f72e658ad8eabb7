#!/bin/bash
# Generator pass: the generator / streamed parity tests first, then the full GPU suite
# and the generation throughput lines.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "generator or streamed or gT or driver or families" > gpurun_out/pytest_gen.log 2>&1
rc=$?; echo "pytest(gen) rc=$rc"; tail -15 gpurun_out/pytest_gen.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/perf_extra.py gen sweep > gpurun_out/perf_gen.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_gen.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(all) rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
exit $rc

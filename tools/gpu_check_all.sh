#!/bin/bash
# Parity suite; FTRL kernel vs the HEAD library at the bench and few-wave shapes; the
# d=64 g(T) sweep points; configs[4] (d=1024) g(T) in exact and butterfly modes.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/tune.py --B 32768 --T 10000 --d 64 --lanes=1 --variants head --probe 0 --rounds 3 > gpurun_out/all_bench.log 2>&1 || { tail -20 gpurun_out/all_bench.log; exit 3; }
grep '^{' gpurun_out/all_bench.log | cut -c1-200
timeout -k 10 400 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes=1 --variants head --probe 0 --rounds 2 > gpurun_out/all_small.log 2>&1 || { tail -20 gpurun_out/all_small.log; exit 4; }
grep '^{' gpurun_out/all_small.log | cut -c1-200
timeout -k 10 400 python tools/perf_extra.py sweep > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 5; }
grep '^{' gpurun_out/sweep.log
timeout -k 10 400 python tools/perf_extra.py config4 > gpurun_out/c4.log 2>&1 || { tail -20 gpurun_out/c4.log; exit 6; }
grep '^{' gpurun_out/c4.log

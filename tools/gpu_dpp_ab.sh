#!/bin/bash
# Parity suite; FTRL kernel vs the HEAD library: bench shape, few-wave exact, d=1024
# exact and butterfly.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/tune.py --B 32768 --T 10000 --d 64 --lanes=1 --variants head --probe 0 --rounds 3 > gpurun_out/dpp_bench.log 2>&1 || { tail -20 gpurun_out/dpp_bench.log; exit 3; }
grep '^{' gpurun_out/dpp_bench.log | cut -c1-200
timeout -k 10 400 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes=1 --variants head --probe 0 --rounds 2 > gpurun_out/dpp_small.log 2>&1 || { tail -20 gpurun_out/dpp_small.log; exit 4; }
grep '^{' gpurun_out/dpp_small.log | cut -c1-200
timeout -k 10 400 python tools/tune.py --B 2048 --T 10000 --d 1024 --lanes=1,0 --variants head --probe 0 --rounds 2 > gpurun_out/dpp_d1024.log 2>&1 || { tail -20 gpurun_out/dpp_d1024.log; exit 5; }
grep '^{' gpurun_out/dpp_d1024.log | cut -c1-200

#!/bin/bash
# Parity suite, then the FTRL kernel at few-wave shapes (exact lane splits) and the
# default bench line (headline kernel must not regress).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes=-4,-8,-16 --probe 0 --rounds 2 > gpurun_out/chain_d64.log 2>&1 || { tail -20 gpurun_out/chain_d64.log; exit 3; }
grep '^{' gpurun_out/chain_d64.log
timeout -k 10 400 python tools/tune.py --B 2048 --T 10000 --d 1024 --lanes=-32 --probe 0 --rounds 2 > gpurun_out/chain_d1024.log 2>&1 || { tail -20 gpurun_out/chain_d1024.log; exit 4; }
grep '^{' gpurun_out/chain_d1024.log
timeout -k 10 400 python bench.py --cpu-seconds 2 > gpurun_out/bench_chain.log 2>&1 || { tail -20 gpurun_out/bench_chain.log; exit 5; }
grep '^{' gpurun_out/bench_chain.log | cut -c1-400

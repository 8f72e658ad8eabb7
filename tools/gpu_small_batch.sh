#!/bin/bash
# Lane splits of the FTRL kernel at capacity-limited (few-wave) batch shapes:
# d=64, T=1e5, 3328 sequences (the resident g(T) batch at T=1e5) and d=1024, T=1e4, 2048.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes=-1,-2,-4,-8,-16,-32,0 --probe 0 --rounds 2 > gpurun_out/small_d64.log 2>&1 || { tail -20 gpurun_out/small_d64.log; exit 3; }
grep '^{' gpurun_out/small_d64.log
timeout -k 10 400 python tools/tune.py --B 2048 --T 10000 --d 1024 --lanes=-16,-32,-64,0 --variants nowide --probe 0 --rounds 2 > gpurun_out/small_d1024.log 2>&1 || { tail -20 gpurun_out/small_d1024.log; exit 4; }
grep '^{' gpurun_out/small_d1024.log

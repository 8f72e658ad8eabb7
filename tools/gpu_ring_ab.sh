#!/bin/bash
# Ring-depth variants of the FTRL kernel at the few-wave exact shape (d=64, T=1e5,
# 3328 sequences, 8 lanes) and a mid-size batch.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
V=${VARIANTS:-nb6,nb8,nb8p8,p8}
timeout -k 10 400 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes=-8 --variants $V --probe 0 --rounds 2 > gpurun_out/ring_small.log 2>&1 || { tail -20 gpurun_out/ring_small.log; exit 4; }
grep '^{' gpurun_out/ring_small.log | cut -c1-200
timeout -k 10 400 python tools/tune.py --B 8192 --T 10000 --d 64 --lanes=-8 --variants $V --probe 0 --rounds 2 > gpurun_out/ring_mid.log 2>&1 || { tail -20 gpurun_out/ring_mid.log; exit 5; }
grep '^{' gpurun_out/ring_mid.log | cut -c1-200

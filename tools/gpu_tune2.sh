#!/bin/bash
# Generator section costs (tuning builds) and few-wave ring depth.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_gen.py --variants nostore,nonorm,noparse,nostore_nonorm,all3 > gpurun_out/tune_gen.jsonl || exit 2
cat gpurun_out/tune_gen.jsonl | cut -c1-200
: > gpurun_out/tune_ring.jsonl
for B in 3328 4900; do
timeout -k 10 300 python tools/tune.py --B $B --T 100000 --d 64 --lanes 16,8,1 --probe 0 --rounds 2 --variants nb12,nb16 | sed "s/^{/{\"B\": $B, /" >> gpurun_out/tune_ring.jsonl || exit 3
done
cut -c1-200 gpurun_out/tune_ring.jsonl

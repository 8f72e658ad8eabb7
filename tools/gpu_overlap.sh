#!/bin/bash
# Does capping the generator's resident waves let it overlap the FTRL kernel?
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/overlap.jsonl
for W in 0 4 3 2; do
  OCX_GEN_WAVES_PER_SIMD=$W timeout -k 10 300 python tools/overlap_probe.py --cases 16384x10000x64 --nbatch 6 --lanes 1 | sed "s/^{/{\"gen_waves_per_simd\": $W, /" >> gpurun_out/overlap.jsonl || exit 2
done
cut -c1-400 gpurun_out/overlap.jsonl

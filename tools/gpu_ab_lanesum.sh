#!/bin/bash
# A/B of the FTRL step's tree-mode arithmetic: per-step scale (old) vs the 64-step scale
# table (new default) vs in-lane pairwise sums; per-kernel times on resident batches.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
CASES="4900x100000x64x128,32768x10000x64x128,3400x10000x1024x128,1000000x100x64x128,333334x1000x64x128"
for V in default stepscale pairwise; do
  if [ "$V" = default ]; then unset OCX_LIB; else export OCX_LIB="$R/tune_ab/libocx_$V.so"; fi
  timeout -k 10 400 python tools/batch_probe.py $CASES > gpurun_out/ab_$V.jsonl 2> gpurun_out/ab_$V.err || { tail gpurun_out/ab_$V.err; exit 3; }
  sed "s/^{/{\"variant\": \"$V\", /" gpurun_out/ab_$V.jsonl
done
unset OCX_LIB
# T = 1e5 few-wave batches: generation of batch k+1 beside the FTRL of batch k (half-size,
# double-buffered) vs serial
timeout -k 10 400 python tools/overlap2.py --B 2450 --T 100000 --nbatch 6 --splits "80:16,128:8" --tag t1e5 > gpurun_out/ov_t1e5.jsonl 2> gpurun_out/ov_t1e5.err || { tail gpurun_out/ov_t1e5.err; exit 4; }
cat gpurun_out/ov_t1e5.jsonl

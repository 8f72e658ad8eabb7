#!/bin/bash
# Few-wave FTRL batches: one-wave vs four-wave workgroups, exact chains vs butterfly.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/fewwave.jsonl; : > $out
for BW in 4 0; do
  OCX_BLOCK_WAVES=$BW timeout -k 10 300 python tools/tune.py --B 3328 --T 100000 --d 64 --lanes 1,-16,0,8,16 --probe 0 --rounds 2 | sed "s/^{/{\"block_waves\": $BW, \"B\": 3328, \"T\": 100000, \"d\": 64, /" >> $out || exit 3
  OCX_BLOCK_WAVES=$BW timeout -k 10 300 python tools/tune.py --B 2048 --T 10000 --d 1024 --lanes 1,0,32 --probe 0 --rounds 2 | sed "s/^{/{\"block_waves\": $BW, \"B\": 2048, \"T\": 10000, \"d\": 1024, /" >> $out || exit 4
done
cat $out | cut -c1-220

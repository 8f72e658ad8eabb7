#!/bin/bash
# Generation beside simulation with the generator's resident waves capped and the FTRL
# kernel at issue priority 3 (tune_ship/libocx_prio3.so).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/overlap2.jsonl
for W in 3 4 2; do
OCX_GEN_WAVES_PER_SIMD=$W OCX_LIB=$R/tune_ship/libocx_prio3.so timeout -k 10 300 python tools/overlap2.py --B 16384 --splits "" --tag prio3_cap$W >> gpurun_out/overlap2.jsonl 2>> gpurun_out/overlap2.err || { tail -20 gpurun_out/overlap2.err; exit 3; }
done
cat gpurun_out/overlap2.jsonl

#!/bin/bash
# Round 3: generation of batch k+1 beside the FTRL pass over batch k (two streams, double
# buffered; tools/overlap2.py) with the pipelined 8 x 8 kernel, plain and with the FTRL waves
# at issue priority 3.  Needs tune_r03/libocx_prio3.so: _build.build_variant("prio3",
# ["OCX_ALG_PRIO=3"], source="ocx_alg_pipe.hip", out_dir="tune_r03").
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap2.py --B 16384 --nbatch 6 --splits "" --tag base > gpurun_out/r03_overlap.jsonl 2> gpurun_out/r03_overlap.err || { echo "overlap failed"; tail -20 gpurun_out/r03_overlap.err; exit 2; }
OCX_LIB="$R/tune_r03/libocx_prio3.so" timeout -k 10 400 python -u tools/overlap2.py --B 16384 --nbatch 6 --splits "" --tag prio3 >> gpurun_out/r03_overlap.jsonl 2>> gpurun_out/r03_overlap.err || { echo "overlap prio failed"; tail -20 gpurun_out/r03_overlap.err; exit 3; }
for cap in 2 3; do
OCX_GEN_WAVES_PER_SIMD=$cap OCX_LIB="$R/tune_r03/libocx_prio3.so" timeout -k 10 400 python -u tools/overlap2.py --B 16384 --nbatch 6 --splits "" --tag prio3_cap$cap >> gpurun_out/r03_overlap.jsonl 2>> gpurun_out/r03_overlap.err || { echo "overlap cap failed"; tail -20 gpurun_out/r03_overlap.err; exit 4; }
done
cut -c1-260 gpurun_out/r03_overlap.jsonl

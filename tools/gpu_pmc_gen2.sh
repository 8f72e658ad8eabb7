#!/bin/bash
# SQ counters of the d = 64 generator alone (32768 x 1e4, one launch per pass), and its time.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 python tools/gen_only.py 32768 10000 64 3 > gpurun_out/gen_time.log 2>&1 || exit 2
cat gpurun_out/gen_time.log
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc_gen$i" -o pmc -- python3 "$R/tools/gen_only.py" 32768 10000 64 1 > "$R/gpurun_out/pmc_gen$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc_gen$i.log"; exit 3; }
done
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_gen1 gpurun_out/pmc_gen2 gpurun_out/pmc_gen3 > gpurun_out/pmc_gen_summary.txt 2>&1; cat gpurun_out/pmc_gen_summary.txt

#!/bin/bash
# Round 3: where the d = 64 generator's time goes.  Section-removal variants (tune_r03,
# wrong outputs, timing only) beside the product library, then three SQ counter passes of
# the product generator alone (32768 x 1e4, one launch per pass; <= 8 SQ counters a pass).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune_gen.py --rounds 3 --lanes 128 --dir tune_r03 --variants noparse,nowedge,cheapmul,nostore > gpurun_out/r03_gen_costs.jsonl 2> gpurun_out/r03_gen_costs.err || { echo "variants failed"; tail -20 gpurun_out/r03_gen_costs.err; exit 2; }
cat gpurun_out/r03_gen_costs.jsonl
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf "$R/gpurun_out/pmc_gen$i"
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc_gen$i" -o pmc -- python3 "$R/tools/gen_only.py" 32768 10000 64 1 > "$R/gpurun_out/pmc_gen$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc_gen$i.log"; exit 3; }
done
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_gen1 gpurun_out/pmc_gen2 gpurun_out/pmc_gen3 > gpurun_out/pmc_gen_summary.txt 2>&1; cat gpurun_out/pmc_gen_summary.txt

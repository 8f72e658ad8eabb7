#!/bin/bash
# SQ counters of the few-wave FTRL kernel (d=64, T=1e5, 4 900 sequences, 8 x 8 butterfly,
# one pass over z): what bounds its 61 % of the HBM roofline.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/fewwave_pmc.py"
rm -rf "$R/gpurun_out/pmc_fw_a" "$R/gpurun_out/pmc_fw_b"
mkdir -p "$R/gpurun_out"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_fw_a" -o pmc -- $CMD > "$R/gpurun_out/pmc_fw_a.log" 2>&1 || { echo "pmc a failed"; tail -20 "$R/gpurun_out/pmc_fw_a.log"; exit 8; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_fw_b" -o pmc -- $CMD > "$R/gpurun_out/pmc_fw_b.log" 2>&1 || { echo "pmc b failed"; tail -20 "$R/gpurun_out/pmc_fw_b.log"; exit 9; }
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_fw_a gpurun_out/pmc_fw_b --kernel ocx_alg_kernel > gpurun_out/pmc_fewwave_best.txt && cat gpurun_out/pmc_fewwave_best.txt

#!/bin/bash
# SQ counters of the few-wave exact FTRL kernel (d=64, T=1e5, 3328 sequences, 8 lanes),
# two passes, summarised per kernel.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/tune.py --B 3328 --T 100000 --d 64 --lanes=-8 --probe 0 --rounds 1"
rm -rf "$R/gpurun_out/pmc_as_a" "$R/gpurun_out/pmc_as_b"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_as_a" -o pmc -- $CMD > "$R/gpurun_out/pmc_as_a.log" 2>&1 || { echo "pmc a failed"; tail -20 "$R/gpurun_out/pmc_as_a.log"; exit 8; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_as_b" -o pmc -- $CMD > "$R/gpurun_out/pmc_as_b.log" 2>&1 || { echo "pmc b failed"; tail -20 "$R/gpurun_out/pmc_as_b.log"; exit 9; }
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_as_a gpurun_out/pmc_as_b --kernel ocx_alg_kernel

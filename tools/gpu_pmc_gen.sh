#!/bin/bash
# SQ counters of the generator (tools/perf_extra.py gen1), two passes + an optional
# VALU-mix pass (allowed to fail: counter names differ across ROCm releases).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/pmc_gen1a" "$R/gpurun_out/pmc_gen1b" "$R/gpurun_out/pmc_gen1c"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_gen1a" -o pmc -- python3 "$R/tools/perf_extra.py" gen1 > "$R/gpurun_out/pmc_gen1a.log" 2>&1 || { echo "pmc a failed"; tail -20 "$R/gpurun_out/pmc_gen1a.log"; exit 8; }
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc_gen1b" -o pmc -- python3 "$R/tools/perf_extra.py" gen1 > "$R/gpurun_out/pmc_gen1b.log" 2>&1 || { echo "pmc b failed"; tail -20 "$R/gpurun_out/pmc_gen1b.log"; exit 9; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$R/gpurun_out/pmc_gen1c" -o pmc -- python3 "$R/tools/perf_extra.py" gen1 > "$R/gpurun_out/pmc_gen1c.log" 2>&1 || { echo "pmc c failed (ignored)"; tail -5 "$R/gpurun_out/pmc_gen1c.log"; }
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_gen1a gpurun_out/pmc_gen1b gpurun_out/pmc_gen1c --kernel gen_wave

#!/bin/bash
# Round 3, final build: SQ counters of the d = 64 generator (one 32 768 x 1e4 x 64 launch
# after a warm-up launch) and its rocprofv3 kernel stats.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/gen_sq" "$R/gpurun_out/gen_stats"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/gen_sq" -o sq -- python3 "$R/tools/gen_only.py" 32768 10000 64 2 128 > "$R/gpurun_out/gen_sq.log" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/gen_sq.log"; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/gen_stats" -o gs -- python3 "$R/tools/gen_only.py" 32768 10000 64 5 128 > "$R/gpurun_out/gen_stats.log" 2>&1 || { echo "stats failed"; tail -20 "$R/gpurun_out/gen_stats.log"; exit 3; }
cd "$R" && python3 tools/pmc_summary.py --kernel gen_wave gpurun_out/gen_sq
head -3 gpurun_out/gen_stats/gs_kernel_stats.csv | cut -c1-200

#!/bin/bash
# Lean d=64 generator loop: generator/g(T) parity tests, generator times, SALU/VALU counts.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -k "generator or gT or closed or streamed or best_mode or resident or full_size or config_shapes" > gpurun_out/pytest_gen.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
for S in "32768 10000" "4900 100000" "131072 1000" "1000000 100"; do
  timeout -k 10 200 python tools/gen_only.py $S 64 3 || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d "$R/gpurun_out/pmc_lean" -o pmc -- python3 "$R/tools/gen_only.py" 32768 10000 64 1 > "$R/gpurun_out/pmc_lean.log" 2>&1 || { echo "pmc failed"; exit 4; }
cd "$R" && python tools/pmc_summary.py gpurun_out/pmc_lean --kernel ocx_gen_wave

#!/bin/bash
# Generator pass: parity of the generator paths, throughput, then SQ counters of gen1.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "generator or streamed or gT or driver or families" > gpurun_out/pytest_gen.log 2>&1
rc=$?; echo "pytest(gen) rc=$rc"; tail -15 gpurun_out/pytest_gen.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/perf_extra.py gen > gpurun_out/perf_gen.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_gen.log | tail -12
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_gen1a" -o pmc -- python3 "$R/tools/perf_extra.py" gen1 > "$R/gpurun_out/pmc_gen1a.log" 2>&1 || { echo "pmc a failed"; tail -20 "$R/gpurun_out/pmc_gen1a.log"; exit 8; }
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d "$R/gpurun_out/pmc_gen1b" -o pmc -- python3 "$R/tools/perf_extra.py" gen1 > "$R/gpurun_out/pmc_gen1b.log" 2>&1 || { echo "pmc b failed"; tail -20 "$R/gpurun_out/pmc_gen1b.log"; exit 9; }
echo done

#!/bin/bash
# Round 3: the d = 1024 generator's swizzled ring (OCX_GEN_SWZ1K) — generator parity on the
# default build, A/B against the unswizzled variant (bit identity + timings), LDS bank-conflict
# counters of both, then the whole GPU suite, smoke, bench and the sweep.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "generator" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "gen pytest failed"; tail -40 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
timeout -k 10 400 python -u tools/r03_gen_lib_ab.py swz1,swz0,u2 > gpurun_out/r03_swz_ab.jsonl 2> gpurun_out/r03_swz_ab.err || { echo "ab failed"; tail -20 gpurun_out/r03_swz_ab.err; exit 3; }
cat gpurun_out/r03_swz_ab.jsonl
for v in swz1 swz0; do
  OCX_LIB="$R/tune_r03/libocx_$v.so" timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace --stats -d gpurun_out/pmc_swz_$v -o pmc -- python3 tools/gen_only.py 2048 10000 1024 1 128 > gpurun_out/pmc_swz_$v.log 2>&1 || { echo "pmc $v failed"; tail -20 gpurun_out/pmc_swz_$v.log; exit 4; }
done
echo pmc done
bash tools/r03_check8.sh

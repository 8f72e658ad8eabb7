#!/bin/bash
# Round 3: labels staged through LDS (OCX_GEN_STAGE_Y) — A/B of the generator with and
# without (outputs compared, timed), then FETCH_SIZE / WRITE_SIZE of each on the bench batch.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/ys
export TMPDIR=/tmp
[ "${SKIP_AB:-0}" = 1 ] || timeout -k 10 400 python -u tools/r03_gen_lib_ab.py ${AB:-ys0,ys1} > gpurun_out/r03_ystage_ab.jsonl 2> gpurun_out/r03_ystage_ab.err || { echo "ab failed"; tail -20 gpurun_out/r03_ystage_ab.err; exit 3; }
[ "${SKIP_AB:-0}" = 1 ] || cat gpurun_out/r03_ystage_ab.jsonl
for v in ${PMCV:-ys0 ys1}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    OCX_LIB="$R/tune_r03/libocx_$v.so" timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/ys/${v}_$c" -o run -- python3 tools/gen_only.py 32768 10000 64 1 > gpurun_out/ys/${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; tail -5 gpurun_out/ys/${v}_$c.log; exit 4; }
  done
  python tools/pmc_traffic.py --fetch gpurun_out/ys/${v}_FETCH_SIZE --write gpurun_out/ys/${v}_WRITE_SIZE --kernel ocx_gen_wave_kernel --B 32768 --T 10000 --d 64 --P 4 --passes 1 --out gpurun_out/ys/traffic_$v.json || exit 5
done

#!/bin/bash
# ROUND 1 (two-pass comparator default). For the closed-form default use tools/gpu_final_r02.sh:
# this script times and counts every ocx_alg_kernel launch, two-pass ones included.
# End-of-round evidence for the bench kernel: smoke(), kernel-trace stats of the default
# bench command, and the two PMC HBM passes (FETCH_SIZE, WRITE_SIZE) -> traffic.json.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 2; }
tail -2 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_final" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_final" -o r01 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/prof_final.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_final.log"; exit 5; }
grep '^{' "$R/gpurun_out/prof_final.log" | cut -c1-200
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 6; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --out gpurun_out/traffic.json && head -8 gpurun_out/prof_final/r01_kernel_stats.csv | cut -c1-160
cd "$R" && cp gpurun_out/traffic.json profiles/traffic.json && timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 7; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json && cut -c1-300 gpurun_out/bench_default.json

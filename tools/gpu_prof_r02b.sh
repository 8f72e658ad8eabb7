#!/bin/bash
# Round-2 evidence for the default bench kernel (closed-form comparator, one pass over z):
# kernel-trace stats of the default bench command (no two-pass launches in the trace), the
# two PMC HBM passes (FETCH_SIZE, WRITE_SIZE) -> traffic.json, then the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_closed" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_closed" -o r02 --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --two-pass-steps 0 > "$R/gpurun_out/prof_closed.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_closed.log"; exit 5; }
grep '^{' "$R/gpurun_out/prof_closed.log" > "$R/gpurun_out/prof_closed_bench.json"; cut -c1-200 "$R/gpurun_out/prof_closed_bench.json"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 --two-pass-steps 0 --e2e-steps 0 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 6; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --passes 1 --out gpurun_out/traffic.json && head -8 gpurun_out/prof_closed/r02_kernel_stats.csv | cut -c1-200
cd "$R" && cp gpurun_out/traffic.json profiles/traffic.json && timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 7; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json && cut -c1-300 gpurun_out/bench_default.json

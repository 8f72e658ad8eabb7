#!/bin/bash
# Round-3 evidence set: GPU suite + smoke; the default bench line; rocprofv3 kernel stats of
# the default bench command (closed-form kernel only) and of the few-wave T=1e5 batches
# (pipelined kernel); the two PMC HBM passes (FETCH_SIZE, WRITE_SIZE) over the bench command
# with one end-to-end batch (FTRL kernel and generator); the d=64 g(T) sweep and configs[4];
# the general exact solver's timings.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r03.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r03.log; exit 4; }
grep '^{' gpurun_out/bench_r03.log > gpurun_out/bench_r03.json; cut -c1-300 gpurun_out/bench_r03.json
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_r03" "$R/gpurun_out/prof_fw" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03" -o r03 --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --two-pass-steps 0 > "$R/gpurun_out/prof_r03.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_r03.log"; exit 5; }
grep '^{' "$R/gpurun_out/prof_r03.log" > "$R/gpurun_out/prof_r03_bench.json"
OCX_PROBE_SHORT=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fw" -o fw --output-format csv -- python3 "$R/tools/r03_alg_probe.py" > "$R/gpurun_out/prof_fw.log" 2>&1 || { echo "rocprof fw failed"; tail -20 "$R/gpurun_out/prof_fw.log"; exit 6; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 --two-pass-steps 0 --e2e-steps 1 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 7; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --passes 1 --out gpurun_out/traffic.json > /dev/null && head -c 1500 gpurun_out/traffic.json; echo
head -8 gpurun_out/prof_r03/r03_kernel_stats.csv | cut -c1-160
head -8 gpurun_out/prof_fw/fw_kernel_stats.csv | cut -c1-160
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_r03.log 2>&1 || { tail -20 gpurun_out/sweep_r03.log; exit 8; }
grep '^{' gpurun_out/sweep_r03.log | cut -c1-220
timeout -k 10 300 python -u tools/r03_exact_probe.py > gpurun_out/r03_exact_probe.jsonl 2> gpurun_out/r03_exact_probe.err || { echo "exact probe failed"; tail -20 gpurun_out/r03_exact_probe.err; exit 9; }
cut -c1-250 gpurun_out/r03_exact_probe.jsonl

#!/bin/bash
# Round-3 evidence on the final build: the two PMC HBM passes (FETCH_SIZE, WRITE_SIZE) over
# the bench command (FTRL kernel and generator), then the default bench line reading that
# traffic, rocprofv3 kernel stats of the bench command, the GPU suite + smoke, and the d=64
# g(T) sweep and configs[4].
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_fin" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 --two-pass-steps 0 --e2e-steps 1 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 7; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --kernel ocx_alg_pipe_kernel --B 32768 --T 10000 --d 64 --P 8 --passes 1 --out gpurun_out/traffic.json > /dev/null && head -c 900 gpurun_out/traffic.json; echo
timeout -k 10 600 python bench.py --traffic gpurun_out/traffic.json > gpurun_out/bench_fin.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_fin.log; exit 4; }
grep '^{' gpurun_out/bench_fin.log > gpurun_out/bench_fin.json; cut -c1-400 gpurun_out/bench_fin.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fin" -o fin --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 --two-pass-steps 0 --traffic "$R/gpurun_out/traffic.json" > "$R/gpurun_out/prof_fin.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_fin.log"; exit 5; }
grep '^{' "$R/gpurun_out/prof_fin.log" > "$R/gpurun_out/prof_fin_bench.json"
head -6 "$R/gpurun_out/prof_fin/fin_kernel_stats.csv" | cut -c1-160
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_fin.log 2>&1 || { tail -20 gpurun_out/sweep_fin.log; exit 8; }
grep '^{' gpurun_out/sweep_fin.log | cut -c1-220

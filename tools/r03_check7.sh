#!/bin/bash
# Round 3: GPU suite + smoke on the current build (labels staged through LDS, 8-wave blocks,
# lane states), bench line, generator write traffic at P = 4 and P = 8, sweep + configs[4].
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/g7
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r03e.log 2>&1 || { tail -20 gpurun_out/bench_r03e.log; exit 4; }
tail -1 gpurun_out/bench_r03e.log | cut -c1-300
for P in 4 8; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/g7/p${P}_$c" -o run -- python3 tools/gen_only.py 32768 10000 64 1 $P > gpurun_out/g7/p${P}_$c.log 2>&1 || { echo "pmc $P $c failed"; tail -5 gpurun_out/g7/p${P}_$c.log; exit 5; }
  done
  python tools/pmc_traffic.py --fetch gpurun_out/g7/p${P}_FETCH_SIZE --write gpurun_out/g7/p${P}_WRITE_SIZE --kernel ocx_gen_wave_kernel --B 32768 --T 10000 --d 64 --P $P --passes 1 --out gpurun_out/g7/traffic_gen_p$P.json | cut -c1-400 || exit 6
  grep "ms per launch" gpurun_out/g7/p${P}_WRITE_SIZE.log
done
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_r03e.log 2>&1 || { tail -20 gpurun_out/sweep_r03e.log; exit 8; }
grep '^{' gpurun_out/sweep_r03e.log | cut -c1-200

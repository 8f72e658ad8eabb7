#!/bin/bash
# Round 3: GPU suite + smoke, bench, sweep + configs[4] after OCX_LANES_BEST took the 8 x 8
# butterfly for big d = 64 batches.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r03f.log 2>&1 || { tail -20 gpurun_out/bench_r03f.log; exit 4; }
tail -1 gpurun_out/bench_r03f.log | cut -c1-600
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_r03f.log 2>&1 || { tail -20 gpurun_out/sweep_r03f.log; exit 8; }
grep '^{' gpurun_out/sweep_r03f.log | cut -c1-200

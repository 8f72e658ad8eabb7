#!/bin/bash
# Round 2 (re-entry, rebuilt libocx.so): GPU suite, smoke, the configs[3] g(T) sweep
# (regrets to the host and g(T) reduced on device) and the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python tools/perf_extra.py sweep > gpurun_out/sweep_final.jsonl || { echo "sweep failed"; exit 4; }
cut -c1-400 gpurun_out/sweep_final.jsonl
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 5; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json; cut -c1-300 gpurun_out/bench_default.json

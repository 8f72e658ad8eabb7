#!/bin/bash
# GPU suite + smoke after a kernel change, then per-kernel times of the d=1024 / few-wave
# batches and the configs[3]/[4] sweeps.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
timeout -k 10 400 python tools/batch_probe.py 1000000x100x64x128,32768x10000x64x128,3400x10000x1024x128,4900x100000x64x128 > gpurun_out/bp_c.jsonl 2> gpurun_out/bp_c.err || { tail gpurun_out/bp_c.err; exit 4; }
cat gpurun_out/bp_c.jsonl
timeout -k 10 600 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_c.log 2>&1 || { tail -20 gpurun_out/sweep_c.log; exit 5; }
grep '^{' gpurun_out/sweep_c.log | cut -c1-220

#!/bin/bash
# Round 3: the pipelined butterfly FTRL kernel — full GPU suite, then timings vs the plain one.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/r03_alg_probe.py > gpurun_out/r03_alg_pipe.jsonl 2> gpurun_out/r03_alg_pipe.err || { echo "probe failed"; tail -20 gpurun_out/r03_alg_pipe.err; exit 3; }
cat gpurun_out/r03_alg_pipe.jsonl
OCX_ALG_NO_PIPE=1 timeout -k 10 300 python -u tools/r03_alg_probe.py > gpurun_out/r03_alg_nopipe.jsonl 2> gpurun_out/r03_alg_nopipe.err || { echo "probe2 failed"; tail -20 gpurun_out/r03_alg_nopipe.err; exit 4; }
cat gpurun_out/r03_alg_nopipe.jsonl

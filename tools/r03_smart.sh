#!/bin/bash
# Round 3: SMART O(T·d) kernel — its GPU tests, then the timing probe.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_smart.py tests/test_gpu_parity.py -k "smart or SMART" -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_smart.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_smart.log; exit 2; }
tail -3 gpurun_out/pytest_smart.log
timeout -k 10 600 python -u tools/r03_smart_probe.py > gpurun_out/r03_smart_probe.jsonl 2>gpurun_out/r03_smart_probe.err || { echo "probe failed"; tail -20 gpurun_out/r03_smart_probe.err; exit 3; }
cat gpurun_out/r03_smart_probe.jsonl

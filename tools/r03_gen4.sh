#!/bin/bash
# Round 3: generator variants (d = 1024 rows with the flat lane-state round; lane states
# advanced before the table lookup; the d = 64 unroll by two) against the default build:
# generator parity on the default build, then bit identity + timings.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "generator" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "gen pytest failed"; tail -40 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
timeout -k 10 400 python -u tools/r03_gen_lib_ab.py base,nou2,f1k,lse,f1klse > gpurun_out/r03_gen4_ab.jsonl 2> gpurun_out/r03_gen4_ab.err || { echo "ab failed"; tail -20 gpurun_out/r03_gen4_ab.err; exit 3; }
cat gpurun_out/r03_gen4_ab.jsonl

#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_gen.py --variants w4,w5,nowedge,noparse,nonorm --rounds 3 > gpurun_out/tune_gen4.jsonl || exit 2
cut -c1-200 gpurun_out/tune_gen4.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/pytest_gpu.log

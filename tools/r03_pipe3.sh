#!/bin/bash
# Round 3: full GPU suite on the current build (late-load ring in the pipelined kernel,
# prologue loads pinned in slot order), then few-wave FTRL timings: pipelined kernel at the
# default ring depth and at 7 / 12 slots (tune_r03 variants), and the plain kernel.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
for v in base nb7 nb12 nopipe; do
  unset OCX_LIB OCX_ALG_NO_PIPE
  case $v in nb*) export OCX_LIB=$R/tune_r03/libocx_$v.so;; nopipe) export OCX_ALG_NO_PIPE=1;; esac
  timeout -k 10 300 python -u tools/r03_alg_probe.py > gpurun_out/r03_alg3_$v.jsonl 2> gpurun_out/r03_alg3_$v.err || { echo "probe $v failed"; tail -20 gpurun_out/r03_alg3_$v.err; exit 5; }
  echo "== $v"; cut -c1-150 gpurun_out/r03_alg3_$v.jsonl
done

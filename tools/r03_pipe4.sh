#!/bin/bash
# Round 3: GPU suite on the current build, few-wave FTRL/FTL timings (pipelined kernel:
# uniform tile bases, running ||θ||², FTL as a template flag; and the plain kernel), and the
# general exact-FTL solver's timings.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
for v in base nopipe; do
  unset OCX_ALG_NO_PIPE
  [ $v = nopipe ] && export OCX_ALG_NO_PIPE=1 OCX_PROBE_SHORT=1
  timeout -k 10 400 python -u tools/r03_alg_probe.py > gpurun_out/r03_alg4_$v.jsonl 2> gpurun_out/r03_alg4_$v.err || { echo "probe $v failed"; tail -20 gpurun_out/r03_alg4_$v.err; exit 5; }
  echo "== $v"; cut -c1-170 gpurun_out/r03_alg4_$v.jsonl
done
unset OCX_ALG_NO_PIPE OCX_PROBE_SHORT
timeout -k 10 300 python -u tools/r03_exact_probe.py > gpurun_out/r03_exact_probe.jsonl 2> gpurun_out/r03_exact_probe.err || { echo "exact probe failed"; tail -20 gpurun_out/r03_exact_probe.err; exit 6; }
cat gpurun_out/r03_exact_probe.jsonl

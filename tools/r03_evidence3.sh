#!/bin/bash
# Round-3 evidence, third part: the general exact solver's timings, configs[2] end to end,
# the d=64 g(T) sweep and configs[4].
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r03_exact_probe.py > gpurun_out/r03_exact_probe.jsonl 2> gpurun_out/r03_exact_probe.err || { echo "exact probe failed"; tail -20 gpurun_out/r03_exact_probe.err; exit 9; }
cut -c1-250 gpurun_out/r03_exact_probe.jsonl
timeout -k 10 900 python tools/perf_extra.py config3 sweep config4 > gpurun_out/sweep_r03.log 2>&1 || { tail -20 gpurun_out/sweep_r03.log; exit 8; }
grep '^{' gpurun_out/sweep_r03.log | cut -c1-260

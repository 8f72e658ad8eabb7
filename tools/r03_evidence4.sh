#!/bin/bash
# Round-3 evidence, fourth part: the general exact solver's timings with its worst problem
# per shape; the d=64 g(T) sweep and configs[4] in a fresh process (nothing else holding HBM).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r03_exact_probe.py > gpurun_out/r03_exact_probe.jsonl 2> gpurun_out/r03_exact_probe.err || { echo "exact probe failed"; tail -20 gpurun_out/r03_exact_probe.err; exit 9; }
cut -c1-400 gpurun_out/r03_exact_probe.jsonl
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_r03b.log 2>&1 || { tail -20 gpurun_out/sweep_r03b.log; exit 8; }
grep '^{' gpurun_out/sweep_r03b.log | cut -c1-200

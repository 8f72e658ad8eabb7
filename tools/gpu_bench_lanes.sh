#!/bin/bash
# One-pass FTRL kernel at the bench shape (32768 x 1e4 x 64): lane layouts.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
C=""
for L in -1 -2 -4 -8 1 2 4 8 16; do C="$C,32768x10000x64x$L"; done
timeout -k 10 900 python tools/batch_probe.py ${C:1} > gpurun_out/bp_bench_lanes.jsonl 2>gpurun_out/bp.err || { tail gpurun_out/bp.err; exit 3; }
cut -c1-250 gpurun_out/bp_bench_lanes.jsonl

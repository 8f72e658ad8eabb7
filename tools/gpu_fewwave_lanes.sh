#!/bin/bash
# One-pass (closed-form comparator) FTRL on the few-wave batches: lane layouts.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
C=""
for L in 128 0 4 8 16 32 -4 -8 -16; do C="$C,4900x100000x64x$L"; done
for L in 128 32 16 64 -32; do C="$C,3400x10000x1024x$L"; done
timeout -k 10 900 python tools/batch_probe.py ${C:1} > gpurun_out/bp_lanes.jsonl 2>gpurun_out/bp_lanes.err || { tail gpurun_out/bp_lanes.err; exit 3; }
cat gpurun_out/bp_lanes.jsonl

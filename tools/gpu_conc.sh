#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/concurrency_probe.py > gpurun_out/conc.jsonl 2> gpurun_out/conc.err || { tail -20 gpurun_out/conc.err; exit 2; }
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/concurrency_probe.py >> gpurun_out/conc.jsonl 2>> gpurun_out/conc.err || { tail -20 gpurun_out/conc.err; exit 3; }
cat gpurun_out/conc.jsonl

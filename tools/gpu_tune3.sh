#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_gen.py --variants r8,r8w5,w8,w5,w4 --rounds 3 > gpurun_out/tune_gen3.jsonl || exit 2
cut -c1-200 gpurun_out/tune_gen3.jsonl

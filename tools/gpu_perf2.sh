#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python tools/perf_extra.py smart gen sweep driver > gpurun_out/perf_extra.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/perf_extra.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --B 8192 --steps 3 --warmup 1 --cpu-seconds 1 --dist-backend gloo > gpurun_out/bench_gloo2.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/bench_gloo2.log | tail -3
exit $rc

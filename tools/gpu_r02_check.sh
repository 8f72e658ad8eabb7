#!/bin/bash
# Round 2: GPU suite (incl. exact_ftl drop-in and multi-device tests), smoke, a 1-rank
# RCCL bench (nccl init + device all-gather) and the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-steps 1 --dist-backend nccl > gpurun_out/bench_nccl1.log 2>&1 || { echo "nccl1 failed"; tail -20 gpurun_out/bench_nccl1.log; exit 4; }
grep '^{' gpurun_out/bench_nccl1.log > gpurun_out/bench_nccl1.json; cut -c1-200 gpurun_out/bench_nccl1.json
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 5; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json; cut -c1-300 gpurun_out/bench_default.json

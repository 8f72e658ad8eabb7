#!/bin/bash
# Round 3, final tree: GPU suite + smoke, the default bench line (the driver's command), and a
# 2-rank torchrun rehearsal of bench.py over gloo on the one GPU (B = 8192 per rank).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_verify.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_verify.log; exit 4; }
grep '^{' gpurun_out/bench_verify.log | cut -c1-300
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --B 8192 --dist-backend gloo --e2e-steps 2 > gpurun_out/bench_gloo2.log 2>&1 || { echo "gloo2 failed"; tail -30 gpurun_out/bench_gloo2.log; exit 5; }
grep '^{' gpurun_out/bench_gloo2.log | cut -c1-400

#!/bin/bash
# Round-end rehearsal of what the driver runs: the GPU parity suite, smoke(), a 2-rank
# gloo rehearsal of the multi-GPU bench (both ranks on the one GPU, B=8192 each) and the
# default bench line.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --B 8192 --steps 3 --warmup 1 --cpu-seconds 1 --dist-backend gloo > gpurun_out/bench_gloo2.log 2>&1 || { echo "gloo2 failed"; tail -20 gpurun_out/bench_gloo2.log; exit 4; }
grep '^{' gpurun_out/bench_gloo2.log > gpurun_out/bench_gloo2.json; cut -c1-200 gpurun_out/bench_gloo2.json
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 5; }
grep '^{' gpurun_out/bench_default.log | cut -c1-300

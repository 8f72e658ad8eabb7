#!/bin/bash
# Round 3: the pipelined kernel's own tests; the generator's streamlined rejection round
# (tune_r03: rej1) against the general path (rej0), outputs compared and timed; the N>1 bench
# path rehearsed with two gloo ranks on the one GPU (smaller batches: they share its HBM).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1 || { echo "pipe tests failed"; tail -40 gpurun_out/pytest_pipe.log; exit 2; }
tail -3 gpurun_out/pytest_pipe.log
timeout -k 10 400 python -u tools/r03_gen_lib_ab.py rej0,rej1 > gpurun_out/r03_gen_rej_ab.jsonl 2> gpurun_out/r03_gen_rej_ab.err || { echo "gen A/B failed"; tail -20 gpurun_out/r03_gen_rej_ab.err; cat gpurun_out/r03_gen_rej_ab.jsonl; exit 4; }
cat gpurun_out/r03_gen_rej_ab.jsonl
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --B 8192 --steps 5 --warmup 1 --cpu-seconds 0 --e2e-steps 1 --two-pass-steps 0 --dist-backend gloo > gpurun_out/bench_gloo2.log 2>&1 || { echo "gloo2 failed"; tail -30 gpurun_out/bench_gloo2.log; exit 3; }
grep '^{' gpurun_out/bench_gloo2.log > gpurun_out/bench_gloo2.json; cut -c1-400 gpurun_out/bench_gloo2.json

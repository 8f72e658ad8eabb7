#!/bin/bash
# First GPU pass: parity tests, a small and a full bench, a kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --B 8192 --steps 5 --warmup 1 --cpu-seconds 3 > gpurun_out/bench_small.log 2>&1 || { echo "small bench failed"; tail -20 gpurun_out/bench_small.log; exit 3; }
tail -2 gpurun_out/bench_small.log
timeout -k 10 900 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_full.log 2>&1 || { echo "full bench failed"; tail -20 gpurun_out/bench_full.log; exit 4; }
tail -2 gpurun_out/bench_full.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o r01 --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 5; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head

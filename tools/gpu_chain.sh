#!/bin/bash
# Chained-sum change: full parity suite, then the bench and the d=1024 exact splits.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 1 --cpu-seconds 1 > gpurun_out/bench_chain.log 2>&1 || { tail -5 gpurun_out/bench_chain.log; exit 4; }
grep '^{' gpurun_out/bench_chain.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', r['value']/1e9, r['roofline']['frac'], r['parity'])"
bash tools/gpu_d1024.sh

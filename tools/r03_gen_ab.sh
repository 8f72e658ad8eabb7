#!/bin/bash
# Round 3: generator correctness (the device-generator parity tests on the default build)
# and A/B timings of the generator variants in tune_r03/ (built in the container).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "generator or gT or families or published or full_size or config" -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gen.log; exit 2; }
tail -2 gpurun_out/pytest_gen.log
timeout -k 10 300 python -u tools/tune_gen.py --dir tune_r03 --variants old,f32only,speconly,cheapmul --rounds 3 > gpurun_out/r03_gen_ab.jsonl 2> gpurun_out/r03_gen_ab.err || { echo "ab failed"; tail -20 gpurun_out/r03_gen_ab.err; exit 3; }
cat gpurun_out/r03_gen_ab.jsonl
timeout -k 10 300 python -u tools/tune_gen.py --dir tune_r03 --variants old --B 4900 --T 100000 --lanes 128 --rounds 2 >> gpurun_out/r03_gen_ab.jsonl 2>> gpurun_out/r03_gen_ab.err || { echo "ab2 failed"; exit 4; }
tail -2 gpurun_out/r03_gen_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_smart.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_smart.log 2>&1 || { echo "smart pytest failed"; tail -40 gpurun_out/pytest_smart.log; exit 5; }
tail -2 gpurun_out/pytest_smart.log
timeout -k 10 600 python -u tools/r03_smart_probe.py > gpurun_out/r03_smart_probe.jsonl 2>gpurun_out/r03_smart_probe.err || { echo "probe failed"; tail -20 gpurun_out/r03_smart_probe.err; exit 6; }
cat gpurun_out/r03_smart_probe.jsonl

#!/bin/bash
# Generator with the hand-scheduled 128-bit multiply-add (uniform base in SGPRs, one-xor
# sign): generator/g(T) parity tests, then batch times vs the __int128 build.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -k "generator or gT or families or full_size or closed or streamed or best_mode or resident" > gpurun_out/pytest_gen.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
CASES=32768x10000x64x128,4900x100000x64x128,2926x10000x1024x128
timeout -k 10 300 python tools/batch_probe.py $CASES | sed 's/^{/{"lib": "asm_mul", /' > gpurun_out/bp_mul.jsonl 2>/dev/null || exit 3
OCX_LIB=$R/tune_ship/libocx_int128mul.so timeout -k 10 300 python tools/batch_probe.py $CASES | sed 's/^{/{"lib": "int128_mul", /' >> gpurun_out/bp_mul.jsonl 2>/dev/null || exit 4
cut -c1-220 gpurun_out/bp_mul.jsonl

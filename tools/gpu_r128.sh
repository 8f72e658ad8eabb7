#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
OCX_LIB="$R/tune_build/libocx_r128.so" timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "generator or streamed or gT or driver or families" > gpurun_out/pytest_r128.log 2>&1
rc=$?; echo "pytest(r128) rc=$rc"; tail -15 gpurun_out/pytest_r128.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="r64 r128 r64 r128" bash tools/gpu_genvar.sh

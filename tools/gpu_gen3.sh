#!/bin/bash
# Generator iteration: parity of the generator paths, then variant throughput.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf -k "generator or streamed or gT or driver or families" > gpurun_out/pytest_gen.log 2>&1
rc=$?; echo "pytest(gen) rc=$rc"; tail -15 gpurun_out/pytest_gen.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-genw1 genw5 genw6}" bash tools/gpu_genvar.sh

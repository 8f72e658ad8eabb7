#!/bin/bash
# FTRL kernel A/B (tune_build variants) at the bench shape, after the parity suite.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/tune.py --lanes ${LANES:-1} --variants ${VARIANTS:-alg_lb2} --rounds 6 --probe 0 > gpurun_out/tune_ab.log 2>&1; rc=$?
grep '^{' gpurun_out/tune_ab.log
exit $rc

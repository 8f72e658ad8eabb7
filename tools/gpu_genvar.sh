#!/bin/bash
# Generator register-budget variants (tune_build/libocx_genw*.so): gen1 throughput each.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/genvar.log
for v in ${VARIANTS:-genw1 genw5 genw6 genw8}; do
  echo "variant $v" >> gpurun_out/genvar.log
  OCX_LIB="$R/tune_build/libocx_$v.so" timeout -k 10 300 python tools/perf_extra.py gen1 >> gpurun_out/genvar.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/genvar.log; exit 3; }
done
grep -v amdgpu gpurun_out/genvar.log

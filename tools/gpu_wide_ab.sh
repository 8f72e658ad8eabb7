#!/bin/bash
# Parity suite, then kernel-trace stats of prof_long (configs[4] d=1024 exact and a
# T=1e5 d=64 sweep point) for: the default library, OCX_ALG_DEEP=0 (no deep register
# ring for small batches) and the library built without the wide-chain FTRL/comparator
# variant (tune_build/libocx_nowide.so).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in default nodeep nowide; do
  rm -rf "$R/gpurun_out/ab_$v"
  if [ "$v" = nodeep ]; then export OCX_ALG_DEEP=0; else unset OCX_ALG_DEEP; fi
  if [ "$v" = nowide ]; then export OCX_LIB="$R/tune_build/libocx_nowide.so"; else unset OCX_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ab_$v" -o ab --output-format csv -- python3 "$R/tools/perf_extra.py" prof_long > "$R/gpurun_out/ab_$v.log" 2>&1 || { echo "$v failed"; tail -20 "$R/gpurun_out/ab_$v.log"; exit 5; }
  echo "== $v"; grep '^{' "$R/gpurun_out/ab_$v.log"
  grep ocx_alg "$R/gpurun_out/ab_$v/ab_kernel_stats.csv" | cut -c1-40,100-200
done

#!/bin/bash
# Second GPU pass: full parity suite, PMC HBM traffic of the FTRL kernel (two passes).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 5; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --out gpurun_out/traffic.json

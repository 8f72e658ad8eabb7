#!/bin/bash
# Generator probe (where the g(T) sampler's time goes), then the end-of-round profiles of
# the default bench: kernel-trace stats and the two PMC HBM passes.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out build
hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/gen_probe.hip \
  -I online_convex_optimization_amd/csrc -o build/gen_probe || exit 2
timeout -k 10 300 build/gen_probe 262144 2048 > gpurun_out/gen_probe.log 2>&1 || { echo "probe failed"; cat gpurun_out/gen_probe.log; exit 3; }
timeout -k 10 300 build/gen_probe 32768 4096 >> gpurun_out/gen_probe.log 2>&1 || { echo "probe2 failed"; cat gpurun_out/gen_probe.log; exit 3; }
cat gpurun_out/gen_probe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_exact" -o r01 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/prof_exact.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_exact.log"; exit 5; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 6; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --out gpurun_out/traffic.json || exit 7
cd /tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$R/gpurun_out/pmc_gen" -o pmc -- python3 "$R/tools/perf_extra.py" gen > "$R/gpurun_out/pmc_gen.log" 2>&1 || { echo "pmc gen failed"; tail -20 "$R/gpurun_out/pmc_gen.log"; exit 8; }
echo done

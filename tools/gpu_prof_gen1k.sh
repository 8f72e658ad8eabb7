#!/bin/bash
# Evidence for the d=1024 generator (full rounds) and the on-device g(T) max: rocprofv3
# kernel-trace stats of one d=1024 resident batch and of the T=100 sweep point, and the
# generator's HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_1k" "$R/gpurun_out/prof_t100" "$R/gpurun_out/pmc1k_FETCH_SIZE" "$R/gpurun_out/pmc1k_WRITE_SIZE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_1k" -o r02 --output-format csv -- python3 "$R/tools/batch_probe.py" 3400x10000x1024x128 > "$R/gpurun_out/prof_1k.log" 2>&1 || { echo "rocprof 1k failed"; tail -20 "$R/gpurun_out/prof_1k.log"; exit 2; }
grep '^{' "$R/gpurun_out/prof_1k.log" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_t100" -o r02 --output-format csv -- python3 "$R/tools/perf_extra.py" --Ts 100 sweep > "$R/gpurun_out/prof_t100.log" 2>&1 || { echo "rocprof t100 failed"; tail -20 "$R/gpurun_out/prof_t100.log"; exit 3; }
grep '^{' "$R/gpurun_out/prof_t100.log" | cut -c1-300
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc1k_$C" -o pmc -- python3 "$R/tools/batch_probe.py" 3400x10000x1024x128 > "$R/gpurun_out/pmc1k_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc1k_$C.log"; exit 4; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc1k_FETCH_SIZE --write gpurun_out/pmc1k_WRITE_SIZE --kernel ocx_gen_wave_kernel --B 3400 --T 10000 --d 1024 --P 32 --out gpurun_out/traffic_gen1k.json; head -20 gpurun_out/traffic_gen1k.json
head -12 gpurun_out/prof_1k/r02_kernel_stats.csv | cut -c1-200
head -8 gpurun_out/prof_t100/r02_kernel_stats.csv | cut -c1-200

#!/bin/bash
# Round-3 evidence, second half (the first ran the suite, smoke, bench and the bench's
# rocprofv3 stats): rocprofv3 kernel stats of the few-wave T=1e5 batches; the PMC HBM passes
# over the bench command with one end-to-end batch; the generator scalar-jump A/B; the g(T)
# sweep and configs[4]; the general exact solver's timings.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/gpurun_out/prof_fw" "$R/gpurun_out/pmc_FETCH_SIZE" "$R/gpurun_out/pmc_WRITE_SIZE"
OCX_PROBE_SHORT=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fw" -o fw --output-format csv -- python3 "$R/tools/r03_alg_probe.py" > "$R/gpurun_out/prof_fw.log" 2>&1 || { echo "rocprof fw failed"; tail -20 "$R/gpurun_out/prof_fw.log"; exit 6; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 --two-pass-steps 0 --e2e-steps 1 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$R/gpurun_out/pmc_$C.log"; exit 7; }
done
cd "$R" && python tools/pmc_traffic.py --fetch gpurun_out/pmc_FETCH_SIZE --write gpurun_out/pmc_WRITE_SIZE --B 32768 --T 10000 --d 64 --P 4 --passes 1 --out gpurun_out/traffic.json > /dev/null && head -c 1500 gpurun_out/traffic.json; echo
grep -v "^W20\|^I20" gpurun_out/prof_fw.log | cut -c1-200 | head -12
head -8 gpurun_out/prof_fw/fw_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python -u tools/r03_gen_scalar_ab.py > gpurun_out/r03_gen_scalar_ab.jsonl 2> gpurun_out/r03_gen_scalar_ab.err || { echo "gen A/B failed"; tail -20 gpurun_out/r03_gen_scalar_ab.err; exit 10; }
cat gpurun_out/r03_gen_scalar_ab.jsonl
timeout -k 10 300 python -u tools/r03_exact_probe.py > gpurun_out/r03_exact_probe.jsonl 2> gpurun_out/r03_exact_probe.err || { echo "exact probe failed"; tail -20 gpurun_out/r03_exact_probe.err; exit 9; }
cut -c1-250 gpurun_out/r03_exact_probe.jsonl
timeout -k 10 900 python tools/perf_extra.py sweep config4 > gpurun_out/sweep_r03.log 2>&1 || { tail -20 gpurun_out/sweep_r03.log; exit 8; }
grep '^{' gpurun_out/sweep_r03.log | cut -c1-220

#!/bin/bash
# Round-2 evidence: rocprofv3 kernel stats + HBM PMC (separate FETCH_SIZE / WRITE_SIZE passes)
# for the default (OCX_LANES_BEST) FTRL kernel on the few-wave d=64 T=1e5 batch and on
# configs[4]'s d=1024 batch, and kernel stats for SMART and the fused exact kernel.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/prof_r02"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # name, then the program and its arguments
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n" -o "$n" -- "$@" > "$O/$n.log" 2>&1 || { echo "$n failed"; tail -20 "$O/$n.log"; exit 2; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/${n}_$C" -o pmc -- "$@" > "$O/${n}_$C.log" 2>&1 || { echo "$n $C failed"; tail -20 "$O/${n}_$C.log"; exit 3; }
  done
  grep '^{' "$O/$n.log" | cut -c1-220
}
run fewwave python3 "$R/tools/tune.py" --B 4900 --T 100000 --d 64 --lanes 128 --probe 0 --rounds 1
run d1024 python3 "$R/tools/tune.py" --B 2048 --T 10000 --d 1024 --lanes 128 --probe 0 --rounds 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/smart_exact" -o se -- python3 "$R/tools/perf_extra.py" smart config3 > "$O/smart_exact.log" 2>&1 || { echo "smart/exact failed"; tail -20 "$O/smart_exact.log"; exit 4; }
grep '^{' "$O/smart_exact.log" | cut -c1-220
cd "$R"
for n in fewwave d1024; do
  python tools/pmc_traffic.py --fetch "$O/${n}_FETCH_SIZE" --write "$O/${n}_WRITE_SIZE" --kernel ocx_alg_kernel --B $([ $n = fewwave ] && echo "4900 --T 100000 --d 64 --P 16" || echo "2048 --T 10000 --d 1024 --P 64") --out "$O/traffic_$n.json" | cut -c1-300
done
find "$O" -name "*kernel_stats.csv" | head

#!/bin/bash
# Round 3: generator A/B — the libraries in tune_r03/ named by $1 (comma-separated, the
# first the reference) run the generator parity tests' shapes for bit identity, then timings
# twice (forward and reversed order), on one box.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
LIBS="$1"; OUT="gpurun_out/$2"
REV=$(echo "$LIBS" | tr ',' '\n' | tac | paste -sd,)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "generator" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "gen pytest failed"; tail -40 gpurun_out/pytest_gen.log; exit 2; }
tail -1 gpurun_out/pytest_gen.log
timeout -k 10 400 python -u tools/r03_gen_lib_ab.py "$LIBS" > "$OUT" 2> "$OUT.err" || { echo "ab failed"; tail -20 "$OUT.err"; exit 3; }
timeout -k 10 400 python -u tools/r03_gen_lib_ab.py "$REV" >> "$OUT" 2>> "$OUT.err" || { echo "ab2 failed"; tail -20 "$OUT.err"; exit 4; }
grep -v '"what"' "$OUT" | sort | uniq -c
grep ms_min "$OUT" | cut -c1-120

#!/bin/bash
# Register-ring depth of the C <= 8 FTRL kernel on the few-wave T=1e5 batch (one pass).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/bp_nb.jsonl
C=4900x100000x64x128,3328x100000x64x8
timeout -k 10 300 python tools/batch_probe.py $C | sed 's/^{/{"lib": "nb8", /' >> gpurun_out/bp_nb.jsonl || exit 3
for V in nb6 nb12 nb16; do
  OCX_LIB=$R/tune_ship/libocx_$V.so timeout -k 10 300 python tools/batch_probe.py $C | sed "s/^{/{\"lib\": \"$V\", /" >> gpurun_out/bp_nb.jsonl || exit 4
done
python -c "
import json
for l in open('gpurun_out/bp_nb.jsonl'):
    d=json.loads(l); print(d['lib'], d['B'], d['P'], d['C'], round(d['sim_closed_ms'],1), round(d['sim_two_pass_ms'],1))"

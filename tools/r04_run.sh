#!/bin/bash
# Round 4 GPU session: the -m gpu suite, then the probes.  A test failure (pytest exit 1)
# does not stop the probes; any other non-zero exit (a crash, an abort, a time limit) ends
# the script there.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04_gputest_${1:-b}.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
shift || true
for probe in "$@"; do
  timeout -k 10 300 python -u tools/$probe.py > $O/$probe.jsonl 2> $O/$probe.err || { rc=$?; echo "$probe rc=$rc"; exit $rc; }
done

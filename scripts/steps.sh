#!/bin/bash
# Generic GPU experiment runner: each argument is one command, run from the
# repo root under its own time limit (STEP_TIMEOUT, default 300 s); stdout is
# appended to gpurun_out/TAG/out.jsonl, stderr to gpurun_out/TAG/err.log.
# Stops at the first failing step (pool rule: nothing more on the GPU after
# a fault, abort or time-out). The commands behind every A/B file under
# profiles/r06/ab/ are listed in profiles/r06/ab/README.md.
# Usage: scripts/steps.sh TAG 'cmd 1' 'cmd 2' ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for c in "$@"; do
  echo "== $c" >> $O/err.log
  timeout -k 10 ${STEP_TIMEOUT:-300} bash -c "$c" >> $O/out.jsonl 2>>$O/err.log
  rc=$?
  tail -1 $O/out.jsonl
  if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $c"; tail -5 $O/err.log; exit $rc; fi
done

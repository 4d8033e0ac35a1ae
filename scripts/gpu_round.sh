#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults/aborts/times out (exit >= 2 other than
# a plain pytest failure), per the pool rules. Usage: scripts/gpu_round.sh TAG
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }

step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
fatal $rc && exit $rc
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider; rc=$?
fatal $rc && exit $rc
step bench 600 python bench.py --steps 100 --warmup 10; rc=$?
fatal $rc && exit $rc
cd /tmp
step_prof() {
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --sweep "" --no-cpu \
    > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
}
step_prof; rc=$?
echo "== prof rc=$rc" | tee -a $GRAFT_REPO_ROOT/$OUT/steps.log
exit $rc

#!/bin/bash
# One GPU session: smoke -> GPU tests (junit xml) -> bench.
# Stops at the first step that faults/aborts/times out (exit >= 2 other than
# a plain pytest failure), per the pool rules. Usage: scripts/gpu_check.sh TAG
set -u
TAG=${1:-r02}
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread --junitxml=$OUT/junit.xml; rc=$?
fatal $rc && exit $rc
step bench 300 python bench.py; rc=$?
exit $rc

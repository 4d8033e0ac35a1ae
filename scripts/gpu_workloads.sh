#!/bin/bash
# BASELINE configs 3-5 on one GPU: their parity tests, one bench line each,
# and a rocprofv3 kernel-trace summary per workload. Usage: gpu_workloads.sh TAG
set -u
TAG=${1:-r01w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { local name=$1 to=$2; shift 2; echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log; tail -3 $OUT/$name.log; return $rc; }
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
step pytest_cfg 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "config3 or config4 or config5"; rc=$?; fatal $rc && exit $rc
for w in sdd_dds moe panel; do
  step bench_$w 300 python bench.py --workload $w --steps 50 --warmup 20; rc=$?; fatal $rc && exit $rc
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/prof_$w -o run -- \
      python3 $R/bench.py --workload $w --steps 50 --warmup 20 > $R/$OUT/prof_$w.log 2>&1 ); rc=$?
  echo "== prof_$w rc=$rc" | tee -a $OUT/steps.log; fatal $rc && exit $rc
done
exit 0

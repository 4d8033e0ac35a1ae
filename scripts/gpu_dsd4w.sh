#!/bin/bash
# 4-wave DSD kernel session: experiment ablations, bit-identity tests, A/B.
# Stops at the first step that faults / aborts / times out.
set -u
TAG=${1:-dsd4w}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
echo "== k4w ablations"
timeout -k 10 180 python microbench/k4w/run_k4w.py --uniform --variants 0,3 --rounds 5 > $OUT/k4w_u50.log 2>&1; rc=$?
tail -2 $OUT/k4w_u50.log; fatal $rc && exit $rc
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsd4w.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; fatal $rc && exit $rc
echo "== ab"
timeout -k 10 300 python scripts/ab_dsd4w.py > $OUT/ab.log 2>&1; rc=$?
cat $OUT/ab.log | grep density; exit $rc

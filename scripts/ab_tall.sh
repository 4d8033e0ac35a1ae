#!/bin/bash
# Tall-path parity tests, then interleaved A/B of build/exp variants on config 5.
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/abt; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -m gpu -k "tall or panel or persist" tests \
  > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/exp_bench.py --m 131072 --density 0.02 "$@" > $OUT/ab.log 2>&1; rc=$?
tail -1 $OUT/ab.log; exit $rc

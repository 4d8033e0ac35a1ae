#!/bin/bash
# Full GPU suite on the in-tree library, then interleaved A/B of two
# build/exp variants on config 5 and DSD 4096 at 10% / 50%.
set -u
A=$1; B=$2
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/abg; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
E="timeout -k 10 300 python scripts/exp_bench.py"
$E --m 131072 --density 0.02 $A $B > $OUT/c5.log 2>&1 && tail -1 $OUT/c5.log &&
$E --density 0.1 $A $B > $OUT/d10.log 2>&1 && tail -1 $OUT/d10.log &&
$E --density 0.5 $A $B > $OUT/d50.log 2>&1 && tail -1 $OUT/d50.log

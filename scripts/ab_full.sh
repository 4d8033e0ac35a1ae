#!/bin/bash
# Full GPU suite on the in-tree library, then interleaved A/B of build/exp
# variants on DSD 4096^3 at four densities and the MoE workload.
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/abf; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_dens.sh "$@" || exit $?
timeout -k 10 300 python scripts/exp_bench.py --op moe "$@" > $OUT/moe.log 2>&1 || exit $?
tail -1 $OUT/moe.log

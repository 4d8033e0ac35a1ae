#!/bin/bash
# One iteration: GPU parity tests, then interleaved A/B of build/exp/*.so.
# Usage: gpu_iter.sh TAG [densities]
set -u
TAG=$1; DENS=${2:-"0.5 0.1 0.9"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/exp_run.sh $TAG "$DENS" || exit $?

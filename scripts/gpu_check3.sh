#!/bin/bash
# GPU tests + captured-graph throughput (headline and config 3).
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread --junitxml=$OUT/junit.xml > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for g in "" "--graph"; do
  timeout -k 10 300 python bench.py --sweep "" --no-cpu $g > $OUT/dsd$g.json 2> $OUT/dsd$g.err; rc=$?
  echo "dsd $g rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/dsd$g.err; exit $rc; }
  timeout -k 10 300 python bench.py --workload sdd_dds $g > $OUT/pair$g.json 2> $OUT/pair$g.err; rc=$?
  echo "pair $g rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/pair$g.err; exit $rc; }
done
grep -h -o '"value": [0-9.]*, "unit": "TFLOP/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $OUT/dsd*.json $OUT/pair*.json
exit 0

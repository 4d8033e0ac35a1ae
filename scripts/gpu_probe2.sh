#!/bin/bash
# L2 -> CU throughput by load form (microbench/l2_to_cu) and captured-graph
# throughput of the headline and config 3. Usage: scripts/gpu_probe2.sh TAG
set -u
TAG=$1; R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for mb in 2 16 64; do
  timeout -k 10 60 ./microbench/l2_to_cu $mb >> $OUT/l2_to_cu.jsonl 2>&1; rc=$?
  echo "l2_to_cu $mb rc=$rc"; fatal $rc && exit $rc
done
cat $OUT/l2_to_cu.jsonl
for g in "" "--graph"; do
  timeout -k 10 300 python bench.py --sweep "" --no-cpu $g > $OUT/dsd$g.json 2> $OUT/dsd$g.err
  rc=$?; echo "dsd $g rc=$rc"; fatal $rc && exit $rc
  timeout -k 10 300 python bench.py --workload sdd_dds $g > $OUT/pair$g.json 2> $OUT/pair$g.err
  rc=$?; echo "pair $g rc=$rc"; fatal $rc && exit $rc
done
grep -h -o '"value": [0-9.]*, "unit": "TFLOP/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $OUT/dsd*.json $OUT/pair*.json
exit 0

#!/bin/bash
# Runs exp_bench.py over build/exp/*.so at a few densities. Usage: exp_run.sh TAG [densities]
TAG=$1; DENS=${2:-"0.5 0.1 0.9"}; OPS=${3:-""}
mkdir -p gpurun_out/$TAG
for d in $DENS; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d build/exp/*.so >> gpurun_out/$TAG/exp.jsonl 2> gpurun_out/$TAG/exp_$d.err
  rc=$?; echo "density $d rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/exp_$d.err; exit $rc; }
done
for op in $OPS; do
  timeout -k 10 300 python scripts/exp_bench.py --op $op --density 0.2 build/exp/*.so >> gpurun_out/$TAG/exp.jsonl 2> gpurun_out/$TAG/exp_$op.err
  rc=$?; echo "op $op rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/exp_$op.err; exit $rc; }
done
cat gpurun_out/$TAG/exp.jsonl

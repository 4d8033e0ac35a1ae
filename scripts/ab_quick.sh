#!/bin/bash
# Interleaved A/B of build/exp/*.so: DSD 4096^3 at the given densities, then
# optional extra exp_bench.py argument sets (each a quoted string).
# Usage: scripts/ab_quick.sh TAG "densities" ["--m 1024" ...]
set -u
TAG=$1; DENS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for d in $DENS; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d build/exp/*.so >> $OUT/exp.jsonl 2> $OUT/exp_d$d.err
  rc=$?; echo "density $d rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/exp_d$d.err; exit $rc; }
done
i=0
for extra in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python scripts/exp_bench.py $extra build/exp/*.so >> $OUT/exp.jsonl 2> $OUT/exp_x$i.err
  rc=$?; echo "extra '$extra' rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/exp_x$i.err; exit $rc; }
done
cat $OUT/exp.jsonl

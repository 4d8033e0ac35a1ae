#!/bin/bash
# GPU tests, then interleaved A/B of build/exp/*.so on the headline shape
# (densities) and on the strong-scaling row panels (M = 512 / 1024 / 2048).
# Usage: scripts/ab_split.sh TAG [tests=1]
set -u
TAG=$1; TESTS=${2:-1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$TESTS" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for d in 0.5 0.1 0.9; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d build/exp/*.so >> $OUT/exp.jsonl 2> $OUT/exp_d$d.err
  rc=$?; echo "density $d rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/exp_d$d.err; exit $rc; }
done
for m in 512 1024 2048; do
  timeout -k 10 300 python scripts/exp_bench.py --m $m --density 0.5 build/exp/*.so >> $OUT/exp.jsonl 2> $OUT/exp_m$m.err
  rc=$?; echo "m $m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/exp_m$m.err; exit $rc; }
done
cat $OUT/exp.jsonl
SPUTNIK_AMD_LIB=build/seg/seg.so timeout -k 10 300 python scripts/exp_segments.py dsd50 dsd10 dsd90 > $OUT/segments.jsonl 2> $OUT/segments.err
rc=$?; echo "segments rc=$rc"; cat $OUT/segments.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/segments.err; exit $rc; }
exit 0

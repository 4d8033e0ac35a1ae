#!/bin/bash
# A/B session: the GPU suite on the working library, then interleaved
# same-process timing of build/exp/*.so (scripts/exp_run.sh) at the
# headline densities, config 3's pair, and the timeline build.
TAG=$1; TESTS=${2:-1}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "$TESTS" = "1" ]; then
  echo "== pytest" | tee -a $OUT/steps.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread --junitxml=$OUT/junit.xml > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest rc=$rc" | tee -a $OUT/steps.log; tail -2 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
echo "== ab" | tee -a $OUT/steps.log
bash scripts/exp_run.sh $TAG "0.5 0.1 0.3 0.9" "pair" > $OUT/ab.log 2>&1; rc=$?
echo "== ab rc=$rc" | tee -a $OUT/steps.log
[ $rc -ne 0 ] && exit $rc
# split mode (the N = 2 strong-scaling panel, M = 2048)
for d in 0.5 0.1; do
  timeout -k 10 300 python scripts/exp_bench.py --m 2048 --density $d build/exp/*.so \
    >> $OUT/exp.jsonl 2> $OUT/exp_m2048.err; rc=$?
  [ $rc -ne 0 ] && exit $rc
done
if [ -f $R/build/tlx/tl4.so ]; then
  echo "== timeline" | tee -a $OUT/steps.log
  SPUTNIK_AMD_LIB=$R/build/tlx/tl4.so timeout -k 10 300 python scripts/exp_timeline4w.py \
    0.5 0.1 0.3 0.9 > $OUT/tl4.log 2>&1; rc=$?
  echo "== timeline rc=$rc" | tee -a $OUT/steps.log
fi
exit $rc

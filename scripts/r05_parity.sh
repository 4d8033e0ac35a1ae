#!/bin/bash
# Round-5 parity session: the regular session (smoke, full GPU suite incl.
# the topology fuzz and the full-output config tests, the driver's bench
# command and its trace), then the new parity tests against
# build/bug/preload_bug.so (scripts/build_preload_bug.sh: the f327921
# index-preload bug on today's sources), which must FAIL.
TAG=$1
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_session.sh $TAG 1 - -; rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
OUT=$R/gpurun_out/$TAG
cd $R
echo "== bug_lib" | tee -a $OUT/steps.log
SPUTNIK_AMD_LIB=$R/build/bug/preload_bug.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_dsd4w.py::test_dsd4w_index_preload_odd_count_last_entry \
  tests/test_gpu_fuzz.py -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "dsd or dds" --junitxml=$OUT/junit_bug.xml > $OUT/bug_lib.log 2>&1; rc2=$?
echo "== bug_lib rc=$rc2 (1 = tests failed, as they must)" | tee -a $OUT/steps.log
tail -5 $OUT/bug_lib.log
[ $rc2 -ne 1 ] && exit 3
# per-workgroup timeline of the shipped DSD NN variants (SPUTNIK_EXP & 512
# build of the same sources, scripts/exp_timeline4w.py)
if [ -f $R/build/tlx/tl4.so ]; then
  echo "== timeline" | tee -a $OUT/steps.log
  SPUTNIK_AMD_LIB=$R/build/tlx/tl4.so timeout -k 10 300 python scripts/exp_timeline4w.py \
    0.5 0.1 0.3 0.9 > $OUT/tl4.log 2>&1; rc3=$?
  echo "== timeline rc=$rc3" | tee -a $OUT/steps.log
  [ $rc3 -ne 0 ] && exit $rc3
fi
echo "== ab" | tee -a $OUT/steps.log
timeout -k 10 400 python scripts/ab_dsd4w.py --densities 0.5,0.1,0.3,0.9 --rounds 7 \
  > $OUT/ab.jsonl 2> $OUT/ab.err; rc4=$?
echo "== ab rc=$rc4" | tee -a $OUT/steps.log
[ $rc4 -ne 0 ] && exit $rc4
exit $rc

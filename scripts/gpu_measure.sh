#!/bin/bash
# Measurement session: smoke -> GPU tests (junit) -> bench (headline +
# density sweep, CPU baseline, config-1 line) -> rocprofv3 kernel-trace
# summary of the headline -> the other workloads (configs 3-5, the backward
# variants with MatmulEx and with Matmul, the device Transpose).
# Stops at the first step that faults/aborts/times out (exit >= 2 other than
# a plain pytest failure), per the pool rules. Usage: gpu_measure.sh TAG [skip_tests]
set -u
TAG=${1:-r02}; SKIP_TESTS=${2:-0}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
cd $R
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
fatal $rc && exit $rc
if [ "$SKIP_TESTS" = "0" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread --junitxml=$OUT/junit.xml; rc=$?
  fatal $rc && exit $rc
fi
step bench 300 python bench.py; rc=$?
fatal $rc && exit $rc
cd /tmp
echo "== prof" | tee -a $OUT/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --sweep "" --no-cpu > $OUT/prof.log 2>&1; rc=$?
echo "== prof rc=$rc" | tee -a $OUT/steps.log; tail -2 $OUT/prof.log
fatal $rc && exit $rc
for w in sdd_dds panel; do
  echo "== prof_$w" | tee -a $OUT/steps.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$w -o run -- \
    python3 $R/bench.py --workload $w > $OUT/prof_$w.log 2>&1; rc=$?
  echo "== prof_$w rc=$rc" | tee -a $OUT/steps.log
  fatal $rc && exit $rc
done
cd $R
for w in sdd_dds moe panel transpose; do
  step w_$w 300 python bench.py --workload $w; rc=$?; fatal $rc && exit $rc
done
for v in "dsd TN ex" "dsd TN matmul" "dsd TT ex" "dsd TT matmul" "dsd NT ex" \
         "dds NN ex" "dds NN matmul" "dds TN ex" "dds TN matmul" "dds NT ex" \
         "sdd NN ex"; do
  set -- $v
  step op_$1_$2_$3 300 python bench.py --workload op --op $1 --trans $2 --api $3
  rc=$?; fatal $rc && exit $rc
done
exit 0

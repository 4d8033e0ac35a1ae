#!/bin/bash
# One measurement session on the GPU box, each GPU step under its own time
# limit; stops at the first step that faults / aborts / times out (exit >= 2
# other than a plain pytest failure), per the pool rules.
#   smoke -> pytest -m gpu (junit) -> the driver's bench command
#   (--steps 20 --warmup 5) -> rocprofv3 kernel trace of that same command
#   (timed dispatches extracted by scripts/trace_headline.py) -> PMC passes
#   (scripts/pmc.sh; config 3 and 5 by scripts/pmc_workload.sh) -> optional interleaved A/B of build/exp/*.so.
# Usage: scripts/gpu_session.sh TAG [tests=1] [pmc densities or -] [ab densities or -]
set -u
TAG=$1; TESTS=${2:-1}; PMC=${3:-"0.5 0.1 0.3 0.9"}; AB=${4:--}
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
if [ "$TESTS" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread --junitxml=$OUT/junit.xml; rc=$?
  fatal $rc && exit $rc
fi
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5; rc=$?
fatal $rc && exit $rc
cd /tmp
echo "== prof_driver" | tee -a $OUT/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_driver -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1; rc=$?
echo "== prof_driver rc=$rc" | tee -a $OUT/steps.log
fatal $rc && exit $rc
cd $R
python3 scripts/trace_headline.py $OUT/prof_driver $OUT/prof_driver.log 5 20 \
  $OUT/headline_trace.json
if [ "$PMC" != "-" ]; then
  bash scripts/pmc.sh $TAG "$PMC"; rc=$?
  fatal $rc && exit $rc
  bash scripts/pmc_workload.sh $TAG sdd_dds "--workload sdd_dds"; rc=$?
  fatal $rc && exit $rc
  bash scripts/pmc_workload.sh $TAG panel "--workload panel"; rc=$?
  fatal $rc && exit $rc
  bash scripts/pmc_workload.sh $TAG moe "--workload moe"; rc=$?
  fatal $rc && exit $rc
  python3 scripts/pmc_merge_workloads.py $OUT $OUT/pmc_workloads.json
fi
if [ "$AB" != "-" ]; then
  bash scripts/exp_run.sh $TAG "$AB"; rc=$?
  fatal $rc && exit $rc
fi
exit 0

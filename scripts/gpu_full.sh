#!/bin/bash
# Full measurement session: smoke, GPU tests, PMC traffic, bench (reads the
# traffic), rocprofv3 kernel-trace summary. Usage: gpu_full.sh TAG
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log; tail -3 $OUT/$name.log; return $rc; }
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; fatal $rc && exit $rc
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?; fatal $rc && exit $rc
R=$GRAFT_REPO_ROOT
( cd /tmp && for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((${i:-0}+1)); timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $R/$OUT/pmc/p$i -o pass -- \
      python3 $R/bench.py --steps 20 --warmup 3 --sweep "" --no-cpu > $R/$OUT/pmc_p$i.log 2>&1 || exit $?
  done ); rc=$?; echo "== pmc rc=$rc" | tee -a $OUT/steps.log; fatal $rc && exit $rc
python scripts/pmc_traffic.py $OUT/pmc dsd_4096x4096x4096_0.5_f16 $OUT/pmc_latest.json
step bench 600 python bench.py --pmc $OUT/pmc_latest.json; rc=$?; fatal $rc && exit $rc
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/prof -o run -- \
    python3 $R/bench.py --sweep "" --no-cpu --pmc $R/$OUT/pmc_latest.json > $R/$OUT/prof.log 2>&1 ); rc=$?
echo "== prof rc=$rc" | tee -a $OUT/steps.log; fatal $rc && exit $rc
for w in sdd_dds moe panel; do
  step bench_$w 300 python bench.py --workload $w; rc=$?; fatal $rc && exit $rc
done
exit 0

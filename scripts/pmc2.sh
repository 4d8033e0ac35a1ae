#!/bin/bash
# Counter listing + load-path counters for one bench config. Usage: pmc2.sh TAG
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --sweep "" --no-cpu \
    > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && tail -3 $OUT/p$i.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0

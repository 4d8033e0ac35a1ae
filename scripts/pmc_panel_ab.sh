#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of config 5 under an env knob (0 and 1).
set -u
V=${1:-SPUTNIK_AMD_TALL_XCD}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmcab; mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
for v in 0 1; do
  export $V=$v
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/v$v -o pass -- \
    python3 $R/bench.py --workload panel --steps 20 --warmup 5 > $OUT/v$v.log 2>&1
  rc=$?; echo "$V=$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/v$v.log; exit $rc; }
done
exit 0

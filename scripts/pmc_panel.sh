#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over config 5.
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmcp; mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $R/bench.py --workload panel --steps 20 --warmup 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
exit 0

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over
# one bench.py workload, then a per-kernel summary (scripts/pmc_kernels.py).
# Usage: scripts/pmc_workload.sh TAG NAME "bench.py args"
#   (PMC_GROUPS="g1;g2" replaces the default counter groups)
#   e.g. scripts/pmc_workload.sh r03m sdd_dds "--workload sdd_dds"
set -u
TAG=$1; NAME=$2; ARGS=$3
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG/pmc_$NAME; mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
i=0
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $R/bench.py $ARGS --steps 20 --warmup 5 --no-cpu > $OUT/p$i.log 2>&1
  rc=$?; echo "$NAME pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 $R/scripts/pmc_kernels.py $OUT $R/gpurun_out/$TAG/pmc_$NAME.json "$ARGS"

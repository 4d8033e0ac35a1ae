#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over
# any python script, then the per-kernel summary (scripts/pmc_kernels.py).
# Usage: scripts/pmc_cmd.sh TAG NAME script.py [args...]
#   (PMC_GROUPS="g1;g2" replaces the default counter groups)
set -u
TAG=$1; NAME=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG/pmc_$NAME; mkdir -p $OUT
SCRIPT=$R/$1; shift
cd /tmp; export TMPDIR=/tmp
i=0
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "$NAME pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 $R/scripts/pmc_kernels.py $OUT $R/gpurun_out/$TAG/pmc_$NAME.json "$NAME"

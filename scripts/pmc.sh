#!/bin/bash
# PMC passes over the bench's DSD kernel at each density (one counter group
# per rocprofv3 run, --kernel-trace only: no sys/runtime tracing next to
# --pmc on this pool), then the per-density summary with the library's build
# hash (scripts/pmc_summary.py -> gpurun_out/TAG/pmc_latest.json).
# Usage: scripts/pmc.sh TAG [densities]
set -u
TAG=$1; DENS=${2:-"0.5 0.1 0.3 0.9"}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG/pmc
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for d in $DENS; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv \
      -d $OUT/d$d/p$i -o pass -- \
      python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --no-cpu \
      --density $d > $OUT/d$d.p$i.log 2>&1
    rc=$?
    echo "density $d pass $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/d$d.p$i.log; exit $rc; fi
  done
done
python3 $R/scripts/pmc_summary.py $OUT $R/gpurun_out/$TAG/pmc_latest.json

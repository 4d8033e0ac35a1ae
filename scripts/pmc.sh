#!/bin/bash
# PMC passes over the bench kernel (one counter group per rocprofv3 run,
# --kernel-trace only: no sys/runtime tracing next to --pmc on this pool).
# Usage: scripts/pmc.sh TAG [bench args...]
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/pmc
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_F16 SQ_WAIT_INST_LDS" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "TCC_HIT_sum TCC_MISS_sum" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --sweep "" --no-cpu "$@" \
    > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0

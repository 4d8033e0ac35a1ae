#!/bin/bash
# Lists the PMC counters of the box and collects LDS / MFMA / wait counters
# for the current library on DSD 4096^3 50%. Usage: pmc_probe.sh TAG [lib]
TAG=$1; LIB=${2:-sputnik_amd/libsputnik.so}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1; rc=$?
[ $rc -ge 124 ] && exit $rc
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA" \
           "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pass -- \
    python3 $GRAFT_REPO_ROOT/scripts/exp_bench.py --rounds 2 --iters 20 $GRAFT_REPO_ROOT/$LIB > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

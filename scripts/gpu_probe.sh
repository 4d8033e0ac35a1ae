#!/bin/bash
# Counter list, captured-graph throughput, stall-breakdown PMC passes of the
# headline and the reference's benchmark sweep (bench.py --workload sweep).
# Usage: scripts/gpu_probe.sh TAG [sweep=1]
set -u
TAG=$1; SWEEP=${2:-1}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $R
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
for g in "" "--graph"; do
  timeout -k 10 300 python bench.py --sweep "" --no-cpu $g > $OUT/dsd$g.json 2> $OUT/dsd$g.err
  rc=$?; echo "dsd $g rc=$rc"; fatal $rc && exit $rc
  timeout -k 10 300 python bench.py --workload sdd_dds $g > $OUT/pair$g.json 2> $OUT/pair$g.err
  rc=$?; echo "pair $g rc=$rc"; fatal $rc && exit $rc
done
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "TA_TA_BUSY_sum TA_BUSY_avr" "TD_TD_BUSY_sum TD_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/stall/p$i -o pass -- \
    python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --no-cpu > $OUT/stall_p$i.log 2>&1
  echo "stall pass $i rc=$?"
done
cd $R
if [ "$SWEEP" = "1" ]; then
  timeout -k 10 900 python bench.py --workload sweep --steps 20 --warmup 10 > $OUT/sweep.jsonl 2> $OUT/sweep.err
  rc=$?; echo "sweep rc=$rc"; wc -l $OUT/sweep.jsonl
fi
exit 0

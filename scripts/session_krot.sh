#!/bin/bash
# SDD k-rotation experiment (knob sdd_krot): numerics at 4096 / 8192, then
# same-process A/B of the modes at 16384^3 and 8192^3.
# Usage: scripts/session_krot.sh TAG
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
D="timeout -k 10 120 python -u scripts/diag_krot.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kat.py -k "krot" > $O/kat0.log 2>&1 || { tail -30 $O/kat0.log; exit 1; }
for t in NT NN TT TN; do
  $D $t 8192 0.5 >> $O/krot_numerics.jsonl 2>>$O/err.log || exit $?
done
$D NT 16384 0.1 >> $O/krot_numerics.jsonl 2>>$O/err.log || exit $?
cat $O/krot_numerics.jsonl
K="timeout -k 10 300 python -u scripts/exp_knob_ab.py sdd_krot 0,1,2,3,4"
for w in op:sdd:NT:16384 op:sdd:NN:16384 op:sdd:TT:16384 op:sdd:NT:8192; do
  $K --workload $w --density 0.5 --rounds 5 --iters 10 >> $O/krot_ab.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/krot_ab.jsonl
done
$K --workload op:sdd:NT:16384 --density 1.0 --rounds 5 --iters 6 >> $O/krot_ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/krot_ab.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kat.py -k "krot or sdd" > $O/kat.log 2>&1 || { tail -30 $O/kat.log; exit 1; }
tail -3 $O/kat.log

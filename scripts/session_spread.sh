#!/bin/bash
# SDD group spread (knob sdd_spread) on rows of equal count: KATs, then
# same-process A/B on config 4's SDD and dense 8192 / 16384 SDD.
# Usage: scripts/session_spread.sh TAG
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kat.py -k "spread or krot" > $O/kat0.log 2>&1 || { tail -30 $O/kat0.log; exit 1; }
tail -1 $O/kat0.log
K="timeout -k 10 300 python -u scripts/exp_knob_ab.py sdd_spread 0,1"
$K --workload moe_sdd --rounds 7 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/ab.jsonl
for w in op:sdd:NN:16384 op:sdd:NT:16384 op:sdd:TT:16384 op:sdd:TN:16384 op:sdd:NN:8192 op:sdd:NT:8192; do
  $K --workload $w --density 1.0 --rounds 5 --iters 8 >> $O/ab.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/ab.jsonl
done
$K --workload moe --rounds 7 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/ab.jsonl

#!/bin/bash
# sdd_spread on NT over rows of equal count: config 4 in MegaBlocks' own w1
# layout and dense NT / NN at 4096-16384.
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
K="timeout -k 10 300 python -u scripts/exp_knob_ab.py sdd_spread 0,1"
$K --workload moe_sdd_nt --rounds 7 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/ab.jsonl
for w in op:sdd:NT:4096 op:sdd:NT:12288 op:sdd:NT:16384 op:sdd:NN:12288 op:sdd:TT:12288; do
  $K --workload $w --density 1.0 --rounds 5 --iters 8 >> $O/ab.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/ab.jsonl
done

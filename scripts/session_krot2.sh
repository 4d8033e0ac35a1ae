#!/bin/bash
# SDD k-rotation (knob sdd_krot) A/B, modes 0 / 2 / 4, over NT densities
# and strides, TT / TN at 16384.  Usage: scripts/session_krot2.sh TAG
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
K="timeout -k 10 300 python -u scripts/exp_knob_ab.py sdd_krot 0,2,4"
for wd in op:sdd:NT:16384@0.1 op:sdd:NT:16384@0.3 op:sdd:NT:16384@0.7 op:sdd:NT:12288@0.5 \
          op:sdd:NT:12288@1.0 op:sdd:TT:16384@1.0 op:sdd:NN:16384@1.0 op:sdd:TN:16384@0.5 \
          op:sdd:NT:8192@1.0 op:sdd:NT:16384@0.5; do
  w=${wd%@*}; d=${wd#*@}
  $K --workload $w --density $d --rounds 5 --iters 8 >> $O/krot_ab.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/krot_ab.jsonl
done

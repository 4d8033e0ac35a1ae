#!/bin/bash
# A/B of the smallest pair hand-off (knob min_handoff) on DSD 4096^3 at
# each density and on config 3's DDS, same process, interleaved.
# Usage: scripts/ab_pairs.sh TAG
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py min_handoff 2,1,3"
for d in 0.5 0.1 0.3 0.9; do
  $K --workload dsd --density $d --rounds 9 --iters 30 >> $O/ab_pairs.jsonl 2>>$O/ab_err.log || exit $?
done
$K --workload dds --density 0.2 --rounds 9 --iters 30 >> $O/ab_pairs.jsonl 2>>$O/ab_err.log || exit $?
cat $O/ab_pairs.jsonl

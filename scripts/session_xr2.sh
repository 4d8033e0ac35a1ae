#!/bin/bash
# xcd_rows A/B on the uniform-row sweep points (dense DSD / DDS, 8192^3 and
# 16384^3) where the XCD-row map also applies.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-xr2}; mkdir -p $O
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py xcd_rows 1,0 --density 1.0"
for w in op:dsd:NN:8192 op:dds:NN:8192 op:dsd:NT:8192 op:dsd:NN:16384 op:dds:NN:16384; do
  $K --workload $w --rounds 5 --iters 5 >> $O/ab.jsonl 2>>$O/err.log || exit $?
done
cat $O/ab.jsonl

#!/bin/bash
# What 32-KiB row strides cost SDD 16384^3 (scripts/exp_sdd_stride16k.py).
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for d in 1.0 0.5; do
  timeout -k 10 300 python -u scripts/exp_sdd_stride16k.py --density $d >> $O/stride16k.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/stride16k.jsonl
done

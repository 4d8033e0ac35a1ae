#!/bin/bash
# A/B of the XCD-row tile map (knob xcd_rows) on config 4's DSD h . w2 and
# the whole MoE step, plus its KAT.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-xr}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kat.py -q -p no:cacheprovider \
  -k "uniform_rows or 4096_pairs or kernel_queries" --timeout 120 --timeout-method thread > $O/kat.log 2>&1
rc=$?; tail -2 $O/kat.log; [ $rc -ne 0 ] && exit $rc
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py"
$K xcd_rows 1,0 --workload moe_dsd --rounds 7 --iters 4 >> $O/ab.jsonl 2>>$O/err.log || exit $?
$K xcd_rows 1,0 --workload moe --rounds 7 --iters 3 >> $O/ab.jsonl 2>>$O/err.log || exit $?
cat $O/ab.jsonl

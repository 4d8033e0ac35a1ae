#!/bin/bash
# Same-process A/B of the round-5 library (build/exp/r05.so, commit 6823fb1)
# against the current one (build/exp/cur.so) on config 5 (DSD M = 131072,
# 2%), the headline and config 3.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-reg}; mkdir -p $O
E="timeout -k 10 240 python -u scripts/exp_bench.py"
$E --op dsd --m 131072 --density 0.02 build/exp/r05.so build/exp/cur.so >> $O/ab.jsonl 2>>$O/err.log || exit $?
$E --op dsd --density 0.5 build/exp/r05.so build/exp/cur.so >> $O/ab.jsonl 2>>$O/err.log || exit $?
$E --op pair --density 0.2 build/exp/r05.so build/exp/cur.so >> $O/ab.jsonl 2>>$O/err.log || exit $?
cat $O/ab.jsonl

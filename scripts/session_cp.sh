#!/bin/bash
# Cache-policy bits on the LDS-DMA loads (scripts/build_cp_variant.py):
# same-process A/B of the variant libraries on SDD 16384 / config 4 / the
# headline DSD, after the 16384 stride measurement.
set -u
TAG=$1; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
bash scripts/session_stride16k.sh $TAG || exit $?
L="build/exp/cur.so build/exp/cp_nt.so build/exp/cp_sc1.so build/exp/cp_sc0sc1.so"
E="timeout -k 10 300 python -u scripts/exp_bench.py"
for tr in NT NN TT; do
  $E --op op --xop sdd --trans $tr --k 16384 --density 1.0 --rounds 5 --iters 4 $L >> $O/cp_ab.jsonl 2>>$O/err.log || exit $?
  tail -1 $O/cp_ab.jsonl
done
$E --op moe_sdd --rounds 5 --iters 10 $L >> $O/cp_ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/cp_ab.jsonl
$E --op dsd --density 0.5 --rounds 7 --iters 50 $L >> $O/cp_ab.jsonl 2>>$O/err.log || exit $?
tail -1 $O/cp_ab.jsonl

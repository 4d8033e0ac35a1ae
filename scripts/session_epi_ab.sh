#!/bin/bash
# Same-process A/B of the 4-wave epilogue variants on DSD 4096^3 (knob
# dsd4w: 1 shipped choice, 5 double slots kEpi 3, 6 bar2 kEpi 4, 7 the
# interleaved copy-out kEpi 5) and of the DDS 20% pair placement.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-epi_ab}; mkdir -p $O
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py"
for d in 0.5 0.1 0.3 0.9; do
  $K dsd4w 1,5,6,7 --workload dsd --density $d --rounds 9 --iters 30 >> $O/ab.jsonl 2>>$O/err.log || exit $?
done
$K dds_xcd2 3,0,1 --workload dds --density 0.2 --rounds 9 --iters 30 >> $O/ab.jsonl 2>>$O/err.log || exit $?
cat $O/ab.jsonl

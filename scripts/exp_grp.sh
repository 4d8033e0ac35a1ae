#!/bin/bash
# SDD 8192^2 x 8192 between 4 and 8 blocks per CU (256 CUs: 1024..2048
# blocks): the grouped 128x512 tile (forced from 4 per CU) vs the k-split
# block tile (grouped off), same library, same process per point.
set -o pipefail
mkdir -p gpurun_out/grp
L=sputnik_amd/libsputnik.so
for d in 0.25 0.3125 0.375 0.4375 0.5; do
  SPUTNIK_AMD_GROUPED_MIN_PER_CU=4 timeout -k 10 300 python scripts/exp_bench.py --op sdd --k 8192 --density $d $L | sed 's/"op": "sdd"/"op": "sdd_grouped"/' >> gpurun_out/grp/exp.jsonl 2>> gpurun_out/grp/exp.err || exit $?
  SPUTNIK_AMD_GROUPED_SDD=0 timeout -k 10 300 python scripts/exp_bench.py --op sdd --k 8192 --density $d $L | sed 's/"op": "sdd"/"op": "sdd_ksplit"/' >> gpurun_out/grp/exp.jsonl 2>> gpurun_out/grp/exp.err || exit $?
done
cat gpurun_out/grp/exp.jsonl

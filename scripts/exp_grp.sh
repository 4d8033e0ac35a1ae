# SDD between 4 and 16 blocks per CU: grouped 128x512 tile vs the k-split block tile.
set -o pipefail
mkdir -p gpurun_out/grp
L=sputnik_amd/libsputnik.so
for d in 0.25 0.5 1.0; do
  timeout -k 10 300 python scripts/exp_bench.py --op sdd --k 8192 --density $d $L >> gpurun_out/grp/exp.jsonl 2>> gpurun_out/grp/exp.err || exit $?
  SPUTNIK_AMD_GROUPED_SDD=0 timeout -k 10 300 python scripts/exp_bench.py --op sdd --k 8192 --density $d $L | sed 's/"op": "sdd"/"op": "sdd_ksplit"/' >> gpurun_out/grp/exp.jsonl 2>> gpurun_out/grp/exp.err || exit $?
done
cat gpurun_out/grp/exp.jsonl

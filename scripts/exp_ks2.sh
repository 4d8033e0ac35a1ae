# k-split SDD vs CfgBlock vs grouped at several block counts.
set -o pipefail
mkdir -p gpurun_out/ks2
for d in 0.5 0.9 0.99; do
  timeout -k 10 300 python scripts/exp_bench.py --op sdd --density $d build/exp/base.so build/exp/ks.so >> gpurun_out/ks2/sdd.jsonl 2>> gpurun_out/ks2/sdd.err || exit $?
  SPUTNIK_AMD_GROUPED_SDD=0 timeout -k 10 300 python scripts/exp_bench.py --op sdd --density $d build/exp/base.so build/exp/ks.so | sed 's/"op": "sdd"/"op": "sdd_nogroup"/' >> gpurun_out/ks2/sdd.jsonl 2>> gpurun_out/ks2/sdd.err || exit $?
done
timeout -k 10 300 python scripts/exp_bench.py --op moe_sdd build/exp/ks.so >> gpurun_out/ks2/sdd.jsonl 2>> gpurun_out/ks2/sdd.err || exit $?
SPUTNIK_AMD_GROUPED_SDD=0 timeout -k 10 300 python scripts/exp_bench.py --op moe_sdd build/exp/ks.so | sed 's/"op": "moe_sdd"/"op": "moe_sdd_nogroup"/' >> gpurun_out/ks2/sdd.jsonl 2>> gpurun_out/ks2/sdd.err || exit $?
cat gpurun_out/ks2/sdd.jsonl

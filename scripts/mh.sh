set -o pipefail
O=gpurun_out/mh1; mkdir -p $O
for d in 0.5 0.1 0.3 0.9; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d build/exp/*.so >> $O/exp.jsonl 2> $O/exp.err || exit 1
done
timeout -k 10 300 python scripts/exp_bench.py --op pair build/exp/*.so >> $O/exp.jsonl 2> $O/exp.err || exit 1
timeout -k 10 300 python scripts/exp_bench.py --op op --xop dds --density 0.2 build/exp/*.so >> $O/exp.jsonl 2> $O/exp.err || exit 1

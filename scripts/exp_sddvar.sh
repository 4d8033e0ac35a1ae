# k-split SDD variants (lag priority off, per-step loop) vs shipped, interleaved A/B.
set -o pipefail
mkdir -p gpurun_out/sddvar
for d in 0.2 0.5; do
  timeout -k 10 300 python scripts/exp_bench.py --op sdd --density $d build/exp/base.so build/exp/noprio.so build/exp/noblk.so >> gpurun_out/sddvar/exp.jsonl 2>> gpurun_out/sddvar/exp.err || exit $?
done
cat gpurun_out/sddvar/exp.jsonl

set -o pipefail
O=gpurun_out/dx2; mkdir -p $O
for d in 0.1 0.9 0.3; do

timeout -k 10 300 python scripts/exp_knob_ab.py dds_xcd2 0,1,3 --workload dds --density $d >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done

set -o pipefail
O=gpurun_out/so; mkdir -p $O
export SPUTNIK_AMD_GROUPED_MIN_PER_CU=4
timeout -k 10 300 python scripts/exp_knob_ab.py sdd_order 0,1,2,3,4 --workload op:sdd:NN:4096 --density 1.0 --rounds 5 --iters 20 >> $O/ab.jsonl 2>> $O/ab.err || exit 1
timeout -k 10 300 python scripts/exp_knob_ab.py sdd_order 0,1,2,3,4 --workload op:sdd:NN:8192 --density 1.0 --rounds 3 --iters 5 >> $O/ab.jsonl 2>> $O/ab.err || exit 1
for o in 1 2 3; do
SPUTNIK_AMD_SDD_ORDER=$o timeout -k 10 200 python bench.py --workload moe --steps 10 --warmup 3 > $O/moe_o$o.json 2> $O/moe.err || exit 1
done

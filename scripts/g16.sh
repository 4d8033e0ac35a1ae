set -o pipefail
O=gpurun_out/g16; mkdir -p $O
for t in NN TN NT; do
timeout -k 10 400 python scripts/exp_knob_ab.py sdd4w_max_ld 16384,1073741824 --workload op:sdd:$t:16384 --density 0.5 --rounds 3 --iters 3 >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
timeout -k 10 400 python scripts/exp_knob_ab.py sdd4w_max_ld 16384,1073741824 --workload op:sdd:NN:8192 --density 0.5 --rounds 3 --iters 5 >> $O/ab.jsonl 2>> $O/ab.err || exit 1

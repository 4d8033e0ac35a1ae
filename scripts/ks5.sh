set -o pipefail
O=gpurun_out/ks5; mkdir -p $O
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py"
$K sdd_ksplit_min_k 6144,4096,2048 --workload op:sdd:NN:4096 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd_ksplit_min_k 6144,2048 --workload op:sdd:NN:4096 --density 0.1 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd_ksplit_min_k 6144,2048 --workload op:sdd:NN:2048 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd_ksplit_min_k 6144,2048 --workload op:sdd:NN:8192 --density 0.1 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd_order 0,1,2,3,4 --workload op:sdd:NT:8192 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd_order 0,1,2,3,4 --workload op:sdd:NN:8192 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd4w_max_ld 16384,32768 --workload op:sdd:NT:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K sdd4w_max_ld 16384,32768 --workload op:sdd:NN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
cat $O/ab.jsonl

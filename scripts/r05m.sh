set -o pipefail
bash scripts/gpu_measure.sh r05m 1 || exit $?
O=gpurun_out/r05m
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py sdd_order 0,1"
$K --workload op:sdd:NN:16384 --density 0.1 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NT:8192 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
cat $O/ab.jsonl

set -o pipefail
O=gpurun_out/moe_ab; mkdir -p $O
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py"
$K sdd_order 1,2,3,4,0 --workload moe_sdd --rounds 5 --iters 4 >> $O/ab.jsonl 2>>$O/err.log || exit $?
$K sdd4w_max_ld 16384,1073741824 --workload moe_sdd --rounds 5 --iters 4 >> $O/ab.jsonl 2>>$O/err.log || exit $?
$K dsd4w 1,0 --workload moe_sdd --rounds 5 --iters 4 >> $O/ab.jsonl 2>>$O/err.log || exit $?
cat $O/ab.jsonl

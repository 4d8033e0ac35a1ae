set -o pipefail
bash scripts/gpu_session.sh r05n || exit $?
O=gpurun_out/r05n
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py sdd4w_max_ld 16384,1073741824"
$K --workload op:sdd:TN:16384 --density 0.1 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
SWEEP_TAG=r05sw4 bash scripts/sweep.sh || exit 1
for w in sdd_dds moe panel; do
  timeout -k 10 300 python bench.py --workload $w > $O/w_$w.json 2> $O/w_$w.err || exit 1
done

set -o pipefail
O=gpurun_out/bo3; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_kat.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "sdd or SDD or moe or config3" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
timeout -k 10 200 python bench.py --workload moe --steps 30 --warmup 5 > $O/moe_$r.json 2> $O/moe.err || exit 1
done
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py sdd_order 0,1"
$K --workload op:sdd:NN:16384 --density 0.1 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NN:4096 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
cat $O/ab.jsonl $O/moe_*.json

set -o pipefail
O=gpurun_out/bo2; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kat.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "sdd or SDD" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
K="timeout -k 10 240 python -u scripts/exp_knob_ab.py sdd_order 0,1"
$K --workload op:sdd:NN:8192 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NT:8192 --density 0.5 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NT:8192 --density 0.1 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NN:8192 --density 1.0 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:NT:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
$K --workload op:sdd:TT:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
SPUTNIK_AMD_SDD4W_MAX_LD=32768 $K --workload op:sdd:NN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
SPUTNIK_AMD_SDD4W_MAX_LD=32768 $K --workload op:sdd:TN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
timeout -k 10 240 python -u scripts/exp_knob_ab.py sdd4w_max_ld 16384,32768 --workload op:sdd:NN:16384 --density 0.5 --rounds 3 --iters 10 >> $O/ab.jsonl 2>>$O/err.log || exit 1
cat $O/ab.jsonl

set -o pipefail
O=gpurun_out/ks4; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kat.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -k "sdd or moe or config3" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for o in 0 1; do
SPUTNIK_AMD_SDD_ORDER=$o timeout -k 10 200 python bench.py --workload moe --steps 30 --warmup 5 > $O/moe_o${o}_$r.json 2> $O/moe.err || exit 1
done; done
PYTHONPATH=$PWD timeout -k 10 300 python scripts/exp_sdd_ks.py > $O/ks.jsonl 2> $O/ks.err || exit 1

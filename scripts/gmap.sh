set -o pipefail
O=gpurun_out/gmap; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kat.py tests/test_gpu_fuzz.py tests/test_gpu_dsd4w.py tests/test_gpu_configs.py -k "sdd or moe or config3" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "--op op --xop sdd --density 1.0" "--op op --xop sdd --density 0.5" "--op op --xop sdd --trans NT --density 1.0" "--op op --xop sdd --trans TN --density 1.0" "--op moe_sdd"; do
  timeout -k 10 300 python scripts/exp_bench.py $a build/exp/*.so >> $O/exp.jsonl 2>> $O/exp.err || exit 1
done
SPUTNIK_AMD_GROUPED_MIN_PER_CU=4 timeout -k 10 300 python scripts/exp_bench.py --op op --xop sdd --density 1.0 build/exp/*.so >> $O/exp4.jsonl 2>> $O/exp.err || exit 1

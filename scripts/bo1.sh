set -o pipefail
O=gpurun_out/bo1; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_fuzz.py tests/test_gpu_kat.py tests/test_gpu_dsd4w.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "--op op --xop dds --density 0.2" "--op op --xop dds --density 0.5" "--op pair" "--op op --xop dsd --trans TN --density 0.5" "--op op --xop dds --trans NT --density 0.5" "--density 0.5"; do
  timeout -k 10 300 python scripts/exp_bench.py $a build/exp/*.so >> $O/exp.jsonl 2>> $O/exp.err || exit 1
done

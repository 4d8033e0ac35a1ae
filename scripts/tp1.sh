set -o pipefail
O=gpurun_out/tp1; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kat.py -k "tall_pipe" > $O/tp_tests.log 2>&1; rc=$?; tail -5 $O/tp_tests.log; [ $rc -ne 0 ] && exit $rc
SPUTNIK_AMD_TALL4W=1 timeout -k 10 600 $T tests/test_gpu_configs.py tests/test_gpu_kat.py -k "tall or config5" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for t in 0 1; do
SPUTNIK_AMD_TALL4W=$t timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_t${t}_$r.json 2> $O/panel.err || exit 1
done; done

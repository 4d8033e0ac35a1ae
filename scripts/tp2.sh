set -o pipefail
O=gpurun_out/tp2; mkdir -p $O
for r in 1 2; do for l in tp_nt tp_wb; do
SPUTNIK_AMD_LIB=$PWD/build/exp/$l.so SPUTNIK_AMD_TALL4W=1 timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_${l}_$r.json 2> $O/panel.err || exit 1
done; done
SPUTNIK_AMD_TALL4W=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kat.py tests/test_gpu_configs.py -k "tall" > $O/tests.log 2>&1; tail -2 $O/tests.log

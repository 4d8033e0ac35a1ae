set -o pipefail
O=gpurun_out/tp9; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
SPUTNIK_AMD_TALL4W=1 timeout -k 10 300 $T tests/test_gpu_kat.py tests/test_gpu_configs.py -k "tall" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
SPUTNIK_AMD_LIB=$PWD/build/tlx/tl4.so SPUTNIK_AMD_TALL4W=1 PYTHONPATH=$PWD timeout -k 10 200 python scripts/exp_timeline_tall.py > $O/tl.jsonl 2> $O/tl.err || exit 1
for r in 1 2; do for l in base zi; do
SPUTNIK_AMD_LIB=$PWD/build/exp/$l.so SPUTNIK_AMD_TALL4W=1 timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_${l}_$r.json 2> $O/panel.err || exit 1
done; done
SPUTNIK_AMD_TALL4W=0 timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_t0.json 2> $O/panel.err || exit 1

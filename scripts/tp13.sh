set -o pipefail
O=gpurun_out/tp13; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kat.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -k "tall or config5" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for a in 100 115 130; do
SPUTNIK_AMD_TALL_ODD_SHARE=$a timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_a${a}_$r.json 2> $O/panel.err || exit 1
done; done
SPUTNIK_AMD_TALL_ODD_SHARE=120 SPUTNIK_AMD_LIB=$PWD/build/tlx/tl4.so PYTHONPATH=$PWD timeout -k 10 200 python scripts/exp_timeline_tall.py > $O/tl.jsonl 2> $O/tl.err || exit 1

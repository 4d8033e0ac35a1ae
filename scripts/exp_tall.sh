# Config 5 (DSD M=131072, 2%): CfgTall alternatives vs the shipped CfgDual.
set -o pipefail
mkdir -p gpurun_out/tall
SPUTNIK_AMD_LIB=$PWD/build/exp/tallw8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "dsd" > gpurun_out/tall/parity.log 2>&1; rc=$?
tail -2 gpurun_out/tall/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/exp_bench.py --m 131072 --density 0.02 build/exp/base.so build/exp/tallw8.so > gpurun_out/tall/exp.jsonl 2> gpurun_out/tall/exp.err || exit $?
cat gpurun_out/tall/exp.jsonl

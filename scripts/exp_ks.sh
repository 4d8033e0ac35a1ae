set -o pipefail
mkdir -p gpurun_out/ks
SPUTNIK_AMD_LIB=$PWD/build/exp/ks.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "sdd" > gpurun_out/ks/parity.log 2>&1; rc=$?
tail -3 gpurun_out/ks/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/exp_bench.py --op sdd --density 0.2 build/exp/base.so build/exp/ks.so > gpurun_out/ks/sdd.jsonl 2> gpurun_out/ks/sdd.err; rc=$?
cat gpurun_out/ks/sdd.jsonl; exit $rc

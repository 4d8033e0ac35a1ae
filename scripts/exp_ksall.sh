# k-split on SSD / SDS / DSS: parity on the reference problem lists, then timing vs base.
set -o pipefail
mkdir -p gpurun_out/ksall
SPUTNIK_AMD_LIB=$PWD/build/exp/ksall.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "ssd or sds or dss or ss_" > gpurun_out/ksall/parity.log 2>&1; rc=$?
tail -3 gpurun_out/ksall/parity.log; [ $rc -ne 0 ] && exit $rc
for lib in base ksall base ksall; do
  SPUTNIK_AMD_LIB=$PWD/build/exp/$lib.so timeout -k 10 300 python scripts/exp_ss.py >> gpurun_out/ksall/ss.jsonl 2>> gpurun_out/ksall/ss.err || exit $?
done
cat gpurun_out/ksall/ss.jsonl

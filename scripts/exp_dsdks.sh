# k-split 128x128 tiles for DSD/DDS (no pairs) vs the shipped 128x512 staggered tile.
set -o pipefail
mkdir -p gpurun_out/dsdks
SPUTNIK_AMD_LIB=$PWD/build/exp/dsdks.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "dsd_reference or dds_reference" > gpurun_out/dsdks/parity.log 2>&1; rc=$?
tail -3 gpurun_out/dsdks/parity.log; [ $rc -ne 0 ] && exit $rc
for d in 0.05 0.1 0.2 0.5; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d build/exp/base.so build/exp/dsdks.so >> gpurun_out/dsdks/exp.jsonl 2>> gpurun_out/dsdks/exp.err || exit $?
done
cat gpurun_out/dsdks/exp.jsonl

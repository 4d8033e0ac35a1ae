#!/bin/bash
# GPU parity (DSD/DDS: KATs, BASELINE configs, reference problem lists)
# against variant libraries: exp_parity.sh TAG lib...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  SPUTNIK_AMD_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_kat.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "dsd or dds or pair or graph or config" \
    > gpurun_out/$TAG/parity_$(basename $lib).log 2>&1
  rc=$?; echo "$lib parity rc=$rc: $(tail -1 gpurun_out/$TAG/parity_$(basename $lib).log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

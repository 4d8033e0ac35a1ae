#!/bin/bash
# GPU parity (DSD/DDS subset) against variant libraries: exp_parity.sh TAG lib...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  SPUTNIK_AMD_LIB=$PWD/$lib timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "dsd or dds" > gpurun_out/$TAG/parity_$(basename $lib).log 2>&1
  rc=$?; echo "$lib parity rc=$rc: $(tail -1 gpurun_out/$TAG/parity_$(basename $lib).log)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0

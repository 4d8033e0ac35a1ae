#!/bin/bash
# A/B of libraries through bench.py itself (sustained protocol), alternating.
# Usage: ab_bench.sh TAG lib1 lib2 ...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for lib in "$@"; do
    SPUTNIK_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --sweep "0.3,0.9" > gpurun_out/$TAG/$(basename $lib .so)_$rep.json 2>gpurun_out/$TAG/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "fail $lib rc=$rc"; tail -3 gpurun_out/$TAG/err.log; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/$TAG/$(basename $lib .so)_$rep.json').read().strip().splitlines()[-1]); print('$(basename $lib)', $rep, {k: v['value'] for k, v in d['by_density'].items()})"
  done
done

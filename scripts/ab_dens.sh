#!/bin/bash
# Interleaved A/B of build/exp variants on DSD 4096^3 at several densities.
set -u; mkdir -p gpurun_out/abd
for d in ${DENS:-0.5 0.3 0.1 0.9}; do
  timeout -k 10 300 python scripts/exp_bench.py --density $d "$@" > gpurun_out/abd/d$d.log 2>&1 || exit $?
  tail -1 gpurun_out/abd/d$d.log
done

#!/bin/bash
# Bitwise parity of build/exp variants vs base, then interleaved timing.
# Usage: ab_var.sh TAG "densities" [extra exp_bench args]
set -u
T=$1; mkdir -p gpurun_out/$T
timeout -k 10 200 python scripts/exp_parity.py build/exp/base.so $(ls build/exp/*.so | grep -v base.so) > gpurun_out/$T/parity.jsonl 2> gpurun_out/$T/parity.err
rc=$?; tail -1 gpurun_out/$T/parity.jsonl; [ $rc -ge 2 ] && { tail gpurun_out/$T/parity.err; exit $rc; }
for d in ${2:-0.5 0.1 0.9}; do
  timeout -k 10 200 python scripts/exp_bench.py --density $d build/exp/base.so $(ls build/exp/*.so | grep -v base.so) >> gpurun_out/$T/ab.jsonl 2>> gpurun_out/$T/ab.err || { tail gpurun_out/$T/ab.err; exit 1; }
done
cat gpurun_out/$T/ab.jsonl

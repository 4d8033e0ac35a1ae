#!/bin/bash
# Bitwise parity of build/exp variants vs base (scripts/exp_parity.py), then
# interleaved timing: DSD NN at the given densities, DDS NN / DSD TN at 50%.
# Usage: ab_var.sh TAG "densities"
set -u
T=$1; mkdir -p gpurun_out/$T
V="build/exp/base.so $(ls build/exp/*.so | grep -v base.so)"
timeout -k 10 300 python scripts/exp_parity.py $V > gpurun_out/$T/parity.jsonl 2> gpurun_out/$T/parity.err
rc=$?; tail -1 gpurun_out/$T/parity.jsonl; [ $rc -ge 2 ] && { tail gpurun_out/$T/parity.err; exit $rc; }
for d in ${2:-0.5 0.1 0.9}; do
  timeout -k 10 200 python scripts/exp_bench.py --density $d $V >> gpurun_out/$T/ab.jsonl 2>> gpurun_out/$T/ab.err || { tail gpurun_out/$T/ab.err; exit 1; }
done
for x in "dds NN" "dsd TN" "dds TN"; do
  set -- $x
  timeout -k 10 200 python scripts/exp_bench.py --op op --xop $1 --trans $2 --density 0.5 $V >> gpurun_out/$T/ab.jsonl 2>> gpurun_out/$T/ab.err || { tail gpurun_out/$T/ab.err; exit 1; }
done
cat gpurun_out/$T/ab.jsonl

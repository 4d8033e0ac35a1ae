#!/bin/bash
# Phase timelines (exp_tl2.py) of every build/exp/tl_*.so. Usage: tl_all.sh TAG [density]
TAG=$1; D=${2:-0.5}
mkdir -p gpurun_out/$TAG
for lib in build/exp/tl_*.so; do
  echo "== $lib" | tee -a gpurun_out/$TAG/tl.txt
  timeout -k 10 120 python scripts/exp_tl2.py $lib --density $D >> gpurun_out/$TAG/tl.txt 2>> gpurun_out/$TAG/tl.err || { echo "fail $lib"; tail -3 gpurun_out/$TAG/tl.err; exit 1; }
done
cat gpurun_out/$TAG/tl.txt

#!/bin/bash
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  for d in 0.5 0.1; do
    echo "== $lib $d" >> gpurun_out/$TAG/tl.txt
    timeout -k 10 120 python scripts/exp_timeline.py $lib --density $d $ACCT --dump gpurun_out/$TAG/$(basename $lib .so)_$d.npy >> gpurun_out/$TAG/tl.txt 2>>gpurun_out/$TAG/tl.err || { echo fail $lib; tail -3 gpurun_out/$TAG/tl.err; exit 1; }
  done
done
cat gpurun_out/$TAG/tl.txt

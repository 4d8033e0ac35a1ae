#!/bin/bash
# Interleaved A/B of build/exp/{base,cached,nodma,nomfma}.so at the given densities.
set -u
mkdir -p gpurun_out/$1
for d in ${2:-0.5 0.1}; do
  timeout -k 10 200 python scripts/exp_bench.py --density $d build/exp/base.so build/exp/cached.so build/exp/nodma.so build/exp/nomfma.so >> gpurun_out/$1/abl.jsonl 2>> gpurun_out/$1/abl.err || { tail gpurun_out/$1/abl.err; exit 1; }
done
cat gpurun_out/$1/abl.jsonl

#!/bin/bash
# Bitwise parity (tall launches included) and config-5 timing of build/exp variants.
set -u
T=$1; mkdir -p gpurun_out/$T
V="build/exp/base.so $(ls build/exp/*.so | grep -v base.so)"
timeout -k 10 300 python scripts/exp_parity.py $V > gpurun_out/$T/parity.jsonl 2> gpurun_out/$T/parity.err
rc=$?; tail -1 gpurun_out/$T/parity.jsonl; [ $rc -ge 2 ] && { tail gpurun_out/$T/parity.err; exit $rc; }
timeout -k 10 300 python scripts/exp_bench.py --m 131072 --density 0.02 --iters 20 $V > gpurun_out/$T/ab_panel.jsonl 2> gpurun_out/$T/ab.err || { tail gpurun_out/$T/ab.err; exit 1; }
timeout -k 10 300 python scripts/exp_bench.py --m 65536 --density 0.05 --iters 20 $V >> gpurun_out/$T/ab_panel.jsonl 2>> gpurun_out/$T/ab.err || { tail gpurun_out/$T/ab.err; exit 1; }
cat gpurun_out/$T/ab_panel.jsonl

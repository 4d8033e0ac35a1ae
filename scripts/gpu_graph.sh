#!/bin/bash
# Captured-graph checks: the graph / pair KATs, then bench.py eager vs
# --graph on the headline and config 3. Usage: gpu_graph.sh TAG
set -u
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kat.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "graph or pair or split or persistent" > $O/kat.log 2>&1
rc=$?; tail -3 $O/kat.log; [ $rc -ne 0 ] && exit $rc
for w in "" "--workload sdd_dds"; do
  for g in "" "--graph"; do
    timeout -k 10 200 python bench.py $w $g >> $O/bench.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
  done
done
python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d.get('graph', d['config'].get('graph')), d['value'], d['ms_per_step'])
"

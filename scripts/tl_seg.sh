#!/bin/bash
# Per-segment k-loop cycle sums (SPUTNIK_EXP=640 build at build/exp/tlseg.so).
set -u
mkdir -p gpurun_out/$1
SPUTNIK_AMD_LIB=build/exp/tlseg.so TIMELINE_SEG=1 TIMELINE_WARM_S=2 timeout -k 10 120 \
  python scripts/exp_timeline.py dsd50 dsd10 dsd90 > gpurun_out/$1/tl_seg.jsonl 2> gpurun_out/$1/tl_seg.err || { tail gpurun_out/$1/tl_seg.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/$1/tl_seg.jsonl'):
    d=json.loads(l); print(d['workload'], d['span_us'], d.get('clock_GHz'), d['pipeline'], d['steps'], json.dumps(d['segments_per_step']))
"

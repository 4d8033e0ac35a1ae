#!/bin/bash
# Same-box A/B of library env settings through bench.py (separate processes,
# alternated twice). Usage: scripts/env_ab.sh TAG "bench args" "ENV=V ..." ...
set -u
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for envs in "$@"; do
    line=$(env $envs timeout -k 10 120 python bench.py $ARGS 2>/dev/null | grep '^{')
    rc=$?
    v=$(echo "$line" | python3 -c "import sys,json; j=json.loads(sys.stdin.read()); print(j['value'], round(j['ms_per_step']*1e3,2))" 2>/dev/null)
    echo "{\"args\": \"$ARGS\", \"env\": \"$envs\", \"rep\": $rep, \"result\": \"$v\"}" | tee -a $OUT/env_ab.jsonl
  done
done

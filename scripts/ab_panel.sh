#!/bin/bash
# Tall-path parity + config-5 A/B of one env knob: scripts/ab_panel.sh VAR
set -u
V=${1:-SPUTNIK_AMD_TALL_XCD}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/abp; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -m gpu -k "tall or panel or persist" tests \
  > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    env $V=$v timeout -k 10 200 python bench.py --workload panel > $OUT/panel_${v}_$i.log 2>&1 || exit $?
    echo "$V=$v run $i: $(tail -1 $OUT/panel_${v}_$i.log | cut -c1-140)"
  done
done

#!/bin/bash
# PMC passes on the current build: the headline DSD at each density
# (scripts/pmc.sh -> pmc_latest.json) and the config 3 / 4 / 5 workloads
# (scripts/pmc_workload.sh -> pmc_workloads.json), then each workload's bench
# line (which picks up the same-build traffic once the summaries are copied
# into profiles/). Usage: scripts/session_pmc.sh TAG
set -u
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
bash scripts/pmc.sh $TAG "0.5 0.1 0.3 0.9" || exit $?
for w in sdd_dds panel moe; do
  bash scripts/pmc_workload.sh $TAG $w "--workload $w" || exit $?
done
python3 scripts/pmc_merge_workloads.py $O $O/pmc_workloads.json
cp $O/pmc_latest.json profiles/pmc_latest.json
cp $O/pmc_workloads.json profiles/pmc_workloads.json
for w in sdd_dds moe panel; do
  timeout -k 10 300 python bench.py --workload $w > $O/w_$w.json 2> $O/w_$w.err || exit $?
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
cat $O/w_*.json

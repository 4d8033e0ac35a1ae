#!/bin/bash
# r06c: GPU tests on the hoist build, then kernel traces of the config-3 and
# config-4 workloads (per-kernel time split).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06c; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread --junitxml=$O/junit.xml > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
cd /tmp; export TMPDIR=/tmp
for w in moe sdd_dds; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$w -o run -- \
    python3 $R/bench.py --workload $w --steps 20 --warmup 5 --no-cpu > $O/prof_$w.log 2>&1 || exit $?
done
cd $R
python3 - << 'PY'
import csv, glob
for w in ("moe", "sdd_dds"):
    for f in glob.glob(f"gpurun_out/r06c/prof_{w}/**/*kernel_stats.csv", recursive=True):
        print(w, f)
        for row in csv.DictReader(open(f)):
            print("  ", row["Name"][:90], row["Calls"], row["AverageNs"])
PY

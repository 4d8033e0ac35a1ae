# rocprofv3 kernel-trace summaries of the non-headline workloads: prof_workloads.sh TAG
set -o pipefail
TAG=${1:-r01}; R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in sdd_dds moe; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$w -o run -- \
    python3 $R/bench.py --workload $w --no-cpu > $OUT/prof_$w.log 2>&1 || exit $?
done

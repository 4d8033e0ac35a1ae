set -o pipefail
O=gpurun_out/ks2; mkdir -p $O
PYTHONPATH=$PWD timeout -k 10 300 python scripts/exp_sdd_ks.py > $O/ks.jsonl 2> $O/ks.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --workload sdd_dds --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1

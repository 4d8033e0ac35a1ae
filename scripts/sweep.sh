set -o pipefail
O=gpurun_out/${SWEEP_TAG:-r05sw2}; mkdir -p $O
timeout -k 10 1150 python bench.py --workload sweep > $O/sweep.jsonl 2> $O/sweep.err; rc=$?
echo "sweep rc=$rc"; wc -l $O/sweep.jsonl; exit $rc

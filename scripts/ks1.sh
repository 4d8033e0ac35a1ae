set -o pipefail
O=gpurun_out/ks1; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kat.py -k "ksplit or sdd" > $O/kat.log 2>&1; rc=$?; tail -3 $O/kat.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "config3" > $O/cfg.log 2>&1; rc=$?; tail -3 $O/cfg.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workload sdd_dds --steps 50 --warmup 10 > $O/bench_ks.json 2> $O/bench_ks.err || exit 1
SPUTNIK_AMD_SDD_KSPLIT=1 timeout -k 10 200 python bench.py --workload sdd_dds --steps 50 --warmup 10 > $O/bench_8w.json 2> $O/bench_8w.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --workload sdd_dds --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1

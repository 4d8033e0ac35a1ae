set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k4w6
timeout -k 10 240 python microbench/k4w/run_k4w.py --uniform --variants 0,3 --rounds 5 > gpurun_out/k4w6/u50.log 2>&1
rc=$?; cat gpurun_out/k4w6/*.log | grep -v Warning; exit $rc

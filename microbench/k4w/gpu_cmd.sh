set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k4w2
timeout -k 10 240 python microbench/k4w/run_k4w.py --uniform --variants 0,3,7,8,9,10,11,12,13,1,2 --rounds 5 > gpurun_out/k4w2/u50.log 2>&1
rc=$?; cat gpurun_out/k4w2/*.log | grep -v Warning; exit $rc

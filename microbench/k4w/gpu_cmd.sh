set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k4w1
timeout -k 10 180 python microbench/k4w/run_k4w.py --uniform > gpurun_out/k4w1/u50.log 2>&1 && \
timeout -k 10 180 python microbench/k4w/run_k4w.py > gpurun_out/k4w1/r50.log 2>&1 && \
timeout -k 10 180 python microbench/k4w/run_k4w.py --uniform --density 0.9 > gpurun_out/k4w1/u90.log 2>&1
rc=$?; cat gpurun_out/k4w1/*.log | grep -v Warning; exit $rc

set -u; mkdir -p gpurun_out/ab4
timeout -k 10 300 python scripts/exp_bench.py --m 131072 --density 0.02 "$@" > gpurun_out/ab4/c5.log 2>&1; tail -1 gpurun_out/ab4/c5.log

set -u
mkdir -p gpurun_out/ab3
E="timeout -k 10 300 python scripts/exp_bench.py"
$E --op pair --density 0.2 build/exp/base.so build/exp/snt.so build/exp/dnt.so > gpurun_out/ab3/pair.log 2>&1 && tail -1 gpurun_out/ab3/pair.log &&
$E --op moe build/exp/base.so build/exp/snt.so build/exp/dnt.so > gpurun_out/ab3/moe.log 2>&1 && tail -1 gpurun_out/ab3/moe.log &&
$E --density 0.5 build/exp/base.so build/exp/dnt.so > gpurun_out/ab3/d50.log 2>&1 && tail -1 gpurun_out/ab3/d50.log &&
$E --density 0.1 build/exp/base.so build/exp/dnt.so > gpurun_out/ab3/d10.log 2>&1 && tail -1 gpurun_out/ab3/d10.log

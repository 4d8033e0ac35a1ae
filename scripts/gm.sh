set -o pipefail
O=gpurun_out/gm2; mkdir -p $O
for spec in "op:sdd:NN:4096 1.0" "op:sdd:NN:4096 0.5" "op:sdd:NT:4096 1.0" "op:sdd:TN:4096 1.0" "op:sdd:TT:4096 1.0" "op:sdd:NN:8192 0.1" "op:sdd:NN:8192 0.2" "op:sdd:NN:2048 1.0" "op:sdd:NN:4096 0.3"; do
  set -- $spec
  timeout -k 10 300 python scripts/exp_knob_ab.py grouped_min_per_cu 1,2,3,4,5 --workload $1 --density $2 --rounds 5 --iters 20 >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done

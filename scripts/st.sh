set -o pipefail
O=gpurun_out/st; mkdir -p $O
for spec in "op:sdd:NN:4096 1.0" "op:sdd:NN:3968 1.0" "op:sdd:NN:4224 1.0" "op:dsd:NN:4096 1.0" "op:dsd:NN:3968 1.0"; do
  set -- $spec
  timeout -k 10 300 python scripts/exp_knob_ab.py grouped_min_per_cu 4 --workload $1 --density $2 --rounds 5 --iters 20 >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done

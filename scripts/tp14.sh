set -o pipefail
O=gpurun_out/tp14; mkdir -p $O
timeout -k 10 400 python scripts/exp_knob_ab.py tall_odd_share 100,110,120,130 > $O/ab.jsonl 2> $O/ab.err || exit 1
timeout -k 10 400 python scripts/exp_knob_ab.py tall_flush_w 0,4,8 >> $O/ab.jsonl 2>> $O/ab.err || exit 1

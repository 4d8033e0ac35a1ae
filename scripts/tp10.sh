set -o pipefail
O=gpurun_out/tp10; mkdir -p $O
for r in 1 2; do for w in 4 8 12; do
SPUTNIK_AMD_TALL_FLUSH_W=$w timeout -k 10 200 python bench.py --workload panel --steps 20 --warmup 5 > $O/panel_w${w}_$r.json 2> $O/panel.err || exit 1
done; done
for w in 4 8; do
SPUTNIK_AMD_TALL_FLUSH_W=$w SPUTNIK_AMD_LIB=$PWD/build/tlx/tl4.so PYTHONPATH=$PWD timeout -k 10 200 python scripts/exp_timeline_tall.py > $O/tl_w$w.jsonl 2> $O/tl.err || exit 1
done

set -o pipefail
O=gpurun_out/tp4; mkdir -p $O
for l in tl4 tlns; do
SPUTNIK_AMD_LIB=$PWD/build/tlx/$l.so SPUTNIK_AMD_TALL4W=1 PYTHONPATH=$PWD timeout -k 10 200 python scripts/exp_timeline_tall.py > $O/tl_$l.jsonl 2> $O/tl.err || exit 1
done

set -o pipefail
O=gpurun_out/tp12; mkdir -p $O
SPUTNIK_AMD_LIB=$PWD/build/tlx/tl4.so PYTHONPATH=$PWD timeout -k 10 200 python scripts/exp_timeline_tall.py > $O/tl.jsonl 2> $O/tl.err || exit 1

set -o pipefail
O=gpurun_out/dds1; mkdir -p $O
export SPUTNIK_AMD_LIB=$PWD/build/tlx/tl4.so
timeout -k 10 200 python scripts/exp_timeline4w.py op=dds 0.2 0.5 > $O/tl_dds.jsonl 2> $O/tl.err || exit 1
timeout -k 10 200 python scripts/exp_timeline4w.py 0.2 > $O/tl_dsd.jsonl 2>> $O/tl.err || exit 1

set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
bash scripts/exp_run.sh r06b "0.5 0.1 0.3 0.9" || exit $?
SPUTNIK_AMD_LIB=build/tlv/tl.so timeout -k 10 200 python -u scripts/exp_timeline4w.py 0.5 0.1 0.3 0.9 > $O/tl4.log 2>&1 || exit $?
SPUTNIK_AMD_LIB=build/tlv/tl.so timeout -k 10 200 python -u scripts/exp_timeline4w.py op=dds 0.2 >> $O/tl4.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/exp_knob_ab.py min_handoff 2,1,3 --workload dsd --density 0.3 --rounds 9 --iters 30 >> $O/ab.jsonl 2>>$O/ab_err.log || exit $?
timeout -k 10 240 python -u scripts/exp_knob_ab.py min_handoff 2,1,3 --workload dds --density 0.2 --rounds 9 --iters 30 >> $O/ab.jsonl 2>>$O/ab_err.log || exit $?
timeout -k 10 240 python -u scripts/exp_knob_ab.py min_handoff 2,1,3 --workload dsd --density 0.1 --rounds 9 --iters 30 >> $O/ab.jsonl 2>>$O/ab_err.log || exit $?
cat $O/ab.jsonl

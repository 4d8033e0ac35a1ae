#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the headline kernel for every build/exp/*.so
# (one rocprofv3 --pmc pass each, bench.py's driver-sized run at one
# density). Usage: scripts/pmc_variants.sh TAG [density]
set -u
TAG=$1; D=${2:-0.5}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG/pmcv; mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
for so in $R/build/exp/*.so; do
  n=$(basename $so .so)
  for grp in FETCH_SIZE WRITE_SIZE; do
    SPUTNIK_AMD_LIB=$so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -f csv \
      -d $OUT/$n/$grp -o pass -- python3 $R/bench.py --steps 20 --warmup 5 --sweep "" \
      --no-cpu --density $D > $OUT/$n.$grp.log 2>&1
    echo "$n $grp rc=$?"
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, statistics, sys
root = sys.argv[1]
for d in sorted(glob.glob(root + "/*/")):
    out = {}
    for grp in ("FETCH_SIZE", "WRITE_SIZE"):
        v = [float(r["Counter_Value"]) for f in glob.glob(d + grp + "/**/*counter_collection.csv", recursive=True)
             for r in csv.DictReader(open(f)) if "block_gemm" in r["Kernel_Name"]]
        out[grp] = statistics.median(v[:26]) if v else None
    f, w = out["FETCH_SIZE"], out["WRITE_SIZE"]
    print(os.path.basename(d.rstrip("/")), "fetch_MB", f and round(f * 2048 / 1e6, 1),
          "write_MB", w and round(w * 1024 / 1e6, 1))
PY
# FETCH_SIZE calibration on known byte counts: microbench/l2_to_cu at a
# 64 MiB span (beyond L2) in the contiguous and the 64-B-row shapes.
cd /tmp
for grp in FETCH_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $grp | cut -c1-12)
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/calib/$n -o pass -- \
    $R/microbench/l2_to_cu 64 > $OUT/calib_$n.log 2>&1
  echo "calib $grp rc=$?"
done
python3 - "$OUT/calib" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    agg = {}
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:40], r["Counter_Name"])
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    for (kn, cn), v in sorted(agg.items()):
        print(kn, cn, "median", sorted(v)[len(v) // 2], "n", len(v))
PY
echo "known bytes per dispatch: 256 x 8 x 4 x 1024 x 2000 = 16.78 GB"

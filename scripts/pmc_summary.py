#!/usr/bin/env python3
"""Per-density PMC summary of the bench's DSD kernel (scripts/pmc.sh output)
-> the JSON bench.py reads as roofline.traffic (keyed by shape, density and
build hash).

Per launch (median over the profiled dispatches of the DSD kernel,
block_gemm_kernel or dsd4w_kernel):
  hbm_bytes_per_launch = FETCH_SIZE x 2 + WRITE_SIZE (kilobytes in the CSV).
      MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes
      of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is
      exact for 16 B/lane stores. Both count L2 <-> fabric traffic, so
      Infinity-Cache hits are included (bytes that left the XCD L2s).
  hbm_GBps = that / the dispatch's duration in the same pass.
  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x SQ_BUSY_CYCLES /
      32): the matrix-pipe busy share of the kernel's SIMD-cycles, taking
      SQ_BUSY_CYCLES as summed over the 32 shader engines.
  l2_hit = TCC_HIT / (TCC_HIT + TCC_MISS).
Usage: pmc_summary.py <pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else None


def main():
    root, out = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    build = subprocess.run([sys.executable, "-c",
                            "import sputnik_amd as s; print(s.build_hash())"],
                           capture_output=True, text=True,
                           cwd=repo).stdout.strip()
    res = {}
    if os.path.exists(out):
        res = json.load(open(out))
    for ddir in sorted(glob.glob(os.path.join(root, "d*"))):
        if not os.path.isdir(ddir):
            continue
        density = os.path.basename(ddir)[1:]
        vals, durs = {}, []
        for f in glob.glob(os.path.join(ddir, "p*", "**", "*counter_collection.csv"),
                           recursive=True):
            for row in csv.DictReader(open(f)):
                if not re.search(r"block_gemm_kernel|dsd4w_kernel", row["Kernel_Name"]):
                    continue
                vals.setdefault(row["Counter_Name"], []).append(
                    float(row["Counter_Value"]))
                durs.append((int(row["End_Timestamp"]) -
                             int(row["Start_Timestamp"])) * 1e-9)
        if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
            continue
        fetch = median(vals["FETCH_SIZE"]) * 1024 * 2
        write = median(vals["WRITE_SIZE"]) * 1024
        dur = median(durs)
        entry = {
            "build_hash": build,
            "hbm_bytes_per_launch": int(fetch + write),
            "fetch_bytes_corrected": int(fetch), "write_bytes": int(write),
            "profiled_kernel_us": round(dur * 1e6, 2),
            "hbm_GBps": round((fetch + write) / dur / 1e9, 1),
            "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE; "
                    "L2<->fabric bytes (MALL hits included)",
        }
        if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals:
            busy = median(vals["SQ_VALU_MFMA_BUSY_CYCLES"])
            sq = median(vals["SQ_BUSY_CYCLES"])
            entry["SQ_VALU_MFMA_BUSY_CYCLES"] = busy
            entry["SQ_BUSY_CYCLES"] = sq
            entry["mfma_busy_frac"] = round(busy / (1024 * sq / 32), 4)
            entry["est_clock_GHz"] = round(sq / 32 / dur / 1e9, 3)
        if "TCC_HIT_sum" in vals:
            h, m = median(vals["TCC_HIT_sum"]), median(vals["TCC_MISS_sum"])
            entry["l2_hit"] = round(h / (h + m), 4)
        res[f"dsd_4096x4096x4096_{density}_f16"] = entry
        print(density, json.dumps(entry))
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

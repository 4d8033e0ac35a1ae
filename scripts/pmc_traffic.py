#!/usr/bin/env python3
"""Parse rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, kilobytes) for the
DSD kernel into a JSON the bench reads as roofline.traffic.

Correction per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the
bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is
exact for 16 B/lane stores. Both count L2 <-> fabric traffic (Infinity Cache
hits included), i.e. bytes that left the XCD L2s.
Usage: pmc_traffic.py <pmc dir> <key> <out.json>"""
import csv
import glob
import json
import os
import sys

root, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
vals = {}
for f in glob.glob(os.path.join(root, "p*", "pass_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if "block_gemm" not in row["Kernel_Name"]:
            continue
        vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
res = {}
if os.path.exists(out):
    res = json.load(open(out))
fetch = sorted(vals.get("FETCH_SIZE", []))
write = sorted(vals.get("WRITE_SIZE", []))
if fetch and write:
    f_med = fetch[len(fetch) // 2] * 1024 * 2
    w_med = write[len(write) // 2] * 1024
    res[key] = {"hbm_bytes_per_launch": int(f_med + w_med),
                "fetch_bytes_corrected": int(f_med), "write_bytes": int(w_med),
                "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE; "
                        "L2<->fabric bytes (MALL hits included)"}
    for k in ("TCC_HIT_sum", "TCC_MISS_sum"):
        if k in vals:
            res[key][k] = sorted(vals[k])[len(vals[k]) // 2]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res.get(key)))

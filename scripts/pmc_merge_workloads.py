#!/usr/bin/env python3
"""Merges the per-workload PMC summaries of one session
(gpurun_out/TAG/pmc_<workload>.json from scripts/pmc_workload.sh) into one
file keyed by workload name, as bench.py --pmc-workloads reads it.
Usage: pmc_merge_workloads.py TAG_DIR OUT.json"""
import json
import os
import sys

src, out = sys.argv[1], sys.argv[2]
merged = {}
for name in ("sdd_dds", "moe", "panel"):
    path = os.path.join(src, f"pmc_{name}.json")
    if os.path.exists(path):
        with open(path) as f:
            merged[name] = json.load(f)
with open(out, "w") as f:
    json.dump(merged, f, indent=1)
print(f"merged {sorted(merged)} -> {out}")

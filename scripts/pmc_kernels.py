#!/usr/bin/env python3
"""Per-kernel PMC summary of one workload (scripts/pmc_workload.sh output):
for every block_gemm / metadata kernel name, the median per dispatch of each
counter over the profiled calls, with the same corrections and derived
numbers as scripts/pmc_summary.py (FETCH_SIZE x2 + WRITE_SIZE = L2<->fabric
bytes per launch; MFMA busy share; clock estimate; L2 hit rate).
Usage: pmc_kernels.py <pmc dir> <out.json> <label>
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


def short(name):
    m = re.search(r"block_gemm_kernelI(DF16_|DF16b)(.*?)NS_10TileConfigI((?:Li\d+E)+)E", name)
    if not m:
        return name[:80]
    flags = "".join(re.findall(r"Lb(\d)", m.group(2)))
    cfg = "x".join(re.findall(r"Li(\d+)E", m.group(3)))
    return f"block_gemm {'f16' if m.group(1) == 'DF16_' else 'bf16'} flags={flags} cfg={cfg}"


def main():
    root, out, label = sys.argv[1], sys.argv[2], sys.argv[3]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    build = subprocess.run([sys.executable, "-c",
                            "import sputnik_amd as s; print(s.build_hash())"],
                           capture_output=True, text=True, cwd=repo).stdout.strip()
    per = {}
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"),
                       recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            d = per.setdefault(k, {"vals": {}, "durs": []})
            d["vals"].setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
            d["durs"].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    res = {"label": label, "build_hash": build, "kernels": {}}
    for k, d in per.items():
        v, dur = d["vals"], median(d["durs"])
        e = {"profiled_kernel_us": round(dur * 1e6, 2), "dispatches": len(d["durs"]),
             "counters": {c: median(x) for c, x in sorted(v.items())}}
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            fetch = median(v["FETCH_SIZE"]) * 1024 * 2
            write = median(v["WRITE_SIZE"]) * 1024
            e.update({"hbm_bytes_per_launch": int(fetch + write),
                      "fetch_bytes_corrected": int(fetch), "write_bytes": int(write),
                      "hbm_GBps": round((fetch + write) / dur / 1e9, 1)})
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "SQ_BUSY_CYCLES" in v:
            busy, sq = median(v["SQ_VALU_MFMA_BUSY_CYCLES"]), median(v["SQ_BUSY_CYCLES"])
            e["mfma_busy_frac"] = round(busy / (1024 * sq / 32), 4)
            e["est_clock_GHz"] = round(sq / 32 / dur / 1e9, 3)
        if "TCC_HIT_sum" in v:
            h, m = median(v["TCC_HIT_sum"]), median(v["TCC_MISS_sum"])
            e["l2_hit"] = round(h / (h + m), 4) if h + m else None
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-dispatch durations of the headline kernel from a rocprofv3
--kernel-trace run of `bench.py --steps K --warmup W` (the driver's command).

bench.py runs the headline density first: its launcher makes one checked
call, then W warm-up calls, then the K timed calls, so the timed launches
are DSD kernel dispatches (block_gemm_kernel / dsd4w_kernel) [1 + W, 1 + W
+ K) in start-time order.
Writes a JSON summary (average / median / min / max over the timed calls,
plus every duration) next to the numbers bench.py reported.
Usage: trace_headline.py <rocprof out dir> <bench json line file> W K <out.json>
"""
import csv
import glob
import json
import statistics
import sys


def main():
    root, bench_file, w, k, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), \
        int(sys.argv[4]), sys.argv[5]
    rows = []
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ("block_gemm_kernel" in r["Kernel_Name"]
                    or "dsd4w_kernel" in r["Kernel_Name"]):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"]))
    rows.sort()
    timed = rows[1 + w:1 + w + k]
    durs = [(e - s) / 1e3 for s, e, _ in timed]
    bench = None
    try:
        for line in open(bench_file):
            line = line.strip()
            if line.startswith("{"):
                bench = json.loads(line)
    except OSError:
        pass
    res = {
        "kernel": timed[0][2] if timed else None,
        "dispatches_total": len(rows),
        "timed_index_range": [1 + w, 1 + w + k],
        "timed_avg_us": round(statistics.mean(durs), 3) if durs else None,
        "timed_median_us": round(statistics.median(durs), 3) if durs else None,
        "timed_min_us": round(min(durs), 3) if durs else None,
        "timed_max_us": round(max(durs), 3) if durs else None,
        "timed_span_us": round((timed[-1][1] - timed[0][0]) / 1e3 / len(timed), 3)
        if timed else None,
        "durations_us": [round(d, 3) for d in durs],
        "warmup_durations_us": [round((e - s) / 1e3, 3) for s, e, _ in rows[1:1 + w]],
    }
    if bench is not None:
        res["bench_ms_per_step_us"] = round(bench["ms_per_step"] * 1e3, 3)
        res["bench_value"] = bench["value"]
        res["bench_build"] = bench.get("build")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k2: v for k2, v in res.items()
                      if k2 not in ("durations_us", "warmup_durations_us")}))


if __name__ == "__main__":
    main()

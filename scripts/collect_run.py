#!/usr/bin/env python3
"""Copy one scripts/gpu_session.sh (or gpu_measure.sh) run from gpurun_out/TAG
into the tracked profiles/rNN/TAG (NN from the tag's first three characters):
each step's JSON line, the rocprofv3 kernel stats of the driver's command and
of the headline, the timed-dispatch extract (headline_trace.json), the PMC
summaries, the step log, and the junit summary.
Usage: scripts/collect_run.py TAG"""
import json
import re
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    rnd = tag[:3] if re.match(r"r\d\d", tag) else "r02"
    dst = os.path.join(ROOT, "profiles", rnd, tag)
    os.makedirs(dst, exist_ok=True)
    for f in sorted(os.listdir(src)):
        if not f.endswith(".log") or f in ("smoke.log", "pytest_gpu.log",
                                           "prof.log", "steps.log"):
            continue
        last = [l for l in open(os.path.join(src, f)) if l.startswith("{")]
        if last:
            json.loads(last[-1])
            open(os.path.join(dst, f[:-4] + ".json"), "w").write(last[-1])
    shutil.copy(os.path.join(src, "steps.log"), dst)
    ks = os.path.join(src, "prof", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "dsd4096_d50_kernel_stats.csv"))
    ks = os.path.join(src, "prof_driver", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "driver_kernel_stats.csv"))
    for f in ("headline_trace.json", "pmc_sdd_dds.json", "pmc_panel.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), dst)
    for w in ("sdd_dds", "panel"):
        ks = os.path.join(src, "prof_" + w, "run_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(dst, w + "_kernel_stats.csv"))
    pmc = os.path.join(src, "pmc_latest.json")
    if os.path.exists(pmc):
        shutil.copy(pmc, os.path.join(dst, "pmc_latest.json"))
        shutil.copy(pmc, os.path.join(ROOT, "profiles", "pmc_latest.json"))
    junit = os.path.join(src, "junit.xml")
    if os.path.exists(junit):
        subprocess.check_call([sys.executable,
                               os.path.join(ROOT, "scripts", "junit_summary.py"),
                               junit,
                               os.path.join(dst, "gputest_summary.json"), tag])
    print("collected", tag, "->", dst)


if __name__ == "__main__":
    main()

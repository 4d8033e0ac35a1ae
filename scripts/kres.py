#!/usr/bin/env python3
"""Compact per-kernel register / scratch table of block_gemm.hip (hipcc
-Rpass-analysis=kernel-resource-usage), to spot spills after an edit.
Usage: kres.py [extra hipcc flags...]   (run from the repo root)"""
import re
import subprocess
import sys

import os
SRC = os.environ.get("KRES_SRC", "sputnik_amd/csrc/block_gemm.hip")


def short(name):
    m = re.search(r"block_gemm_kernelI(DF16_|DF16b)(.*?)NS_10TileConfigI((?:Li\d+E)+)EELb(\d)ELb(\d)", name)
    if not m:
        return name[:60]
    t = "f16" if m.group(1) == "DF16_" else "bf16"
    flags = "".join(re.findall(r"Lb(\d)", m.group(2)))
    cfg = "x".join(re.findall(r"Li(\d+)E", m.group(3)))
    return f"{t} so/skc/dkc/outT={flags} cfg={cfg} sin/sd={m.group(4)}{m.group(5)}"


def main():
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC",
           "--offload-arch=gfx950", "-Iinclude", "-x", "hip", "-c", SRC,
           "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": short(m.group(1))}
            rows.append(cur)
            continue
        for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "TotalSGPRs"):
            m = re.search(key + r": (\d+)", line)
            if m and cur is not None:
                cur[key.split()[0]] = int(m.group(1))
    for r in rows:
        print(f"{r['name']:<75} V{r.get('VGPRs', '?'):>4} A{r.get('AGPRs', '?'):>4} "
              f"S{r.get('TotalSGPRs', '?'):>4} scratch {r.get('ScratchSize', '?')}")


if __name__ == "__main__":
    main()

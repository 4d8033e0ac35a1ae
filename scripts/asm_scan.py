#!/usr/bin/env python3
"""Where do scratch spills sit in one kernel of a --save-temps .s file?
Prints the kernel's line count, its MFMA line span and the scratch
instructions inside / outside the basic blocks that hold MFMAs.
Usage: asm_scan.py file.s kernel_symbol_substring"""
import re
import sys

s = open(sys.argv[1]).read().splitlines()
key = sys.argv[2]
start = next(i for i, l in enumerate(s) if l.startswith("_Z") and key in l and l.rstrip().endswith(key.split()[-1]) or (l.startswith("_Z") and key in l and ":" in l))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
body = s[start:end]
blocks, cur = [], {"label": "entry", "lines": []}
for l in body:
    if re.match(r"^\.LBB\d+_\d+:", l):
        blocks.append(cur)
        cur = {"label": l.split(":")[0], "lines": []}
    cur["lines"].append(l)
blocks.append(cur)
print("lines", len(body), "blocks", len(blocks))
tot_sc = 0
for b in blocks:
    mf = sum("v_mfma" in l for l in b["lines"])
    sc = sum("scratch_" in l for l in b["lines"])
    tot_sc += sc
    if mf or sc:
        print(f'{b["label"]:>14} lines {len(b["lines"]):5d} mfma {mf:4d} scratch {sc:3d}')
print("scratch total", tot_sc)

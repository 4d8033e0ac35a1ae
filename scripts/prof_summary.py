#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel name, calls, avg/min/max us).
Usage: scripts/prof_summary.py <run_results.db> [out.md]"""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute(
    "select name, count(*), avg(duration), min(duration), max(duration), "
    "sum(duration), max(grid_x), max(workgroup_x), max(lds_size), "
    "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count) "
    "from kernels group by name order by sum(duration) desc").fetchall()
total = sum(r[5] for r in rows) or 1
lines = ["| kernel | calls | avg us | min us | max us | % time | grid | wg | LDS | VGPR | AGPR | SGPR |",
         "|---|---|---|---|---|---|---|---|---|---|---|---|"]
for r in rows:
    name = r[0] if len(r[0]) < 110 else r[0][:107] + "..."
    lines.append(f"| `{name}` | {r[1]} | {r[2]/1e3:.2f} | {r[3]/1e3:.2f} | "
                 f"{r[4]/1e3:.2f} | {100*r[5]/total:.1f} | {r[6]} | {r[7]} | "
                 f"{r[8]} | {r[9]} | {r[10]} | {r[11]} |")
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")

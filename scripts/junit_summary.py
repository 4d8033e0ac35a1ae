#!/usr/bin/env python3
"""Summarise a pytest junit XML into a small tracked JSON record.

Usage: junit_summary.py JUNIT.xml OUT.json [label]
The record keeps every test id with its outcome and duration, plus totals,
so a GPU run's pass/fail evidence survives in profiles/ (gpurun_out/ is
scratch).
"""
import json
import sys
import xml.etree.ElementTree as ET


def main():
    src, dst = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    root = ET.parse(src).getroot()
    suites = [root] if root.tag == "testsuite" else list(root)
    tests = []
    for s in suites:
        for c in s.iter("testcase"):
            outcome = "passed"
            for child in c:
                if child.tag in ("failure", "error"):
                    outcome = "failed"
                elif child.tag == "skipped":
                    outcome = "skipped"
            tests.append({
                "id": f"{c.get('classname')}::{c.get('name')}",
                "outcome": outcome,
                "seconds": round(float(c.get("time", 0.0)), 3),
            })
    totals = {}
    for t in tests:
        totals[t["outcome"]] = totals.get(t["outcome"], 0) + 1
    out = {
        "label": label,
        "source": src,
        "timestamp": suites[0].get("timestamp") if suites else None,
        "hostname": suites[0].get("hostname") if suites else None,
        "totals": totals,
        "total_seconds": round(sum(t["seconds"] for t in tests), 2),
        "tests": tests,
    }
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(dst, totals)


if __name__ == "__main__":
    main()

"""Host-side logic of bench.py (no GPU): argument defaults per workload and
the PMC lookups that decide what a line may claim."""

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _parse(argv):
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("argv,steps,warmup", [
    ([], 100, 100),                                   # the headline
    (["--steps", "20", "--warmup", "5"], 20, 5),      # the driver's command
    (["--workload", "sdd_dds"], 1000, 1000),          # >= 100 ms of load
    (["--workload", "panel"], 500, 500),
    (["--workload", "moe"], 100, 100),
    (["--workload", "sdd_dds", "--steps", "7"], 7, 1000),
])
def test_step_defaults_per_workload(argv, steps, warmup):
    a = _parse(argv)
    assert (a.steps, a.warmup) == (steps, warmup)


def test_pmc_traffic_needs_same_build_and_shape(tmp_path):
    p = tmp_path / "pmc.json"
    key = "dsd_4096x4096x4096_0.5_f16"
    p.write_text(json.dumps({key: {"build_hash": "abc", "hbm_bytes_per_launch": 123}}))
    assert bench.pmc_traffic(str(p), key, "abc") == (123, "rocprofv3 --pmc, same build")
    b, note = bench.pmc_traffic(str(p), key, "other")
    assert b is None and "other" in note
    # an N > 1 rank's panel (2176 rows) has no entry of its own
    b, note = bench.pmc_traffic(str(p), "dsd_2176x4096x4096_0.5_f16", "abc")
    assert b is None and "no PMC entry" in note
    assert bench.pmc_traffic(str(tmp_path / "missing.json"), key, "abc")[0] is None

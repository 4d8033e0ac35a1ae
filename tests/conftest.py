"""pytest configuration: repo root on sys.path, the `gpu` marker.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, ABI.
`-m gpu` runs on an MI355X: parity of the HIP kernels (through the C-ABI)
against the CPU oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an AMD MI355X (gfx950) GPU and libsputnik.so")

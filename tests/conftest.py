"""Shared test setup: import paths and the `gpu` marker.

`-m "not gpu"` runs here (no GPU): the oracle against the golden vectors,
host logic, and the C-ABI export check.  `-m gpu` runs on the MI355X box and
compares the HIP path (through the C-ABI) with the oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libedgpu.so)")
    config.addinivalue_line("markers", "slow: long CPU test")

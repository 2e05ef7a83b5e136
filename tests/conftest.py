"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on any CPU box (oracle vs golden fixtures, host logic,
C-ABI exports, gloo multi-process); `-m gpu` needs a gfx950 device and
exercises the HIP kernels through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sdn-mpi-router_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running (full-size fabrics)")

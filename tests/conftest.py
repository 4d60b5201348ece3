"""Test configuration: `gpu` marker, import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, the
C-ABI library's exports.  `-m gpu` runs on an MI355X and calls the HIP path
through the C-ABI, with the oracle as the checker.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simplex-solver_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")

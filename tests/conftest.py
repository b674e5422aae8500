"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs the oracle-vs-golden checks, host logic and C-ABI load
tests on CPU; `-m gpu` runs the HIP parity tests on a real MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")

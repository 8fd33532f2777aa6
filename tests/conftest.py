"""Test configuration: markers and import paths.

`-m "not gpu"` runs here (no GPU): oracle known answers, golden fixtures,
scene loader, host logic, C-ABI exports, 2-rank gloo protocol.
`-m gpu` runs on an MI355X: parity of the gfx950 kernel (through the C ABI)
against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "concurrent-raytracer-go_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # oracle renders in the tests use at most 16 threads (a GPU box's CPU
    # share); the oracle's own default is the affinity count (runtime.NumCPU())
    import oracle

    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    oracle.DEFAULT_THREADS = min(16, aff)


@pytest.fixture(scope="session")
def scenes_dir():
    return SCENES

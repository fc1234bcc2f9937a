import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-through-"
                         "perspective-map-registrations_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (and the HIP library, cross-compiled) if missing."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "lib", "libpanofuse.so")):
        subprocess.run(["make", "-j4", "-C", PKG], check=True)
    yield

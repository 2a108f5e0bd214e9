"""Shared fixtures.  `-m gpu` tests need a HIP device; everything else runs on the CPU.

Nothing here (or in any test) reads /root/reference: scene files and reference-derived data
live in tests/golden/ as fixtures.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the library and the oracle once if they are missing (host-side compile only)."""
    lib = os.path.join(ROOT, "raytracercore_amd", "librtcore_hip.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-j8"], check=True)
    if not os.path.exists(lib) or not os.path.exists(os.path.join(ROOT, "raytracercore_amd", "worker_host")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracercore_amd", "csrc"), "-j8"], check=True)
    yield


@pytest.fixture(scope="session")
def rc():
    import raytracercore_amd

    return raytracercore_amd


@pytest.fixture(scope="session")
def scenes(rc):
    return {name: rc.SceneLoader.from_file(rc.scene_path(name)) for name in ("bounce.txt", "die.txt")}


@pytest.fixture(scope="session")
def has_gpu(rc):
    return rc.device_count() > 0

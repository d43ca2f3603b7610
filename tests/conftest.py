import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def _ensure_built():
    import glob

    pkg = os.path.join(ROOT, "custom_go_client_benchmark_amd")
    if not glob.glob(os.path.join(pkg, "_native*.so")) or not os.path.exists(os.path.join(pkg, "bin", "fakegcs")):
        subprocess.run(["make", "-C", ROOT, "-j", str(min(16, os.cpu_count() or 8)), "all"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def native():
    import custom_go_client_benchmark_amd as pkg

    return pkg._native


@pytest.fixture()
def server(native):
    srv = native.Server({"port": 0})
    srv.start()
    yield srv
    srv.stop()


@pytest.fixture(scope="session")
def gpu_available():
    import custom_go_client_benchmark_amd as pkg

    n = pkg._native.gpu_device_count()
    if n <= 0:
        pytest.fail("GPU test selected but no HIP device is visible (native GPU path cannot run)")
    return n

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "zarr-python_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "tuning: forces a kernel arm (the tuning build, libzarrhip_tune.so; "
                                       "tests/test_gpu_tuning_build.py runs these there)")


def set_tuning(key: int, value: int) -> None:
    """zhip_set_tuning for a test that forces a kernel arm or ablation: the
    knobs and the arm kernels exist only in the tuning build, so in the
    shipped library's process the test skips (test_gpu_tuning_build.py runs
    the `tuning` tests in a child process on libzarrhip_tune.so).  Setting 0
    (the production choice) always works."""
    from zarr_hip import _native as N

    if value and not N.lib().zhip_tuning_build():
        pytest.skip("kernel arm: tuning build only (tests/test_gpu_tuning_build.py)")
    N.check(N.lib().zhip_set_tuning(key, value), "zhip_set_tuning")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def device():
    if not gpu_available():
        pytest.skip("no GPU visible")
    import torch

    return torch.device("cuda:0")

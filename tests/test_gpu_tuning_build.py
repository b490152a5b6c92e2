"""The measurement arms live in a separate build (libzarrhip_tune.so, `make -C
zarr-python_amd tune`, -DZHIP_TUNING=1): the shipped libzarrhip.so has no arm
kernel and no kernel knob.  Tests that force an arm are marked `tuning`; in
the shipped library's process they skip, and this test runs all of them in
ONE child process on the tuning build (its log in gpurun_out/)."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shipped_library_has_no_knobs():  # (CPU: loads the library, launches nothing)
    """The product library refuses every kernel knob except its production
    value and reports that it is not the tuning build."""
    from zarr_hip import _native as N

    if N.tuning_build():
        pytest.skip("this process runs the tuning build")
    L = N.lib()
    for key in (1, 2, 3, 6):
        assert L.zhip_set_tuning(key, 0) == 0
        assert L.zhip_set_tuning(key, 5) == N.E_UNSUPPORTED
    assert L.zhip_set_tuning(5, 1) == 0  # host staging copies: not a kernel knob


@pytest.mark.gpu
@pytest.mark.timeout(1500)
def test_tuning_arms_in_tuning_build(device):
    from zarr_hip import _native as N

    if N.tuning_build():
        pytest.skip("this process already runs the tuning build")
    lib = N.TUNING_LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("tuning build absent (make -C zarr-python_amd tune)")
    logdir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    log = os.path.join(logdir, "tuning_tests.log")
    env = dict(os.environ, ZHIP_LIB=lib, ZARR_HIP_ALLOW_LIB_OVERRIDE="1")
    with open(log, "w") as fh:  # streamed to a file: progress stays visible
        r = subprocess.run([sys.executable, "-u", "-m", "pytest", "tests", "-m", "gpu and tuning", "-x", "-v",
                            "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread"],
                           cwd=ROOT, env=env, stdout=fh, stderr=subprocess.STDOUT, timeout=1400)
    with open(log) as fh:
        tail = fh.read()[-4000:]
    assert r.returncode == 0, tail
    assert " passed" in tail, tail

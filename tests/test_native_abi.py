"""CPU-side checks of the HIP C-ABI library: it loads, exports every symbol
include/zarrhip.h declares, its struct layouts match the ctypes/numpy mirrors,
and the CRC-combine algebra the kernels use (host emulation, same tables and
constants) reproduces CRC-32C exactly.  No GPU needed."""

import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "zarrhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zhip_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from zarr_hip import _native as N

    lib = N.lib()
    names = _header_functions()
    assert "zhip_decode" in names and "zhip_plan_create" in names
    for name in names:
        assert hasattr(lib, name), f"{name} declared in include/zarrhip.h but not exported"


def test_abi_version_and_selftest():
    from zarr_hip import _native as N

    assert N.lib().zhip_abi_version() == 1
    rc = N.lib().zhip_selftest()
    assert rc == 0, N.lib().zhip_last_error()


def test_struct_sizes_match_numpy_mirrors():
    from zarr_hip import _native as N

    chunk, sel, status = N._np_dtypes()
    assert ctypes.sizeof(N.Chunk) == chunk.itemsize == 48
    assert ctypes.sizeof(N.Sel) == sel.itemsize
    assert ctypes.sizeof(N.Status) == status.itemsize == 16
    assert ctypes.sizeof(N.Layout) == 4 + 4 + 32 + 64 + 8 + 16 + 16


@pytest.mark.parametrize("d", [1, 2, 3, 7, 15, 60, 64, 100, 4096, 65537, 1 << 20, (1 << 30) + 7])
def test_fdiv_python_matches_native(d):
    from zarr_hip import _native as N

    m, s = N.fdiv(d)
    rng = np.random.default_rng(d)
    for n in list(range(0, 200)) + list(rng.integers(0, 2**31 - 1, 500)):
        n = int(n)
        assert (n * m) >> s == n // d
        assert N.lib().zhip_fdiv_eval(n, d) == n // d


@pytest.mark.parametrize("n", [0, 1, 5, 16, 31, 4096, 4100, 32767, 32768, 32769, 65536 + 12,
                               1048576])
def test_emulated_kernel_crc_matches_oracle(n):
    """The device decomposition (units end-aligned at align16(N), per-thread Horner
    over 4 KiB strides, per-thread and per-unit shift constants, XOR combine, R->N
    correction) reproduces crc32c on the host."""
    from zarr_hip import _native as N

    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    L = N.Layout()
    L.ndim, L.itemsize = 1, 1
    L.shape[0] = n
    L.nbytes = n
    plan = N.Plan(L, upload=False)
    assert plan.emulate_chunk_crc(data) == O.crc32c(data)


def test_plan_rejects_bad_layouts():
    from zarr_hip import _native as N

    L = N.Layout()
    L.ndim, L.itemsize = 1, 3
    L.shape[0] = 4
    L.nbytes = 12
    with pytest.raises(N.NativeError):
        N.Plan(L, upload=False)
    L.itemsize = 4
    L.nbytes = 99
    with pytest.raises(N.NativeError):
        N.Plan(L, upload=False)

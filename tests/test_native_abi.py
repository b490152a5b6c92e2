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
PKG = os.path.join(ROOT, "zarr-python_amd")


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
    # k_decode_pair's scheme: 11/11/10-bit tables, four word accumulators, A4
    # fold, windowed per-lane multiply
    assert plan.emulate_chunk_crc(data, pair=True) == O.crc32c(data)


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


def _rows_case(shape, itemsize, sels, out_shape):
    """Layout of a C-contiguous out array of `out_shape` (bytes strides) over
    stored chunks of `shape`; sels = [(start, count)] per dim."""
    from zarr_hip import _native as N
    from zarr_hip.planner import SEL_DT, _make_layout

    nd = len(shape)
    ost = [int(np.prod(out_shape[d + 1:], dtype=np.int64)) * itemsize for d in range(nd)]
    L = _make_layout(shape, itemsize, ost, 0, b"\0")
    table = np.zeros(len(sels), SEL_DT)
    for i, (st, ct) in enumerate(sels):
        table[i]["start"][:nd] = st
        table[i]["count"][:nd] = ct
        table[i]["step"][:nd] = 1
    return L, table, ost


@pytest.mark.parametrize("case", [
    # (chunk shape, itemsize, selections, out shape)
    ((64, 64, 64), 4, [((0, 0, 0), (64, 64, 64))], (256, 256, 256)),
    ((64, 64, 64), 4, [((3, 0, 0), (50, 64, 64)), ((0, 17, 0), (64, 9, 64)), ((63, 63, 0), (1, 1, 64))],
     (128, 128, 64)),
    ((16, 32, 128), 2, [((0, 5, 0), (16, 20, 128)), ((7, 0, 0), (2, 32, 128))], (40, 70, 128)),
    ((3, 5, 256, 8), 2, [((1, 2, 5, 0), (2, 3, 240, 8)), ((0, 0, 0, 0), (3, 5, 256, 8))], (9, 11, 300, 8)),
    ((768, 16), 1, [((0, 0), (768, 16)), ((5, 0), (700, 16))], (800, 16)),  # 12 KiB chunks: unit starts before
    ((4096, 1024), 1, [((100, 0), (3000, 1024))], (5000, 1024)),             # 4 MiB chunks: 128 units
])
def test_rows_map_matches_scatter_semantics(case):
    """zhip_rows_map: for every (selection, unit, step, lane) the destination
    the row map gives equals the scatter out[out_sel] = chunk[chunk_sel]
    (chunk_utils.py:88-214) of that lane's 16 bytes, and lanes outside the
    selection or before the chunk start write nothing."""
    from zarr_hip import _native as N

    shape, it, sels, out_shape = case
    L, table, ost = _rows_case(shape, it, sels, out_shape)
    plan = N.Plan(L, upload=False)
    nseg = plan.units_per_chunk
    n = int(N.lib().zhip_rows_map_len(plan.handle, len(table)))
    assert n == len(table) * nseg * 8
    m = np.zeros(n, N.ROWBLK_DT)
    assert N.lib().zhip_rows_map(plan.handle, table.ctypes.data, len(table), m.ctypes.data, n) == 0
    m = m.reshape(len(table), nseg, 8)
    nd = len(shape)
    rb = shape[-1] * it
    nbytes = int(np.prod(shape)) * it
    E = -(-nbytes // 16) * 16
    t = np.arange(256)
    lane_row = (16 * t) // rb
    lane_col = (16 * t) % rb
    lead = shape[:-1]
    for s, (st, ct) in enumerate(sels):
        for u in range(nseg):
            for k in range(8):
                base_o = E - (u + 1) * 8 * 4096 + 4096 * k
                e = m[s, u, k]
                got_ok = (lane_row >= e["lo"]) & (lane_row < e["hi"])
                got_dst = int(e["rel"]) + lane_row * ost[nd - 2] + lane_col
                off = base_o + 16 * t
                R = np.where(off >= 0, off, 0) // rb
                coords = np.stack(np.unravel_index(np.minimum(R, int(np.prod(lead)) - 1), lead))
                want_ok = off >= 0
                dst = lane_col.copy()
                for d in range(nd - 1):
                    rel = coords[d] - st[d]
                    want_ok &= (rel >= 0) & (rel < ct[d])
                    dst = dst + rel * ost[d]
                np.testing.assert_array_equal(got_ok, want_ok, err_msg=f"sel {s} unit {u} step {k}")
                np.testing.assert_array_equal(got_dst[want_ok], dst[want_ok])


def test_rows_map_declines_offsets_beyond_32_bits():
    """A chunk whose footprint in out spans more than 2 GiB has no row map (the
    launch then takes the persistent row decode)."""
    from zarr_hip import _native as N
    from zarr_hip.planner import SEL_DT, _make_layout

    L = _make_layout((4, 64, 64), 4, [1 << 30, 256, 4], 0, b"\0")
    table = np.zeros(1, SEL_DT)
    table[0]["count"][:3] = (4, 64, 64)
    table[0]["step"][:3] = 1
    plan = N.Plan(L, upload=False)
    n = int(N.lib().zhip_rows_map_len(plan.handle, 1))
    m = np.zeros(n, N.ROWBLK_DT)
    assert N.lib().zhip_rows_map(plan.handle, table.ctypes.data, 1, m.ctypes.data, n) == N.E_UNSUPPORTED


def test_rows_map_declines_non_row_layouts():
    from zarr_hip import _native as N

    # 24-byte rows (not 2^k); 16-byte rows but 48 of them (a 4 KiB step would cross dim ndim-2)
    for shape in [(64, 24), (48, 16)]:
        L, table, _ = _rows_case(shape, 1, [((0, 0), shape)], shape)
        plan = N.Plan(L, upload=False)
        n = int(N.lib().zhip_rows_map_len(plan.handle, 1))
        m = np.zeros(max(n, 1), N.ROWBLK_DT)
        assert N.lib().zhip_rows_map(plan.handle, table.ctypes.data, 1, m.ctypes.data, n) == N.E_UNSUPPORTED


@pytest.mark.parametrize("n", [0, 1, 4095, (1 << 20) + 7, (3 << 20) + 123])
def test_host_copy_pool(n):
    """zhip_host_copy (the parallel memcpy of the staging path) is a memcpy."""
    from zarr_hip import _native as N

    src = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    dst = np.zeros(n, np.uint8)
    for threads in (1, 4, 16):
        dst[:] = 0
        assert N.lib().zhip_host_copy(dst.ctypes.data, src.ctypes.data, n, threads) == 0
        assert dst.tobytes() == src.tobytes()


@pytest.mark.parametrize("n", [65536, 126976, 131072, 196608, 524288, 1048576, 2 ** 21, 3 * 2 ** 20, 4100, 65552])
def test_emulated_interleaved_crc_matches_oracle(n):
    """k_decode_il's decomposition (a workgroup's eight 4 KiB steps at a stride
    of S steps, A_(4096 S) tables, per-workgroup lane constants with negative
    shifts where the stride outruns the chunk end) reproduces crc32c, with the
    interleave the decode takes (the widest of S = 32 / 16 / 8 that tiles the
    steps: 1 MiB chunks S = 32, 512 KiB S = 16); layouts whose step count no
    group of S x 8 steps tiles have no interleaved form."""
    from zarr_hip import _native as N

    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    L = N.Layout()
    L.ndim, L.itemsize = 1, 1
    L.shape[0] = n
    L.nbytes = n
    L.flags = N.LF_CRC
    plan = N.Plan(L, upload=False)
    got = plan.emulate_chunk_crc(data, pair="il")
    steps = -(-((n + 15) // 16 * 16) // 32768) * 8
    if steps % 16:
        assert got == 0xFFFFFFFF
    else:
        assert got == O.crc32c(data)


@pytest.mark.parametrize("n", [4096, 32768, 65536, 131072, 1048576, 4100, 65552, 2 ** 21 + 4096])
def test_emulated_xw_crc_matches_oracle(n):
    """k_decode_xw's decomposition (lane l of 8 KiB span r: eight blocks 1 KiB
    apart through the A_1024 tables, per-(span, lane) constants, negative
    shifts for the spans past the chunk end) reproduces crc32c."""
    from zarr_hip import _native as N

    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    L = N.Layout()
    L.ndim, L.itemsize = 1, 1
    L.shape[0] = n
    L.nbytes = n
    L.flags = N.LF_CRC
    plan = N.Plan(L, upload=False)
    assert plan.emulate_chunk_crc(data, pair="xw") == O.crc32c(data)


def _import_native(env_extra):
    """Import zarr_hip._native (and load the library) in a fresh interpreter
    with `env_extra` added; returns (returncode, stderr)."""
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("ZHIP_LIB", "ZARR_HIP_ALLOW_LIB_OVERRIDE")}
    env.update(env_extra)
    code = ("import sys; sys.path.insert(0, %r); from zarr_hip import _native as N; "
            "N.lib(); print('tuning', N.tuning_build())" % PKG)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout + r.stderr


def test_lib_override_needs_explicit_opt_in():
    """ZHIP_LIB alone (a stray variable in a user's environment) raises at
    import instead of swapping the shipped library for the tuning build; with
    ZARR_HIP_ALLOW_LIB_OVERRIDE=1 the named library loads."""
    from zarr_hip import _native as N

    if not os.path.exists(N.TUNING_LIB_PATH):
        pytest.skip("tuning build absent (make -C zarr-python_amd tune)")
    rc, out = _import_native({"ZHIP_LIB": N.TUNING_LIB_PATH})
    assert rc != 0 and "ZARR_HIP_ALLOW_LIB_OVERRIDE" in out and "ImportError" in out, out
    rc, out = _import_native({"ZHIP_LIB": N.TUNING_LIB_PATH, "ZARR_HIP_ALLOW_LIB_OVERRIDE": "1"})
    assert rc == 0 and "tuning True" in out, out
    rc, out = _import_native({})
    assert rc == 0 and "tuning False" in out, out


def test_tuning_build_refused_in_product_path(tmp_path):
    """A tuning build loaded through the opt-in path check alone is still
    refused when the opt-in is absent: copied over (or symlinked as) the
    product name, lib() raises NativeError."""
    import shutil

    from zarr_hip import _native as N

    if not os.path.exists(N.TUNING_LIB_PATH):
        pytest.skip("tuning build absent (make -C zarr-python_amd tune)")
    pkg = tmp_path / "zarr_hip"
    shutil.copytree(os.path.join(PKG, "zarr_hip"), pkg, ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    shutil.copy(N.TUNING_LIB_PATH, pkg / "_lib" / "libzarrhip.so")
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("ZHIP_LIB", "ZARR_HIP_ALLOW_LIB_OVERRIDE")}
    code = "import sys; sys.path.insert(0, %r); from zarr_hip import _native as N; N.lib()" % str(tmp_path)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "tuning build" in r.stderr, r.stderr


def test_non_basic_selections_refused_by_name():
    """zarr's orthogonal / coordinate / mask indexers hand integer arrays or
    masks: the pipeline refuses them with NotImplementedError naming the
    reason (BasicIndexer selections), not a TypeError from
    the planner; slices and integers (numpy ones included) pass."""
    import numpy as np

    from zarr_hip.pipeline import normalize_batch
    from zarr_hip.spec import ArraySpec

    class Spec:  # a foreign (zarr-like) spec object: takes the coercing path
        def __init__(self, s):
            self.s = s

    spec = ArraySpec((4, 4), np.dtype("float32"), 0.0)
    import zarr_hip.pipeline as P

    orig = P.coerce_spec
    P.coerce_spec = lambda s: s.s
    try:
        ok = normalize_batch([(None, Spec(spec), (slice(0, 4, 1), np.int64(2)), (slice(0, 4, 1),), False)])
        assert ok[0][1] is spec
        for bad in (np.array([0, 2]), [1, 3], np.array([True, False, True, False])):
            with pytest.raises(NotImplementedError, match="BasicIndexer"):
                normalize_batch([(None, Spec(spec), (slice(0, 4, 1), bad), (slice(0, 4, 1), slice(0, 2, 1)), False)])
    finally:
        P.coerce_spec = orig

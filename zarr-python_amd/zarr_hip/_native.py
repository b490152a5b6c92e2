"""ctypes binding of the HIP C-ABI library (include/zarrhip.h).

The product path has no CPU fallback: if ``libzarrhip.so`` is missing or a
call fails, this module raises.  The library is built in-tree by
``__graft_entry__.build()`` / ``make -C zarr-python_amd``.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

MAX_DIMS = 8

ST_OK = 0
ST_MISSING = 1
ST_CRC_MISMATCH = 2
ST_INDEX_OOB = 3
ST_LENGTH_MISMATCH = 4

LF_CRC = 1
LF_SWAP = 2
LF_SHARDED = 4
LF_INDEX_START = 8
LF_NO_WRITE = 16
LF_FLOAT = 32

CF_MISSING = 1

E_INVALID = -1
E_HIP = -2
E_IO = -4
E_UNSUPPORTED = -3

DF_FAST_ROWS = 1
DF_TILE = 2
DF_ROWS = 4
DF_TILE_PREFIX = 8
DF_BANK1 = 16  # deferred CRC verdicts: publish into workspace bank 1, check bank 0
DF_DEFER = 32  # opt in to deferred CRC verdicts (the Python path reads the verdict words)
DF_WHOLE = 64  # every selection is its chunk's whole region: affine row destinations (zarrhip.h)

PK_TILE4 = 1
PK_TILE4_ENCODE = 2
PK_TILE = 4
PK_TILEG = 8
PK_IL = 16

PF_INDEX_START = 1
PF_INDEX_CRC = 2
PF_KEEP_EMPTY = 4

_HERE = os.path.dirname(os.path.abspath(__file__))
# the shipped library, and the tuning build of the same sources with every
# measurement arm and kernel knob compiled in (make -C zarr-python_amd tune;
# scripts/armbench.py, tests/test_gpu_tuning_build.py).  ZHIP_LIB names
# another library to load, and is honoured only together with the explicit
# opt-in ZARR_HIP_ALLOW_LIB_OVERRIDE=1 (the measurement scripts set both): a
# stray ZHIP_LIB in a user's environment raises here instead of silently
# swapping the kernels, and lib() refuses a tuning build without the opt-in.
PRODUCT_LIB_PATH = os.path.join(_HERE, "_lib", "libzarrhip.so")
TUNING_LIB_PATH = os.path.join(_HERE, "_lib", "libzarrhip_tune.so")
OVERRIDE_OPT_IN = "ZARR_HIP_ALLOW_LIB_OVERRIDE"


def _override_allowed() -> bool:
    return os.environ.get(OVERRIDE_OPT_IN) == "1"


if os.environ.get("ZHIP_LIB") and not _override_allowed():
    raise ImportError(f"ZHIP_LIB={os.environ['ZHIP_LIB']!r} is set without {OVERRIDE_OPT_IN}=1: refusing to load a "
                      "library other than the shipped libzarrhip.so (unset ZHIP_LIB, or opt in explicitly)")
LIB_PATH = (os.environ.get("ZHIP_LIB") if _override_allowed() else None) or PRODUCT_LIB_PATH


class FDiv(ctypes.Structure):
    _fields_ = [("m", ctypes.c_uint32), ("s", ctypes.c_uint32)]


class Layout(ctypes.Structure):
    _fields_ = [
        ("ndim", ctypes.c_int32),
        ("itemsize", ctypes.c_int32),
        ("shape", ctypes.c_int32 * MAX_DIMS),
        ("out_stride", ctypes.c_int64 * MAX_DIMS),
        ("nbytes", ctypes.c_uint64),
        ("flags", ctypes.c_uint32),
        ("n_inner", ctypes.c_uint32),
        ("index_size", ctypes.c_uint32),
        ("_pad", ctypes.c_uint32),
        ("fill", ctypes.c_uint8 * 16),
    ]


class Chunk(ctypes.Structure):
    _fields_ = [
        ("src", ctypes.c_uint64),
        ("src_len", ctypes.c_uint64),
        ("out_off", ctypes.c_int64),
        ("flags", ctypes.c_uint32),
        ("slot", ctypes.c_uint32),
        ("sel", ctypes.c_uint32),
        ("_pad", ctypes.c_uint32 * 3),
    ]


class Sel(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_int32 * MAX_DIMS),
        ("count", ctypes.c_int32 * MAX_DIMS),
        ("step", ctypes.c_int32 * MAX_DIMS),
        ("div_step", FDiv * MAX_DIMS),
    ]


class Status(ctypes.Structure):
    _fields_ = [
        ("code", ctypes.c_uint32),
        ("stored", ctypes.c_uint32),
        ("computed", ctypes.c_uint32),
        ("aux", ctypes.c_uint32),
    ]


# numpy structured dtypes with the same byte layout (tables are built with numpy
# and uploaded as raw bytes)
def _np_dtypes():
    import numpy as np

    chunk = np.dtype([("src", "<u8"), ("src_len", "<u8"), ("out_off", "<i8"), ("flags", "<u4"),
                      ("slot", "<u4"), ("sel", "<u4"), ("_pad", "<u4", (3,))])
    sel = np.dtype([("start", "<i4", (MAX_DIMS,)), ("count", "<i4", (MAX_DIMS,)),
                    ("step", "<i4", (MAX_DIMS,)), ("div", "<u4", (MAX_DIMS, 2))])
    status = np.dtype([("code", "<u4"), ("stored", "<u4"), ("computed", "<u4"), ("aux", "<u4")])
    return chunk, sel, status


class Predict(ctypes.Structure):
    """zhip_predict (include/zarrhip.h)."""

    _fields_ = [("base", ctypes.c_uint64), ("outer", ctypes.c_uint64), ("inner", ctypes.c_uint64),
                ("per", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


# zhip_piece (include/zarrhip.h)
PIECE_DT = np.dtype([("host", "<u8"), ("nbytes", "<u8"), ("dst_off", "<u8"), ("flags", "<u8"),
                     ("file_off", "<u8")])
PIECE_PINNED = 1
PIECE_FILE = 2

# zhip_item / zhip_batch_geom (include/zarrhip.h): the native host planner's input
ITEM_DT = np.dtype([("src", "<u8"), ("src_len", "<u8"), ("out_off", "<i8"), ("missing", "<u4"), ("res", "<i4"),
                    ("start", "<i8", (MAX_DIMS,)), ("stop", "<i8", (MAX_DIMS,)), ("step", "<i8", (MAX_DIMS,))])
GEOM_DT = np.dtype([("ndim", "<i4"), ("perm", "<i4", (MAX_DIMS,)), ("_pad0", "<i4"),
                    ("shape", "<i8", (MAX_DIMS,)), ("ost", "<i8", (MAX_DIMS,)), ("inner", "<i8", (MAX_DIMS,)),
                    ("index_size", "<u4"), ("index_start", "<u4"), ("index_crc", "<u4"), ("_pad", "<u4")])
RESOLVED_DT = np.dtype([("src", "<u8"), ("len", "<u8"), ("missing", "<u8"), ("index_src", "<u8"),
                        ("n_rows", "<u4"), ("n_inner", "<u4")])
AGG_LAST_FULL, AGG_OUT_ALIGNED, AGG_UNIT_STEPS, AGG_ALL_FULL = 1, 2, 4, 8
E_BOUNDS = -5

# zhip_rowblk (include/zarrhip.h)
ROWBLK_DT = np.dtype([("rel", "<i4"), ("lo", "<u2"), ("hi", "<u2")])


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"zarr_hip native library not built: {LIB_PATH} is missing "
            "(run __graft_entry__.build() or `make -C zarr-python_amd`)")
    # torch first: the library then binds to the HIP runtime torch loaded
    # (one runtime per process; loading ours first leaves two, and the
    # second to initialise sees no device)
    import torch  # noqa: F401

    L = ctypes.CDLL(LIB_PATH)
    L.zhip_abi_version.restype = ctypes.c_int
    L.zhip_last_error.restype = ctypes.c_char_p
    L.zhip_device_count.restype = ctypes.c_int
    L.zhip_plan_create.argtypes = [ctypes.POINTER(Layout), ctypes.POINTER(ctypes.c_void_p)]
    L.zhip_plan_create.restype = ctypes.c_int
    L.zhip_plan_destroy.argtypes = [ctypes.c_void_p]
    L.zhip_plan_destroy.restype = ctypes.c_int
    L.zhip_plan_upload.argtypes = [ctypes.c_void_p]
    L.zhip_plan_upload.restype = ctypes.c_int
    L.zhip_plan_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_uint32)]
    L.zhip_plan_info.restype = ctypes.c_int
    L.zhip_plan_kernel_flags.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    L.zhip_plan_kernel_flags.restype = ctypes.c_int
    L.zhip_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.zhip_decode.restype = ctypes.c_int
    L.zhip_decode_indexed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.zhip_decode_indexed.restype = ctypes.c_int
    L.zhip_decode_predicted.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(Predict),
                                        ctypes.c_void_p]
    L.zhip_decode_predicted.restype = ctypes.c_int
    L.zhip_decode_mapped.argtypes = L.zhip_decode_predicted.argtypes[:-1] + [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_decode_mapped.restype = ctypes.c_int
    L.zhip_rows_map_len.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.zhip_rows_map_len.restype = ctypes.c_uint64
    L.zhip_rows_map.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                ctypes.c_uint64]
    L.zhip_rows_map.restype = ctypes.c_int
    L.zhip_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.zhip_encode.restype = ctypes.c_int
    L.zhip_encode_mapped.argtypes = L.zhip_encode.argtypes[:-1] + [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_encode_mapped.restype = ctypes.c_int
    L.zhip_shard_pack.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p]
    L.zhip_shard_pack.restype = ctypes.c_int
    L.zhip_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
    L.zhip_set_tuning.restype = ctypes.c_int
    L.zhip_last_kernel.argtypes = []
    L.zhip_last_kernel.restype = ctypes.c_char_p
    L.zhip_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.zhip_debug_stamps.restype = ctypes.c_int
    L.zhip_selftest.restype = ctypes.c_int
    L.zhip_emulate_chunk_crc.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_emulate_chunk_crc.restype = ctypes.c_uint32
    L.zhip_stage_h2d.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    L.zhip_stage_h2d.restype = ctypes.c_int
    L.zhip_stage_begin.argtypes = list(L.zhip_stage_h2d.argtypes)
    L.zhip_stage_begin.restype = ctypes.c_void_p
    L.zhip_stage_end.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_stage_end.restype = ctypes.c_int
    L.zhip_host_pinned.argtypes = [ctypes.c_void_p]
    L.zhip_host_pinned.restype = ctypes.c_int
    L.zhip_wait_words.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_wait_words.restype = ctypes.c_int
    L.zhip_wait_ranges.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                   ctypes.c_void_p]
    L.zhip_wait_ranges.restype = ctypes.c_int
    L.zhip_upload.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                              ctypes.c_uint64, ctypes.c_void_p]
    L.zhip_upload.restype = ctypes.c_int
    L.zhip_dv_check.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.zhip_dv_check.restype = ctypes.c_int
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.zhip_plan_batch.argtypes = [vp, vp, u32, vp, vp, u64, vp, vp, u32, vp, vp, vp, vp, vp, vp]
    L.zhip_plan_batch.restype = ctypes.c_int
    L.zhip_crc32c_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.zhip_crc32c_host.restype = ctypes.c_uint32
    L.zhip_host_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
    L.zhip_host_copy.restype = ctypes.c_int
    L.zhip_emulate_chunk_crc_pair.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_emulate_chunk_crc_pair.restype = ctypes.c_uint32
    L.zhip_emulate_chunk_crc_il.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_emulate_chunk_crc_il.restype = ctypes.c_uint32
    L.zhip_emulate_chunk_crc_xw.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.zhip_emulate_chunk_crc_xw.restype = ctypes.c_uint32
    L.zhip_fdiv_eval.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.zhip_fdiv_eval.restype = ctypes.c_uint32
    L.zhip_tuning_build.restype = ctypes.c_int
    if L.zhip_abi_version() != 1:
        raise NativeError("libzarrhip ABI version mismatch")
    if L.zhip_tuning_build() and not _override_allowed():
        raise NativeError(f"{LIB_PATH} is the tuning build (measurement arms compiled in): it loads only with "
                          f"{OVERRIDE_OPT_IN}=1")
    _lib = L
    return L


def tuning_build() -> bool:
    """True when the loaded library is the tuning build (arms, knobs)."""
    return bool(lib().zhip_tuning_build())


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().zhip_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed ({rc}): {msg}")


def fdiv(d: int) -> tuple[int, int]:
    """Magic numbers for n // d with 0 <= n < 2**31 (mirrors make_fdiv in capi.cpp)."""
    d = max(int(d), 1)
    l = (d - 1).bit_length()
    s = 31 + l
    m = ((1 << s) + d - 1) // d
    return m, s


class Plan:
    """Owns a zhip_plan (constant tables for one layout) on the current device."""

    def __init__(self, layout: Layout, upload: bool = True):
        self.layout = layout
        h = ctypes.c_void_p()
        check(lib().zhip_plan_create(ctypes.byref(layout), ctypes.byref(h)), "zhip_plan_create")
        self._h = h
        upc = ctypes.c_uint32()
        wsw = ctypes.c_uint32()
        check(lib().zhip_plan_info(h, ctypes.byref(upc), ctypes.byref(wsw)), "zhip_plan_info")
        self.units_per_chunk = upc.value
        self.workspace_words = wsw.value
        if upload:
            check(lib().zhip_plan_upload(h), "zhip_plan_upload")

    @property
    def handle(self):
        return self._h

    @property
    def kernel_flags(self) -> int:
        """ZHIP_PK_* bits: specialised kernels this layout admits."""
        f = ctypes.c_uint32()
        check(lib().zhip_plan_kernel_flags(self._h, ctypes.byref(f)), "zhip_plan_kernel_flags")
        return f.value

    def emulate_chunk_crc(self, data: bytes, pair: bool = False) -> int:
        buf = ctypes.create_string_buffer(bytes(data) + b"\0" * 16)
        fn = lib().zhip_emulate_chunk_crc_il if pair == "il" else lib().zhip_emulate_chunk_crc_xw if pair == "xw" else \
            lib().zhip_emulate_chunk_crc_pair if pair else lib().zhip_emulate_chunk_crc
        return int(fn(self._h, buf))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.zhip_plan_destroy(h)
            self._h = None

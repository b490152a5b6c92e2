"""Device CRC-32C of many equal-length regions of a device buffer, through the
fused decode kernel in verify-only mode (ZHIP_LF_NO_WRITE): each region is a
"chunk" of a 1-D uint8 layout whose 4-byte trailer is ignored; the kernel
records the computed CRC-32C in the status table.  Used by the encode side to
produce crc32c trailers (crc32c_.py:59-68) and by tests."""

from __future__ import annotations

import numpy as np

from . import _native as N
from .planner import CHUNK_DT, SEL_DT, _make_layout
from .pipeline import DecodeLaunch


def crc32c_regions(src, offsets, length: int, src_size: int | None = None) -> np.ndarray:
    """CRC-32C of src[o : o+length] for every o in offsets (src: torch uint8 CUDA
    tensor readable 64 bytes past each region + 4).  Returns uint32[n] (host)."""
    offsets = np.asarray(offsets, np.uint64)
    n = len(offsets)
    if n == 0:
        return np.zeros(0, np.uint32)
    L = _make_layout([int(length)], 1, [0], N.LF_CRC | N.LF_NO_WRITE, b"\0")
    ch = np.zeros(n, CHUNK_DT)
    ch["src"] = offsets
    ch["src_len"] = int(length) + 4
    size = int(src.numel()) if src_size is None else int(src_size)
    launch = DecodeLaunch(L, ch, np.zeros(1, SEL_DT), src, size, None, False, src.device)
    launch.launch()
    st = launch.statuses()
    return st["computed"].astype(np.uint32)

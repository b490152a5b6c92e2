"""Stores: a host MemoryStore and a device-resident store whose chunk and shard
blobs live in one HBM arena (the data layout the decode kernels read).

  MemoryStore   src/zarr/storage/_memory.py:27-166 (dict of bytes; get_sync returns a view)
  LocalStore    src/zarr/storage/_local.py (files; host side of the e2e path)
  StorePath     src/zarr/storage/_common.py:247 (a store + key acting as ByteGetter/ByteSetter)

DeviceStore has no direct reference counterpart (the reference's GpuMemoryStore,
_memory.py:247-330, is CuPy-only and holds one device buffer per key); here all
blobs share one arena so a whole batch decodes from a single base pointer with
16-byte-aligned, 256-byte-padded placements.
"""

from __future__ import annotations

import os
import threading
import weakref
from dataclasses import dataclass
from typing import Any

import numpy as np

ALIGN = 256
TAIL_SLACK = 64  # kernels read up to 64 bytes past a blob (include/zarrhip.h)

# Store.get_ranges defaults (src/zarr/core/config.py:104-105: sharding_coalesce_*)
MAX_GAP_BYTES = 1 << 20
MAX_COALESCED_BYTES = 16 << 20


@dataclass(frozen=True)
class RangeByteRequest:
    """src/zarr/abc/store.py RangeByteRequest: bytes [start, end)."""

    start: int
    end: int


@dataclass(frozen=True)
class SuffixByteRequest:
    """The last `suffix` bytes."""

    suffix: int


@dataclass(frozen=True)
class OffsetByteRequest:
    """Bytes from `offset` to the end."""

    offset: int


def _resolve_range(req, n: int) -> tuple[int, int]:
    """Byte request -> clamped [a, b) over a value of length n."""
    if req is None:
        return 0, n
    # by attribute, so zarr's own request classes (src/zarr/abc/store.py) work too
    if hasattr(req, "start") and hasattr(req, "end"):
        a, b = req.start, req.end
    elif hasattr(req, "suffix"):
        a, b = max(n - req.suffix, 0), n
    elif hasattr(req, "offset"):
        a, b = req.offset, n
    else:
        a, b = req
    a = min(max(int(a), 0), n)
    return a, min(max(int(b), a), n)


def coalesce_ranges(byte_ranges, *, max_gap_bytes: int = MAX_GAP_BYTES,
                    max_coalesced_bytes: int = MAX_COALESCED_BYTES):
    """Plan merged fetches (src/zarr/core/_coalesce.py:61-135): ranges sorted by
    start merge while the gap to the group's running end is <= max_gap_bytes
    and the merged span stays <= max_coalesced_bytes.  Returns
    (groups of [(input_index, RangeByteRequest)], uncoalescable [(i, req)])."""
    indexed = list(enumerate(byte_ranges))
    mergeable = [(i, r) for i, r in indexed if isinstance(r, RangeByteRequest)]
    other = [(i, r) for i, r in indexed if not isinstance(r, RangeByteRequest)]
    mergeable.sort(key=lambda pr: pr[1].start)
    groups: list = []
    g_start = g_end = 0
    for pr in mergeable:
        r = pr[1]
        if groups and r.start - g_end <= max_gap_bytes:
            new_end = max(g_end, r.end)
            if new_end - g_start <= max_coalesced_bytes:
                groups[-1].append(pr)
                g_end = new_end
                continue
        groups.append([pr])
        g_start, g_end = r.start, r.end
    return groups, other


class _RangesMixin:
    def get_ranges_sync(self, key: str, byte_ranges, *, prototype=None,
                        max_gap_bytes: int = MAX_GAP_BYTES,
                        max_coalesced_bytes: int = MAX_COALESCED_BYTES):
        """Store.get_ranges_sync (src/zarr/abc/store.py:474-539): one fetch per
        coalesced group, sliced back per input; yields (input_index, buf)."""
        groups, other = coalesce_ranges(byte_ranges, max_gap_bytes=max_gap_bytes,
                                        max_coalesced_bytes=max_coalesced_bytes)
        out = []
        for g in groups:
            a = g[0][1].start
            b = max(r.end for _, r in g)
            big = self.get_sync(key, RangeByteRequest(a, b))
            if big is None:
                raise FileNotFoundError(key)
            out.extend((i, big[r.start - a: r.end - a]) for i, r in g)
        for i, r in other:
            v = self.get_sync(key, r)
            if v is None:
                raise FileNotFoundError(key)
            out.append((i, v))
        return out


class MemoryStore(_RangesMixin):
    """Host dict store (MemoryStore restated)."""

    supports_sync_io = True

    def __init__(self, data: dict | None = None):
        self._d: dict[str, bytes] = {} if data is None else data

    def get_sync(self, key: str, byte_range=None, prototype=None):
        v = self._d.get(key)
        if v is None:
            return None
        if byte_range is None:
            return memoryview(v)
        a, b = _resolve_range(byte_range, len(v))
        return memoryview(v)[a:b]

    def set_sync(self, key: str, value) -> None:
        from .interop import byte_payload

        self._d[key] = value if isinstance(value, bytes) else byte_payload(value, host=True).tobytes()

    def delete_sync(self, key: str) -> None:
        self._d.pop(key, None)

    def exists(self, key: str) -> bool:
        return key in self._d

    def keys(self):
        return list(self._d.keys())

    def __contains__(self, key):
        return key in self._d

    def to_dict(self) -> dict[str, bytes]:
        return dict(self._d)


@dataclass(frozen=True)
class FileRef:
    """Bytes [offset, offset + length) of a file: what LocalStore.locate_sync
    returns so staging can pread them straight into pinned memory
    (ZHIP_PIECE_FILE) instead of reading them into Python bytes first."""

    path: str
    offset: int
    length: int

    def __len__(self):
        return self.length


class LocalStore(MemoryStore):
    """Files under a root directory (LocalStore restated, host side only)."""

    def __init__(self, root: str):
        super().__init__()
        self.root = root
        os.makedirs(root, exist_ok=True)

    def _path(self, key):
        return os.path.join(self.root, *key.split("/"))

    def get_sync(self, key, byte_range=None, prototype=None):
        p = self._path(key)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            if byte_range is None:
                return memoryview(f.read())
            a, b = _resolve_range(byte_range, os.fstat(f.fileno()).st_size)
            f.seek(a)
            return memoryview(f.read(b - a))

    def locate_sync(self, key, byte_range=None) -> FileRef | None:
        """Where get_sync's bytes are, without reading them (None: missing key)."""
        p = self._path(key)
        try:
            n = os.stat(p).st_size
        except FileNotFoundError:
            return None
        if byte_range is None:
            return FileRef(p, 0, n)
        a, b = _resolve_range(byte_range, n)
        return FileRef(p, a, b - a)

    def set_sync(self, key, value):
        from .interop import byte_payload

        p = self._path(key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(value if isinstance(value, bytes) else byte_payload(value, host=True).tobytes())

    def delete_sync(self, key):
        p = self._path(key)
        if os.path.exists(p):
            os.remove(p)

    def exists(self, key):
        return os.path.exists(self._path(key))

    def keys(self):
        out = []
        for dp, _, fs in os.walk(self.root):
            for f in fs:
                out.append(os.path.relpath(os.path.join(dp, f), self.root).replace(os.sep, "/"))
        return out

    def __contains__(self, key):
        return self.exists(key)

    def to_dict(self):
        return {k: bytes(self.get_sync(k)) for k in self.keys()}


def _aligned(n: int) -> int:
    return (int(n) + ALIGN - 1) // ALIGN * ALIGN


class DeviceArena:
    """A growable HBM byte arena (torch uint8 tensor) holding encoded blobs.

    Space is handed out in ALIGN-byte granules, first fit from a free list of
    released regions (kept sorted and coalesced), else from the top.  Deleting
    or overwriting a key gives its region back (the reference's MemoryStore /
    GpuMemoryStore drop the value on delete, src/zarr/storage/_memory.py:
    140-146, 317-328), so rewrite loops stay bounded.  Freed bytes are reused
    by work enqueued later on the same device stream, which orders it after
    every earlier reader.

    ``lock`` (re-entrant) serialises placement changes AND the enqueue of a
    device write into ``buf``: a writer holds it from reserve() until its encode
    is launched, so a concurrent grow (which swaps ``buf``) can never leave that
    launch writing into an abandoned buffer."""

    def __init__(self, device, capacity: int = 1 << 24, pinned: bool = False):
        import torch

        self.device = torch.device(device)
        self.pinned = pinned and self.device.type == "cpu"
        self.buf = self._alloc(_aligned(capacity) + TAIL_SLACK)
        self.top = 0
        self.version = 0
        # placement generation: bumped by every reserve / free / grow, so a read
        # planned against these offsets (a DecodeProgram, a ReadGraph, the
        # pipeline's per-call plan cache) can tell that a key it reads may have
        # moved or been reused (freed regions are handed out again at once)
        self.gen = 0
        self.lock = threading.RLock()
        self._free: list[list[int]] = []  # [offset, nbytes], sorted, coalesced, ALIGN granules

    def _alloc(self, n: int):
        import torch

        if self.pinned:
            return torch.empty(n, dtype=torch.uint8, pin_memory=True)
        return torch.empty(n, dtype=torch.uint8, device=self.device)

    @property
    def capacity(self) -> int:
        return self.buf.numel() - TAIL_SLACK

    @property
    def free_bytes(self) -> int:
        return sum(n for _, n in self._free)

    @property
    def used_bytes(self) -> int:
        return self.top - self.free_bytes

    def _grow(self, need: int) -> None:
        import torch

        cap = _aligned(max(need, 2 * self.capacity))
        nb = self._alloc(cap + TAIL_SLACK)
        nb[: self.top].copy_(self.buf[: self.top])
        self.buf = nb
        self.version += 1
        self.gen += 1

    def reserve(self, nbytes: int) -> int:
        """Reserve an aligned region of at least nbytes; returns its offset."""
        need = max(_aligned(nbytes), ALIGN)
        with self.lock:
            self.gen += 1
            for i, (off, n) in enumerate(self._free):
                if n >= need:
                    if n == need:
                        del self._free[i]
                    else:
                        self._free[i] = [off + need, n - need]
                    return off
            off = self.top
            end = off + need
            if end > self.capacity:
                self._grow(end)
            self.top = end
            return off

    def free(self, off: int, nbytes: int) -> None:
        """Give back a region returned by reserve() (or its aligned tail)."""
        off = int(off)
        n = _aligned(nbytes)
        if n <= 0:
            return
        with self.lock:
            self.gen += 1
            fl = self._free
            lo, hi = 0, len(fl)
            while lo < hi:
                mid = (lo + hi) // 2
                if fl[mid][0] < off:
                    lo = mid + 1
                else:
                    hi = mid
            fl.insert(lo, [off, n])
            # coalesce with the neighbours
            if lo + 1 < len(fl) and fl[lo][0] + fl[lo][1] == fl[lo + 1][0]:
                fl[lo][1] += fl[lo + 1][1]
                del fl[lo + 1]
            if lo > 0 and fl[lo - 1][0] + fl[lo - 1][1] == fl[lo][0]:
                fl[lo - 1][1] += fl[lo][1]
                del fl[lo]
                lo -= 1
            # a free block that reaches the top lowers it
            if fl and fl[-1][0] + fl[-1][1] == self.top:
                self.top = fl[-1][0]
                del fl[-1]

    def put(self, data) -> tuple[int, int]:
        """Copy host bytes / numpy / device tensor into the arena."""
        import torch

        if isinstance(data, torch.Tensor):
            t = data.reshape(-1).view(torch.uint8)
            with self.lock:
                off = self.reserve(t.numel())
                self.buf[off: off + t.numel()].copy_(t, non_blocking=True)
            return off, t.numel()
        if self.device.type == "cpu":
            arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
                else np.ascontiguousarray(data).reshape(-1).view(np.uint8)
            with self.lock:
                off = self.reserve(arr.size)
                self.buf[off: off + arr.size].numpy()[:] = arr
            return off, int(arr.size)
        arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) \
            else np.ascontiguousarray(data).reshape(-1).view(np.uint8)
        with self.lock:
            off = self.reserve(arr.size)
            if arr.size:
                self.buf[off: off + arr.size].copy_(torch.from_numpy(arr.copy()))
        return off, int(arr.size)

    def view(self, off: int, n: int):
        return self.buf[off: off + n]


@dataclass
class DeviceRef:
    """A ByteGetter result that stays on the device: (arena, offset, length)."""

    arena: DeviceArena
    offset: int
    length: int

    def __len__(self):
        return self.length

    def to_bytes(self) -> bytes:
        return self.arena.view(self.offset, self.length).cpu().numpy().tobytes()


class DeviceStore:
    """Key -> blob placements in one DeviceArena (HBM-resident chunk store)."""

    supports_sync_io = True

    def __init__(self, device="cuda:0", capacity: int = 1 << 24):
        self.arena = DeviceArena(device, capacity)
        self._index: dict[str, tuple[int, int]] = {}
        self._meta: dict[str, bytes] = {}  # zarr.json documents stay on the host

    @property
    def device(self):
        return self.arena.device

    def get_sync(self, key: str, byte_range=None, prototype=None) -> DeviceRef | None:
        if key.endswith("zarr.json"):
            m = self._meta.get(key)
            return None if m is None else memoryview(m)
        v = self._index.get(key)
        if v is None:
            return None
        off, n = v
        if byte_range is not None:
            a, b = _resolve_range(byte_range, n)
            return DeviceRef(self.arena, off + a, b - a)
        return DeviceRef(self.arena, off, n)

    def set_sync(self, key: str, value: Any, *, byte_range=None) -> None:
        from .interop import byte_payload

        if key.endswith("zarr.json"):
            self._meta[key] = bytes(byte_payload(value, host=True))
            return
        if isinstance(value, DeviceRef):
            value = value.arena.view(value.offset, value.length)
        else:
            value = byte_payload(value)
        with self.arena.lock:
            placed = self.arena.put(value)
            self._release(key)
            self._index[key] = placed

    def set_reserved(self, key: str, nbytes: int) -> int:
        with self.arena.lock:
            off = self.arena.reserve(nbytes)
            self._release(key)
            self._index[key] = (off, nbytes)
        return off

    def _release(self, key: str) -> None:
        old = self._index.pop(key, None)
        if old is not None:
            self.arena.free(old[0], max(old[1], 1))

    def register(self, key: str, off: int, nbytes: int) -> None:
        """Bind a key to bytes already written in the arena (device encode output);
        the key's previous region goes back to the arena."""
        with self.arena.lock:
            self._release(key)
            self._index[key] = (int(off), int(nbytes))

    def commit(self, key: str, off: int, nbytes: int, reserved: int) -> None:
        """register() for a region of `reserved` bytes of which the encode used
        `nbytes` (0 = the chunk / shard was elided: the key is deleted); the
        unused aligned tail goes back to the arena."""
        with self.arena.lock:
            if nbytes <= 0:
                self._release(key)
                self.arena.free(off, max(reserved, 1))
                return
            used = -(-int(nbytes) // ALIGN) * ALIGN
            tail = -(-int(reserved) // ALIGN) * ALIGN - used
            if tail > 0:
                self.arena.free(int(off) + used, tail)
            self._release(key)
            self._index[key] = (int(off), int(nbytes))

    def delete_sync(self, key: str) -> None:
        with self.arena.lock:
            self._release(key)

    def exists(self, key: str) -> bool:
        return key in self._index

    def __contains__(self, key):
        return key in self._index

    def keys(self):
        return list(self._index.keys())

    def placement(self, key: str) -> tuple[int, int] | None:
        return self._index.get(key)

    def to_dict(self) -> dict[str, bytes]:
        host = self.arena.buf[: self.arena.top].cpu().numpy()
        d = {k: host[o: o + n].tobytes() for k, (o, n) in self._index.items()}
        d.update(self._meta)
        return d

    @classmethod
    def from_host(cls, data: dict, device="cuda:0") -> "DeviceStore":
        total = sum((len(v) + ALIGN) for v in data.values()) + ALIGN
        st = cls(device, capacity=max(total, 1 << 16))
        host = np.zeros(total, dtype=np.uint8)
        placements = {}
        top = 0
        for k, v in data.items():
            if k.endswith("zarr.json"):
                st._meta[k] = bytes(v)
                continue
            b = np.frombuffer(bytes(v), dtype=np.uint8)
            placements[k] = (top, b.size)
            host[top: top + b.size] = b
            top = (top + b.size + ALIGN - 1) // ALIGN * ALIGN
        import torch

        st.arena.buf[:top].copy_(torch.from_numpy(host[:top]))
        st.arena.top = top
        st._index = placements
        return st


_PINNED_ARENAS: "weakref.WeakSet[DeviceArena]" = weakref.WeakSet()


def pinned_spans() -> list[tuple[int, int]]:
    """Host address spans of the live pinned store arenas.  Staged pieces
    inside one are DMA'd to HBM directly (ZHIP_PIECE_PINNED), never packed."""
    return [(a.buf.data_ptr(), a.buf.data_ptr() + a.buf.numel()) for a in list(_PINNED_ARENAS)]


class PinnedMemoryStore(MemoryStore):
    """A MemoryStore whose values live in page-locked host memory: one pinned
    arena (DeviceArena on "cpu", same first-fit free list), so a read stages
    its chunk bytes to HBM by DMA straight from the store -- no packing copy --
    and consecutive values go as one copy (csrc/staging.cpp).  Same store
    interface as MemoryStore (src/zarr/storage/_memory.py:32-170); get_sync
    returns uint8 numpy views of the arena.  A value's bytes change only when
    its key is overwritten or deleted, which first waits for the staging copy
    streams so no DMA in flight reads reused space."""

    def __init__(self, data: dict | None = None, capacity: int = 1 << 24):
        self.arena = DeviceArena("cpu", capacity, pinned=True)
        _PINNED_ARENAS.add(self.arena)
        self._d: dict[str, tuple[int, int]] = {}
        self._np, self._np_of = None, None
        for k, v in (data or {}).items():
            self.set_sync(k, v)

    def get_sync(self, key: str, byte_range=None, prototype=None):
        p = self._d.get(key)
        if p is None:
            return None
        off, n = p
        a, b = (0, n) if byte_range is None else _resolve_range(byte_range, n)
        buf = self.arena.buf
        if self._np_of is not buf:  # numpy alias of the (possibly regrown) arena
            self._np, self._np_of = buf.numpy(), buf
        return self._np[off + a: off + b]

    def _release(self, key: str) -> None:
        p = self._d.pop(key, None)
        if p is not None:
            from .staging import quiesce

            quiesce()
            self.arena.free(*p)

    def set_sync(self, key: str, value) -> None:
        from .interop import byte_payload

        data = value if isinstance(value, (bytes, bytearray, memoryview, np.ndarray)) else \
            byte_payload(value, host=True)
        with self.arena.lock:
            self._release(key)
            self._d[key] = self.arena.put(data)

    def delete_sync(self, key: str) -> None:
        with self.arena.lock:
            self._release(key)

    def to_dict(self) -> dict[str, bytes]:
        return {k: self.arena.buf[o: o + n].numpy().tobytes() for k, (o, n) in self._d.items()}


@dataclass(frozen=True)
class StorePath:
    """store + key: the reference's ByteGetter / ByteSetter (storage/_common.py)."""

    store: Any
    path: str

    def get_sync(self, prototype=None, byte_range=None):
        return self.store.get_sync(self.path, byte_range)

    def set_sync(self, value) -> None:
        self.store.set_sync(self.path, value)

    def delete_sync(self) -> None:
        self.store.delete_sync(self.path)

    async def get(self, prototype=None, byte_range=None):
        return self.get_sync(prototype, byte_range)

    async def set(self, value, byte_range=None):
        self.set_sync(value)

    async def delete(self):
        self.delete_sync()

    def __truediv__(self, other: str) -> "StorePath":
        return StorePath(self.store, f"{self.path}/{other}" if self.path else other)

"""The host stage of a codec chain: compression (and whatever follows it) runs
on the host, the fixed-size remainder on the GPU.

The north star keeps compression codecs on the host, outside the timed GPU
path.  A v3 chain ``AA* -> AB -> BB*`` splits at the first host codec
(codecs.split_host_tail): e.g. zarr's default ``[bytes, zstd]`` is GPU
``[bytes]`` + host ``[zstd]``; ``[bytes, crc32c, gzip]`` is GPU ``[bytes,
crc32c]`` + host ``[gzip]``; ``[bytes, gzip, crc32c]`` keeps the crc32c on the
host, where it checks the compressed bytes as the reference's chain order
does (ChunkTransform.decode_chunk, src/zarr/core/chunk_utils.py:304-333).  A
sharding codec's inner chain splits the same way: the shard index and the
fixed-size inner decode stay on the GPU, each touched inner chunk is
decompressed on the host first (ShardingCodec._decode_partial_sync,
src/zarr/codecs/sharding.py:1222-1309, with the inner pipeline's BB stage).

Reads: host bytes -> host stage (thread pool; zlib / zstd / blosc release the
GIL) -> fixed-size bytes staged to HBM -> GPU decode + scatter.
Writes: GPU encode of the fixed-size chain into a collector -> host stage ->
store.  For sharded chains with an inner host stage the GPU writes its fixed
shard layout and ``ShardTranscoder`` re-packs it with the compressed inner
chunks (same physical order, new offsets, index re-encoded with the host
CRC-32C), and the reverse for a read-modify-write.
"""

from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N
from .codecs import Crc32cCodec, ShardingCodec, is_host_codec
from .interop import byte_payload, is_own_store, wrap_for_setter
from .spec import ArraySpec
from .store import _resolve_range

MAX_U64 = np.uint64(0xFFFFFFFFFFFFFFFF)

_POOL: ThreadPoolExecutor | None = None


def _pool() -> ThreadPoolExecutor:
    global _POOL
    if _POOL is None:
        n = os.cpu_count() or 1
        cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        _POOL = ThreadPoolExecutor(max_workers=max(1, min(n, cap or 16, 16)),
                                   thread_name_prefix="zarr_hip_host_stage")
    return _POOL


def crc_message(stored: bytes, computed: bytes) -> str:
    """src/zarr/codecs/crc32c_.py:46-49."""
    return f"Stored and computed checksum do not match. Stored: {stored!r}. Computed: {computed!r}."


def host_crc32c(data) -> int:
    a = data if isinstance(data, np.ndarray) else np.frombuffer(bytes(data), np.uint8)
    a = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    return int(N.lib().zhip_crc32c_host(a.ctypes.data if a.size else None, a.size))


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).reshape(-1).view(np.uint8)
    return np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else \
        byte_payload(data, host=True)


def decode_tail(data, tail: tuple, spec: ArraySpec | None) -> bytes:
    """Undo a host stage (reverse order, chunk_utils.py:315-320)."""
    b = data
    for c in reversed(tail):
        if isinstance(c, Crc32cCodec):  # crc32c_.py:34-50, on the host's bytes
            u = _as_u8(b)
            if u.size < 4:
                raise ValueError("chunk shorter than its crc32c trailer")
            stored = u[-4:].tobytes()
            computed = np.uint32(host_crc32c(u[:-4])).tobytes()
            if stored != computed:
                raise ValueError(crc_message(stored, computed))
            b = u[:-4]
        elif is_host_codec(c):
            b = c.decode_bytes(_as_u8(b), spec)
        else:
            raise NotImplementedError(f"{type(c).__name__} in a host stage")
    return bytes(b) if not isinstance(b, bytes) else b


def encode_tail(data, tail: tuple, spec: ArraySpec | None) -> bytes:
    """Apply a host stage (chunk_utils.py:352-363)."""
    b = data
    for c in tail:
        if isinstance(c, Crc32cCodec):  # crc32c_.py:59-68
            u = _as_u8(b)
            b = u.tobytes() + np.uint32(host_crc32c(u)).tobytes()
        elif is_host_codec(c):
            b = c.encode_bytes(_as_u8(b), spec)
        else:
            raise NotImplementedError(f"{type(c).__name__} in a host stage")
    return bytes(b) if not isinstance(b, bytes) else b


def map_host(fn, items: list) -> list:
    """fn over items on the host-stage pool (in order); small batches inline.
    Items go to the pool in runs (about four per thread), not one future per
    item: thousands of small inner chunks would otherwise spend as long in
    the executor's bookkeeping as in zlib."""
    n = len(items)
    if n <= 1:
        return [fn(x) for x in items]
    pool = _pool()
    per = max(1, -(-n // (4 * pool._max_workers)))
    if per == 1:
        return list(pool.map(fn, items))
    runs = [items[i: i + per] for i in range(0, n, per)]
    out: list = []
    for part in pool.map(lambda run: [fn(x) for x in run], runs):
        out.extend(part)
    return out


def decode_many(raws: list, tail: tuple, spec: ArraySpec | None) -> list:
    return map_host(lambda r: None if r is None else decode_tail(r, tail, spec), raws)


# ------------------------------------------------------------ shard transcoding
class ShardTranscoder:
    """A shard blob between its stored form (inner chunks through the inner
    host stage, e.g. compressed) and the fixed form the GPU writes and reads
    (the inner chain's GPU part only).  Physical inner-chunk order is kept, so
    the subchunk write order the GPU packer chose (sharding.py:1090-1107)
    survives; offsets are re-derived and the index re-encoded
    (_build_shard_layout / _assemble_shard / _encode_shard_index_sync,
    sharding.py:633-640, 887-950)."""

    def __init__(self, sharding: ShardingCodec, shard_shape, inner_tail: tuple, spec: ArraySpec | None):
        self.sh = sharding
        self.cps = sharding.chunks_per_shard(tuple(shard_shape))
        self.n = int(np.prod(self.cps))
        self.index_size = sharding.shard_index_size(self.n)
        self.at_start = sharding.index_location == "start"
        self.crc = sharding.index_has_crc
        self.tail = tuple(inner_tail)
        self.spec = spec

    def read_index(self, blob: np.ndarray) -> np.ndarray:
        """_decode_shard_index_sync (sharding.py:624-631), CRC checked on the host."""
        if blob.size < self.index_size:
            raise ValueError("shard blob is shorter than its index")
        raw = blob[: self.index_size] if self.at_start else blob[blob.size - self.index_size:]
        if self.crc:
            stored = raw[-4:].tobytes()
            computed = np.uint32(host_crc32c(raw[:-4])).tobytes()
            if stored != computed:
                raise ValueError(crc_message(stored, computed))
        return raw[: 16 * self.n].view("<u8").reshape(self.n, 2).copy()

    def write_index(self, idx: np.ndarray) -> bytes:
        b = np.ascontiguousarray(idx, dtype="<u8").tobytes()
        if self.crc:
            b += np.uint32(host_crc32c(b)).tobytes()
        return b

    def _map(self, blob, fn) -> bytes:
        u = _as_u8(blob)
        idx = self.read_index(u)
        present = np.nonzero(~((idx[:, 0] == MAX_U64) & (idx[:, 1] == MAX_U64)))[0]
        order = present[np.argsort(idx[present, 0], kind="stable")]  # physical order
        pieces = map_host(lambda s: fn(u[int(idx[s, 0]): int(idx[s, 0]) + int(idx[s, 1])]), list(order))
        new = np.full((self.n, 2), MAX_U64, np.uint64)
        at = self.index_size if self.at_start else 0
        for s, p in zip(order, pieces):
            new[s] = (at, len(p))
            at += len(p)
        ib = self.write_index(new)
        body = b"".join(pieces)
        return ib + body if self.at_start else body + ib

    def to_fixed(self, blob) -> bytes:
        return self._map(blob, lambda b: decode_tail(b, self.tail, self.spec))

    def to_stored(self, blob) -> bytes:
        return self._map(blob, lambda b: encode_tail(b, self.tail, self.spec))


class TranscodingByteSetter:
    """A chunk's ByteGetter / ByteSetter seen through the host stage: the GPU
    writer reads and writes fixed-size bytes, the store holds the stored form.
    ``outer``: the chain's own host stage; ``shard``: a ShardTranscoder when a
    sharding codec's inner chain has one (applied inside the outer stage)."""

    def __init__(self, inner, outer: tuple, shard: ShardTranscoder | None, spec: ArraySpec):
        self.inner = inner
        self.outer = tuple(outer)
        self.shard = shard
        self.spec = spec

    @property
    def path(self):
        return getattr(self.inner, "path", None)

    def get_sync(self, prototype=None, byte_range=None):
        raw = self.inner.get_sync(prototype=prototype)
        if raw is None:
            return None
        b = _as_u8(raw)
        if self.outer:
            b = decode_tail(b, self.outer, self.spec)
        if self.shard is not None:
            b = self.shard.to_fixed(b)
        b = bytes(b) if not isinstance(b, bytes) else b
        if byte_range is None:
            return b
        a, e = _resolve_range(byte_range, len(b))
        return memoryview(b)[a:e]

    def set_sync(self, value) -> None:
        b = byte_payload(value, host=True)
        if self.shard is not None:
            b = self.shard.to_stored(b)
        if self.outer:
            b = encode_tail(b, self.outer, self.spec)
        b = bytes(b) if not isinstance(b, bytes) else b
        st = getattr(self.inner, "store", None)
        self.inner.set_sync(b if is_own_store(st) else wrap_for_setter(b, self.spec.prototype))

    def delete_sync(self) -> None:
        self.inner.delete_sync()

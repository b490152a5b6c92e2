"""ORACLE — CPU restatement of zarr-python's fixed-size codec chain.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / CPU baseline.  The product (``zarr-python_amd/zarr_hip``) never
imports it; its decode/encode runs on the GPU through the HIP C-ABI library.

Every function restates a reference function (file:line under
/root/reference) using plain numpy.  The reference itself cannot be imported
in this container (Python 3.10 here, zarr needs >= 3.12 and PEP 695 syntax;
google-crc32c / donfig / numcodecs absent — SURVEY.md §8c), so parity is
pinned by:
  * published CRC-32C known-answer vectors (RFC 3720 B.4, "123456789"),
    checked against three independent C implementations (crc32c_oracle.c);
  * the literal Morton-order vectors of tests/test_codecs/test_codecs.py:175-206;
  * the stored-bytes property of tests/test_codecs/test_bytes.py:90,136
    (stored == data.astype(dtype.newbyteorder(endian)).tobytes());
  * the +4 encoded-size rule (tests/test_chunk_transform.py:118-135);
  * the ShardIndex semantics of tests/test_codecs/test_sharding_unit.py:45-170.
"""

from __future__ import annotations

import ctypes
import itertools
import math
import os
from dataclasses import dataclass, field
from typing import Any

import numpy as np

MAX_UINT_64 = 2**64 - 1  # src/zarr/codecs/sharding.py:85

# ---------------------------------------------------------------------------
# CRC-32C (google_crc32c.value, called at src/zarr/codecs/crc32c_.py:44,66)
# ---------------------------------------------------------------------------

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def _load_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = ctypes.CDLL(_LIB_PATH)
        for name in ("oracle_crc32c_bitwise", "oracle_crc32c_slice8", "oracle_crc32c_hw"):
            fn = getattr(lib, name)
            fn.restype = ctypes.c_uint32
            fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        lib.oracle_crc32c.restype = ctypes.c_uint32
        lib.oracle_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_crc32c_many.restype = None
        lib.oracle_crc32c_many.argtypes = [
            ctypes.c_void_p,
            ctypes.c_void_p,
            ctypes.c_void_p,
            ctypes.c_uint64,
        ]
        lib.oracle_has_hw_crc.restype = ctypes.c_int
        _lib = lib
    return _lib


def _as_u8(data: Any) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    arr = np.ascontiguousarray(data)
    return arr.reshape(-1).view(np.uint8)


def crc32c(data: Any, impl: str = "hw") -> int:
    """CRC-32C of ``data`` (reflected 0x82F63B78, init/xorout 0xFFFFFFFF)."""
    u8 = _as_u8(data)
    fn = {
        "hw": _load_lib().oracle_crc32c_hw,
        "slice8": _load_lib().oracle_crc32c_slice8,
        "bitwise": _load_lib().oracle_crc32c_bitwise,
    }[impl]
    return int(fn(u8.ctypes.data if u8.size else None, u8.size, 0))


def crc32c_pure_python(data: bytes) -> int:
    """Fourth, dependency-free statement of the definition (tiny inputs only)."""
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


# ---------------------------------------------------------------------------
# Codecs
# ---------------------------------------------------------------------------


def crc32c_decode(chunk_bytes: np.ndarray) -> np.ndarray:
    """Crc32cCodec._decode_sync (src/zarr/codecs/crc32c_.py:34-50)."""
    data = _as_u8(chunk_bytes)
    crc32_bytes = data[-4:]
    inner_bytes = data[:-4]
    computed_checksum = np.uint32(crc32c(inner_bytes)).tobytes()
    stored_checksum = bytes(crc32_bytes)
    if computed_checksum != stored_checksum:
        raise ValueError(
            f"Stored and computed checksum do not match. Stored: {stored_checksum!r}. "
            f"Computed: {computed_checksum!r}."
        )
    return inner_bytes


def crc32c_encode(chunk_bytes: np.ndarray) -> np.ndarray:
    """Crc32cCodec._encode_sync (crc32c_.py:59-68): append the LE uint32 CRC."""
    data = _as_u8(chunk_bytes)
    checksum = np.array([crc32c(data)], dtype=np.uint32)
    return np.append(data, checksum.view("B"))


def gzip_decode(chunk_bytes: np.ndarray) -> np.ndarray:
    """GzipCodec._decode_sync (src/zarr/codecs/gzip.py:56-61) -> numcodecs.GZip.decode
    (numcodecs 0.16, not vendored under /root/reference): a gzip member, else a
    raw zlib stream; restated over the stdlib."""
    import gzip
    import zlib

    b = _as_u8(chunk_bytes).tobytes()
    out = gzip.decompress(b) if b[:2] == b"\x1f\x8b" else zlib.decompress(b)
    return np.frombuffer(out, dtype=np.uint8)


def gzip_encode(chunk_bytes: np.ndarray, level: int) -> np.ndarray:
    """GzipCodec._encode_sync (gzip.py:70-75) -> numcodecs.GZip.encode: one gzip
    member written by GzipFile at `level` with mtime 0 (byte identity with
    numcodecs' header is unpinned here: numcodecs is absent; the round trip and
    the decode of any valid member are what the tests rely on)."""
    import gzip

    return np.frombuffer(gzip.compress(_as_u8(chunk_bytes).tobytes(), compresslevel=level, mtime=0),
                         dtype=np.uint8)


def _stored_dtype(dtype: np.dtype, endian: str | None) -> np.dtype:
    if dtype.itemsize == 1 or endian is None:
        return dtype
    return dtype.newbyteorder("<" if endian == "little" else ">")


def bytes_decode(chunk_bytes: np.ndarray, shape: tuple[int, ...], dtype: np.dtype,
                 endian: str | None) -> np.ndarray:
    """BytesCodec._decode_sync (src/zarr/codecs/bytes.py:97-131)."""
    view_dtype = _stored_dtype(np.dtype(dtype), endian)
    arr = _as_u8(chunk_bytes).view(view_dtype)
    if view_dtype != np.dtype(dtype):
        arr = arr.astype(dtype)  # the byte-swapping copy (bytes.py:123-127)
    return arr.reshape(shape)


def bytes_encode(chunk_array: np.ndarray, endian: str | None) -> np.ndarray:
    """BytesCodec._encode_sync (bytes.py:140-158)."""
    if chunk_array.dtype.itemsize > 1 and endian is not None:
        new_dtype = chunk_array.dtype.newbyteorder("<" if endian == "little" else ">")
        if new_dtype != chunk_array.dtype:
            chunk_array = chunk_array.astype(new_dtype)
    return np.ascontiguousarray(chunk_array).ravel().view("B")


def transpose_resolve_shape(shape: tuple[int, ...], order: tuple[int, ...]) -> tuple[int, ...]:
    """TransposeCodec.resolve_metadata (src/zarr/codecs/transpose.py:89-96)."""
    return tuple(shape[order[i]] for i in range(len(shape)))


def transpose_decode(arr: np.ndarray, order: tuple[int, ...]) -> np.ndarray:
    """TransposeCodec._decode_sync (transpose.py:98-104): inverse permutation view."""
    inverse_order = tuple(int(i) for i in np.argsort(order))
    return arr.transpose(inverse_order)


def transpose_encode(arr: np.ndarray, order: tuple[int, ...]) -> np.ndarray:
    """TransposeCodec._encode_sync (transpose.py:113-118)."""
    return arr.transpose(order)


# ---------------------------------------------------------------------------
# Codec chain description (restates the JSON forms of zarr.json "codecs")
# ---------------------------------------------------------------------------


@dataclass
class Chain:
    """A v3 codec list split as codecs_from_list does (codec_pipeline.py:859-944).

    aa: transpose orders (ArrayArray), ab: ("bytes", endian) or ("sharding", ShardSpec),
    bb: "crc32c" or ("gzip", level) entries (BytesBytes), in chain order.
    """

    aa: tuple[tuple[int, ...], ...] = ()
    endian: str | None = "little"
    bb: tuple[str, ...] = ()
    shard: "ShardSpec | None" = None

    @staticmethod
    def from_json(codecs: list[dict]) -> "Chain":
        aa: list[tuple[int, ...]] = []
        endian: str | None = None
        bb: list[str] = []
        shard = None
        for c in codecs:
            name = c["name"] if isinstance(c, dict) else c
            conf = c.get("configuration", {}) if isinstance(c, dict) else {}
            if name == "transpose":
                aa.append(tuple(conf["order"]))
            elif name == "bytes":
                endian = conf.get("endian")
            elif name == "crc32c":
                bb.append("crc32c")
            elif name == "gzip":
                bb.append(("gzip", int(conf.get("level", 5))))
            elif name == "sharding_indexed":
                shard = ShardSpec(
                    chunk_shape=tuple(conf["chunk_shape"]),
                    inner=Chain.from_json(conf.get("codecs", [{"name": "bytes"}])),
                    index=Chain.from_json(conf.get(
                        "index_codecs", [{"name": "bytes"}, {"name": "crc32c"}])),
                    index_location=conf.get("index_location", "end"),
                    # not part of the stored metadata (sharding.py:462-464); accepted
                    # here so tests can pick the physical layout a writer uses
                    subchunk_write_order=conf.get("subchunk_write_order", "morton"),
                )
            else:
                raise NotImplementedError(name)
        return Chain(tuple(aa), endian, tuple(bb), shard)


@dataclass
class ShardSpec:
    chunk_shape: tuple[int, ...]
    inner: Chain
    index: Chain
    index_location: str = "end"
    subchunk_write_order: str = "morton"


@dataclass
class Spec:
    """ArraySpec (src/zarr/core/array_spec.py:40-186) restated."""

    shape: tuple[int, ...]
    dtype: np.dtype
    fill_value: Any
    write_empty_chunks: bool = False
    order: str = "C"


def chain_decode(chunk_bytes: np.ndarray, chain: Chain, spec: Spec) -> np.ndarray:
    """ChunkTransform.decode_chunk (src/zarr/core/chunk_utils.py:304-333)."""
    # resolve_aa_specs (codec_pipeline.py:116-140): thread the shape forward
    shapes = []
    shape = spec.shape
    for order in chain.aa:
        shapes.append(shape)
        shape = transpose_resolve_shape(shape, order)
    data = _as_u8(chunk_bytes)
    for name in reversed(chain.bb):
        if name == "crc32c":
            data = crc32c_decode(data)
        else:
            assert name[0] == "gzip"
            data = gzip_decode(data)
    if chain.shard is not None:
        arr = shard_decode(data, chain.shard, Spec(shape, spec.dtype, spec.fill_value,
                                                    spec.write_empty_chunks, spec.order))
    else:
        arr = bytes_decode(data, shape, spec.dtype, chain.endian)
    for order in reversed(chain.aa):
        arr = transpose_decode(arr, order)
    return arr


def chain_encode(chunk_array: np.ndarray, chain: Chain, spec: Spec) -> np.ndarray | None:
    """ChunkTransform.encode_chunk (chunk_utils.py:335-363)."""
    arr = chunk_array
    shape = spec.shape
    for order in chain.aa:
        arr = transpose_encode(arr, order)
        shape = transpose_resolve_shape(shape, order)
    if chain.shard is not None:
        data = shard_encode(arr, chain.shard, Spec(shape, spec.dtype, spec.fill_value,
                                                    spec.write_empty_chunks, spec.order))
        if data is None:
            return None
    else:
        data = bytes_encode(arr, chain.endian)
    for name in chain.bb:
        data = crc32c_encode(data) if name == "crc32c" else gzip_encode(data, name[1])
    return data


def chain_encoded_size(nbytes: int, chain: Chain) -> int:
    """compute_encoded_size: bytes +0, crc32c +4 (crc32c_.py:77-78); gzip has
    none (gzip.py:89-95)."""
    if any(name != "crc32c" for name in chain.bb):
        raise NotImplementedError("gzip output is not fixed-size")
    return nbytes + 4 * len(chain.bb)


# ---------------------------------------------------------------------------
# Morton order (src/zarr/core/indexing.py:1524-1643)
# ---------------------------------------------------------------------------


def decode_morton(z: int, chunk_shape: tuple[int, ...]) -> tuple[int, ...]:
    """indexing.py:1524-1539."""
    bits = tuple((c - 1).bit_length() for c in chunk_shape)
    max_coords_bits = max(bits) if bits else 0
    input_bit = 0
    out = [0] * len(chunk_shape)
    for coord_bit in range(max_coords_bits):
        for dim in range(len(chunk_shape)):
            if coord_bit < bits[dim]:
                bit = (z >> input_bit) & 1
                out[dim] |= bit << coord_bit
                input_bit += 1
    return tuple(out)


def morton_order_coords(shape: tuple[int, ...]) -> list[tuple[int, ...]]:
    """_morton_order / morton_order_coords (indexing.py:1578-1643): the Morton codes of
    the ceiling power-of-two hypercube, in code order, filtered to in-bounds coords.
    (The reference's argsort strategy produces the same order: stable sort by code.)"""
    n_total = math.prod(shape)
    if n_total == 0:
        return []
    total_bits = sum((c - 1).bit_length() for c in shape)
    out = []
    for z in range(1 << total_bits):
        c = decode_morton(z, shape)
        if all(ci < si for ci, si in zip(c, shape)):
            out.append(c)
    return out


def lexicographic_order_coords(shape: tuple[int, ...]) -> list[tuple[int, ...]]:
    return list(itertools.product(*(range(s) for s in shape)))


def colexicographic_order_coords(shape: tuple[int, ...]) -> list[tuple[int, ...]]:
    return [c[::-1] for c in lexicographic_order_coords(shape[::-1])]


def subchunk_order(shape: tuple[int, ...], order: str) -> list[tuple[int, ...]]:
    """ShardingCodec._subchunk_order_iter (sharding.py:1090-1107)."""
    if order == "morton":
        return morton_order_coords(shape)
    if order in ("lexicographic", "unordered"):
        return lexicographic_order_coords(shape)
    if order == "colexicographic":
        return colexicographic_order_coords(shape)
    raise ValueError(order)


# ---------------------------------------------------------------------------
# Sharding (src/zarr/codecs/sharding.py)
# ---------------------------------------------------------------------------


def shard_index_size(n_inner: int, index_chain: Chain) -> int:
    """_shard_index_size (sharding.py:1515-1522): 16 * prod(cps) + 4 per crc."""
    return chain_encoded_size(16 * n_inner, index_chain)


def decode_shard_index(index_bytes: np.ndarray, cps: tuple[int, ...], index_chain: Chain):
    """_decode_shard_index_sync (sharding.py:624-631) with the index spec of
    _get_index_chunk_spec (1524-1533): shape cps+(2,), uint64 little."""
    spec = Spec(tuple(cps) + (2,), np.dtype("<u8"), MAX_UINT_64)
    return chain_decode(index_bytes, index_chain, spec)


def encode_shard_index(offsets_and_lengths: np.ndarray, index_chain: Chain) -> np.ndarray:
    """_encode_shard_index_sync (sharding.py:633-640)."""
    spec = Spec(offsets_and_lengths.shape, np.dtype("<u8"), MAX_UINT_64)
    return chain_encode(offsets_and_lengths.astype("<u8"), index_chain, spec)


def _cps(shard_spec: Spec, sh: ShardSpec) -> tuple[int, ...]:
    """_get_chunks_per_shard (sharding.py:1544-1552)."""
    return tuple(s // c for s, c in zip(shard_spec.shape, sh.chunk_shape))


def shard_reader(blob: np.ndarray, sh: ShardSpec, cps: tuple[int, ...]):
    """_shard_reader_from_bytes_sync (sharding.py:642-655) -> dict coords->bytes|None."""
    size = shard_index_size(math.prod(cps), sh.index)
    blob = _as_u8(blob)
    index_bytes = blob[:size] if sh.index_location == "start" else blob[-size:]
    index = decode_shard_index(index_bytes, cps, sh.index)
    out: dict[tuple[int, ...], np.ndarray | None] = {}
    for coords in lexicographic_order_coords(cps):
        off, ln = (int(v) for v in index[coords])
        if (off, ln) == (MAX_UINT_64, MAX_UINT_64):
            out[coords] = None  # _ShardIndex.get_chunk_slice (248-254)
        else:
            out[coords] = blob[off: off + ln]
    return out


def shard_decode(blob: np.ndarray, sh: ShardSpec, shard_spec: Spec) -> np.ndarray:
    """ShardingCodec._decode_sync (sharding.py:657-714)."""
    cps = _cps(shard_spec, sh)
    inner_spec = Spec(sh.chunk_shape, shard_spec.dtype, shard_spec.fill_value,
                      shard_spec.write_empty_chunks, shard_spec.order)
    out = np.empty(shard_spec.shape, dtype=shard_spec.dtype)
    chunks = shard_reader(blob, sh, cps)
    if all(v is None for v in chunks.values()):
        out.fill(shard_spec.fill_value)
        return out
    for coords in lexicographic_order_coords(cps):
        sel = tuple(slice(c * s, (c + 1) * s) for c, s in zip(coords, sh.chunk_shape))
        raw = chunks[coords]
        if raw is None:
            out[sel] = shard_spec.fill_value  # missing inner -> fill, never raised
        else:
            out[sel] = chain_decode(raw, sh.inner, inner_spec)
    return out


def shard_decode_partial(blob: np.ndarray, sh: ShardSpec, shard_spec: Spec, selection: tuple) -> np.ndarray:
    """ShardingCodec._decode_partial_sync (sharding.py:1222-1309): the shard
    index (its CRC checked) and only the inner chunks `selection` touches are
    decoded -- a corrupted inner chunk outside the selection is never read.
    Returns a shard-shaped array whose touched inner chunks hold their data
    (the rest fill: never selected)."""
    cps = _cps(shard_spec, sh)
    inner_spec = Spec(sh.chunk_shape, shard_spec.dtype, shard_spec.fill_value,
                      shard_spec.write_empty_chunks, shard_spec.order)
    touched = {c for c, *_ in basic_indexer(selection, shard_spec.shape, sh.chunk_shape)[0]}
    chunks = shard_reader(blob, sh, cps)
    out = np.full(shard_spec.shape, shard_spec.fill_value, dtype=shard_spec.dtype)
    for coords in sorted(touched):
        raw = chunks[coords]
        if raw is not None:
            sel = tuple(slice(c * s, (c + 1) * s) for c, s in zip(coords, sh.chunk_shape))
            out[sel] = chain_decode(raw, sh.inner, inner_spec)
    return out


def shard_encode(shard_array: np.ndarray, sh: ShardSpec, shard_spec: Spec) -> np.ndarray | None:
    """ShardingCodec._encode_sync + _build_shard_layout + _assemble_shard
    (sharding.py:716-772, 887-950)."""
    cps = _cps(shard_spec, sh)
    inner_spec = Spec(sh.chunk_shape, shard_spec.dtype, shard_spec.fill_value,
                      shard_spec.write_empty_chunks, shard_spec.order)
    encoded: dict[tuple[int, ...], np.ndarray | None] = {}
    for coords in lexicographic_order_coords(cps):
        sel = tuple(slice(c * s, (c + 1) * s) for c, s in zip(coords, sh.chunk_shape))
        encoded[coords] = encode_or_elide(shard_array[sel], sh.inner, inner_spec)
    return assemble_shard(encoded, sh, cps)


def assemble_shard(encoded: dict, sh: ShardSpec, cps: tuple[int, ...]) -> np.ndarray | None:
    n = math.prod(cps)
    index = np.full(tuple(cps) + (2,), MAX_UINT_64, dtype="<u8")
    isize = shard_index_size(n, sh.index)
    start = isize if sh.index_location == "start" else 0
    bufs = []
    for coords in subchunk_order(cps, sh.subchunk_write_order):
        v = encoded.get(coords)
        if v is None or len(v) == 0:
            continue
        bufs.append(_as_u8(v))
        index[coords] = (start, len(v))
        start += len(v)
    if not bufs:
        return None
    index_bytes = encode_shard_index(index, sh.index)
    assert len(index_bytes) == isize
    if sh.index_location == "start":
        bufs.insert(0, index_bytes)
    else:
        bufs.append(index_bytes)
    return np.concatenate(bufs)


# ---------------------------------------------------------------------------
# Empty-chunk rule (chunk_utils.py:43-85, buffer/core.py:534-558)
# ---------------------------------------------------------------------------


def all_equal(arr: np.ndarray, other: Any) -> bool:
    """NDBuffer.all_equal (src/zarr/core/buffer/core.py:534-558)."""
    if other is None:
        return False
    if np.asarray(other).dtype.kind == "f" and other == 0.0 and arr.dtype.kind not in "USTOV":
        data, oth = np.broadcast_arrays(arr, np.asarray(other, arr.dtype))
        vd = f"V{data.dtype.itemsize}"
        return np.array_equal(data.view(vd), oth.view(vd))
    data, oth = np.broadcast_arrays(arr, other)
    return np.array_equal(data, oth, equal_nan=True)


def encode_or_elide(chunk_array: np.ndarray, chain: Chain, spec: Spec) -> np.ndarray | None:
    """encode_or_elide_chunk + chunk_is_empty (chunk_utils.py:43-85)."""
    if not spec.write_empty_chunks and all_equal(chunk_array, np.asarray(spec.fill_value,
                                                                          spec.dtype)):
        return None
    return chain_encode(chunk_array, chain, spec)


# ---------------------------------------------------------------------------
# Indexing (src/zarr/core/indexing.py:365-621)
# ---------------------------------------------------------------------------


def _ceildiv(a: int, b: int) -> int:
    return -(-a // b)


# ---------------------------------------------------------------------------
# Chunk grids (src/zarr/core/chunk_grids.py): FixedDimension 73-164,
# VaryingDimension 167-293, ChunkGrid.from_sizes 448-487, __getitem__ 528-546
# ---------------------------------------------------------------------------


class VaryingDim:
    """VaryingDimension (chunk_grids.py:167-293): explicit edges; data_size
    clips the last chunk at the extent, chunk_size (the codec shape) does not."""

    def __init__(self, edges, extent: int):
        self.edges = tuple(int(e) for e in edges)
        if not self.edges:
            raise ValueError("VaryingDimension edges must not be empty")
        if any(e <= 0 for e in self.edges):
            raise ValueError(f"All edge lengths must be > 0, got {self.edges}")
        self.cumulative = tuple(itertools.accumulate(self.edges))
        if extent > self.cumulative[-1]:
            raise ValueError(f"VaryingDimension extent {extent} exceeds sum of edges {self.cumulative[-1]}")
        self.extent = int(extent)
        # chunks overlapping [0, extent): bisect_left(cumulative, extent) + 1
        self.nchunks = 0 if extent == 0 else sum(1 for c in self.cumulative if c < extent) + 1

    def index_to_chunk(self, idx: int) -> int:
        if idx < 0 or idx >= self.extent:
            raise IndexError(f"Index {idx} out of bounds for dimension with extent {self.extent}")
        return sum(1 for c in self.cumulative if c <= idx)  # bisect_right

    def chunk_offset(self, ix: int) -> int:
        return self.cumulative[ix - 1] if ix > 0 else 0

    def chunk_size(self, ix: int) -> int:
        return self.edges[ix]

    def data_size(self, ix: int) -> int:
        return max(0, min(self.edges[ix], self.extent - self.chunk_offset(ix)))


class FixedDim:
    """FixedDimension (chunk_grids.py:73-130)."""

    def __init__(self, size: int, extent: int):
        self.size, self.extent = int(size), int(extent)
        self.nchunks = 0 if self.size == 0 else _ceildiv(self.extent, self.size)

    def index_to_chunk(self, idx: int) -> int:
        return 0 if self.size == 0 else idx // self.size

    def chunk_offset(self, ix: int) -> int:
        return ix * self.size

    def chunk_size(self, ix: int) -> int:
        return self.size

    def data_size(self, ix: int) -> int:
        return 0 if self.size == 0 else max(0, min(self.size, self.extent - ix * self.size))


def grid_dims(shape: tuple[int, ...], chunk_sizes) -> list:
    """ChunkGrid.from_sizes (chunk_grids.py:448-487): an int per dim is
    regular; an edge list is regular when its edges are equal and cover the
    extent, else varying."""
    dims = []
    for spec, extent in zip(chunk_sizes, shape):
        if isinstance(spec, (int, np.integer)):
            dims.append(FixedDim(int(spec), extent))
            continue
        edges = [int(e) for e in spec]
        if edges and edges[0] > 0 and all(e == edges[0] for e in edges) and (
                extent == sum(edges) or len(edges) == _ceildiv(extent, edges[0])):
            dims.append(FixedDim(edges[0], extent))
        else:
            dims.append(VaryingDim(edges, extent))
    return dims


def grid_getitem(dims: list, coords: tuple[int, ...]):
    """ChunkGrid.__getitem__ (chunk_grids.py:528-546): (slices, codec_shape),
    None out of bounds."""
    slices, cshape = [], []
    for d, ix in zip(dims, coords):
        if ix < 0 or ix >= d.nchunks:
            return None
        off = d.chunk_offset(ix)
        slices.append(slice(off, off + d.data_size(ix), 1))
        cshape.append(d.chunk_size(ix))
    return tuple(slices), tuple(cshape)


def dim_projections(sel: Any, dim_len: int, chunk_len):
    """IntDimIndexer / SliceDimIndexer.__iter__ (indexing.py:369-468) over a
    regular chunk length or a dimension grid (FixedDim / VaryingDim).
    Yields (chunk_ix, chunk_sel, out_sel|None, is_complete)."""
    if not isinstance(chunk_len, (int, np.integer)):
        yield from _dim_projections_grid(sel, dim_len, chunk_len)
        return
    nchunks = _ceildiv(dim_len, chunk_len)
    if isinstance(sel, (int, np.integer)):
        i = int(sel)
        if i < 0:
            i += dim_len
        if not 0 <= i < dim_len:
            raise IndexError(f"index out of bounds for dimension with length {dim_len}")
        ix = i // chunk_len
        data_size = min(chunk_len, dim_len - ix * chunk_len)
        yield ix, i - ix * chunk_len, None, data_size == 1
        return
    start, stop, step = sel.indices(dim_len)
    if step < 1:
        raise IndexError("only slices with step >= 1 are supported.")
    if start >= stop:
        return
    ix_from = start // chunk_len if start > 0 else 0
    ix_to = (stop - 1) // chunk_len + 1 if stop > 0 else 0
    for ix in range(ix_from, min(ix_to, nchunks)):
        off = ix * chunk_len
        clen = min(chunk_len, dim_len - off)  # FixedDimension.data_size (chunk_grids.py:119)
        limit = off + clen
        if start < off:
            s0 = 0
            rem = (off - start) % step
            if rem:
                s0 += step - rem
            out_off = _ceildiv(off - start, step)
        else:
            s0 = start - off
            out_off = 0
        s1 = clen if stop > limit else stop - off
        nitems = _ceildiv(s1 - s0, step)
        if nitems <= 0:
            continue
        complete = s0 == 0 and stop >= limit and step == 1
        yield ix, slice(s0, s1, step), slice(out_off, out_off + nitems), complete


def _dim_projections_grid(sel: Any, dim_len: int, g):
    """indexing.py:369-468 with the DimensionGrid protocol (index_to_chunk,
    chunk_offset, data_size)."""
    if isinstance(sel, (int, np.integer)):
        i = int(sel)
        if i < 0:
            i += dim_len
        if not 0 <= i < dim_len:
            raise IndexError(f"index out of bounds for dimension with length {dim_len}")
        ix = g.index_to_chunk(i)
        yield ix, i - g.chunk_offset(ix), None, g.data_size(ix) == 1
        return
    start, stop, step = sel.indices(dim_len)
    if step < 1:
        raise IndexError("only slices with step >= 1 are supported.")
    if start >= stop:
        return
    ix_from = g.index_to_chunk(start) if start > 0 else 0
    ix_to = g.index_to_chunk(stop - 1) + 1 if stop > 0 else 0
    for ix in range(ix_from, ix_to):
        off = g.chunk_offset(ix)
        clen = g.data_size(ix)
        limit = off + clen
        if start < off:
            s0 = 0
            rem = (off - start) % step
            if rem:
                s0 += step - rem
            out_off = _ceildiv(off - start, step)
        else:
            s0 = start - off
            out_off = 0
        s1 = clen if stop > limit else stop - off
        nitems = _ceildiv(s1 - s0, step)
        if nitems <= 0:
            continue
        complete = s0 == 0 and stop >= limit and step == 1
        yield ix, slice(s0, s1, step), slice(out_off, out_off + nitems), complete


def basic_indexer(selection: tuple, shape: tuple[int, ...], chunk_shape):
    """BasicIndexer (indexing.py:571-621): list of ChunkProjection + output shape."""
    if not isinstance(selection, tuple):
        selection = (selection,)
    sel = list(selection)
    if any(s is Ellipsis for s in sel):
        i = sel.index(Ellipsis)
        sel = sel[:i] + [slice(None)] * (len(shape) - len(sel) + 1) + sel[i + 1:]
    sel += [slice(None)] * (len(shape) - len(sel))
    per_dim = [list(dim_projections(s, n, c)) for s, n, c in zip(sel, shape, chunk_shape)]
    out_shape = []
    for s, n in zip(sel, shape):
        if isinstance(s, (int, np.integer)):
            continue
        a, b, st = s.indices(n)
        out_shape.append(max(0, _ceildiv(b - a, st)))
    projections = []
    for combo in itertools.product(*per_dim):
        coords = tuple(p[0] for p in combo)
        csel = tuple(p[1] for p in combo)
        osel = tuple(p[2] for p in combo if p[2] is not None)
        complete = all(p[3] for p in combo)
        projections.append((coords, csel, osel, complete))
    return projections, tuple(out_shape)


# ---------------------------------------------------------------------------
# Array-level read/write (FusedCodecPipeline.read_sync / write_sync,
# src/zarr/core/codec_pipeline.py:1095-1253, array.py:5393-5675)
# ---------------------------------------------------------------------------


@dataclass
class ArrayMeta:
    shape: tuple[int, ...]
    chunk_shape: tuple[int, ...]
    dtype: np.dtype
    fill_value: Any
    codecs: list = field(default_factory=lambda: [{"name": "bytes",
                                                   "configuration": {"endian": "little"}}])
    write_empty_chunks: bool = False

    def __post_init__(self):
        # chunk_shape may name a rectilinear grid: per dim an int or an edge list
        self.chunk_shape = tuple(c if isinstance(c, (int, np.integer)) else tuple(int(e) for e in c)
                                 for c in self.chunk_shape)

    @property
    def regular(self) -> bool:
        return all(isinstance(c, (int, np.integer)) for c in self.chunk_shape)

    def dims(self) -> list:
        return grid_dims(self.shape, self.chunk_shape)

    def chunk_spec(self, coords: tuple[int, ...]) -> Spec:
        """_get_chunk_spec (array.py:5373-5390): the chunk's codec shape."""
        if self.regular:
            return self.spec()
        got = grid_getitem(self.dims(), coords)
        if got is None:
            raise IndexError(f"Chunk coordinates {coords} are out of bounds.")
        return Spec(got[1], np.dtype(self.dtype), self.fill_value, self.write_empty_chunks)

    @property
    def chain(self) -> Chain:
        return Chain.from_json(self.codecs)

    def chunk_key(self, coords: tuple[int, ...]) -> str:
        """DefaultChunkKeyEncoding.encode_chunk_key (chunk_key_encodings.py:87-88)."""
        return "/".join(map(str, ("c",) + tuple(coords)))

    def spec(self) -> Spec:
        return Spec(self.chunk_shape, np.dtype(self.dtype), self.fill_value,
                    self.write_empty_chunks)


def read(store: dict, meta: ArrayMeta, selection: Any = Ellipsis) -> np.ndarray:
    """Array._get_selection + FusedCodecPipeline.read_sync (per-chunk decode &
    scatter; a sharding codec with no array->array / bytes->bytes codec around
    it takes the partial-decode path, codec_pipeline.py:1136-1150, 143-166)."""
    grid = meta.chunk_shape if meta.regular else meta.dims()
    projections, out_shape = basic_indexer(selection if isinstance(selection, tuple)
                                           else (selection,), meta.shape, grid)
    out = np.empty(out_shape, dtype=meta.dtype)
    chain = meta.chain
    partial = chain.shard is not None and not chain.aa and not chain.bb
    for coords, csel, osel, _ in projections:
        raw = store.get(meta.chunk_key(coords))
        if raw is None:
            out[osel] = meta.fill_value  # scatter_chunk(None, ...) (chunk_utils.py:106-108)
            continue
        if partial:
            chunk = shard_decode_partial(_as_u8(raw), chain.shard, meta.chunk_spec(coords), csel)
        else:
            chunk = chain_decode(_as_u8(raw), chain, meta.chunk_spec(coords))
        out[osel] = chunk[csel]
    return out


def _merge(existing: np.ndarray | None, value: np.ndarray, osel, spec: Spec, csel,
           complete: bool) -> np.ndarray:
    """_merge_chunk_array (chunk_utils.py:115-162)."""
    if complete and value.shape != ():
        selected = value[osel]
        if selected.shape == tuple(spec.shape):
            return selected
    chunk = np.full(spec.shape, spec.fill_value, dtype=spec.dtype) if existing is None \
        else existing.copy()
    chunk[csel] = value if value.shape == () else value[osel].reshape(chunk[csel].shape)
    return chunk


def shard_encode_partial(store: dict, key: str, chunk_value: np.ndarray, selection: tuple,
                         sh: ShardSpec, shard_spec: Spec) -> None:
    """ShardingCodec._encode_partial_sync (sharding.py:774-885), reached from
    FusedCodecPipeline.write_sync when the chain is a sharding codec alone
    (codec_pipeline.py:1211-1220): only the inner chunks the selection touches
    are merged and re-encoded; the others keep their stored bytes (or absence)."""
    cps = _cps(shard_spec, sh)
    inner_spec = Spec(sh.chunk_shape, shard_spec.dtype, shard_spec.fill_value,
                      shard_spec.write_empty_chunks, shard_spec.order)
    projections, _ = basic_indexer(selection, shard_spec.shape, sh.chunk_shape)
    touched = {c for c, *_ in projections}
    complete_shard = touched == set(lexicographic_order_coords(cps)) and all(
        p[3] for p in projections)  # _is_complete_shard_write (1437-1445)
    existing = None if complete_shard else store.get(key)
    if existing is None:
        shard_dict = dict.fromkeys(lexicographic_order_coords(cps))
    else:
        shard_dict = shard_reader(_as_u8(existing), sh, cps)
    for coords, csel, osel, complete in projections:
        raw = None if complete else shard_dict.get(coords)
        old = None if raw is None else chain_decode(raw, sh.inner, inner_spec)
        merged = _merge(old, chunk_value, osel, inner_spec, csel, complete)
        shard_dict[coords] = encode_or_elide(merged, sh.inner, inner_spec)
    blob = assemble_shard(shard_dict, sh, cps)
    if blob is None:
        store.pop(key, None)
    else:
        store[key] = bytes(blob)


def write(store: dict, meta: ArrayMeta, selection: Any, value: Any) -> None:
    """Array._set_selection + FusedCodecPipeline.write_sync + merge_and_encode_chunk
    (partial shard encode when the chain is a sharding codec alone)."""
    grid = meta.chunk_shape if meta.regular else meta.dims()
    projections, out_shape = basic_indexer(selection if isinstance(selection, tuple)
                                           else (selection,), meta.shape, grid)
    value = np.asarray(value, dtype=meta.dtype)
    chain = meta.chain
    if chain.shard is not None and not chain.aa and not chain.bb:
        for coords, csel, osel, complete in projections:
            chunk_value = value if value.shape == () else value[osel]
            shard_encode_partial(store, meta.chunk_key(coords), chunk_value, csel, chain.shard,
                                 meta.chunk_spec(coords))
        return
    for coords, csel, osel, complete in projections:
        key = meta.chunk_key(coords)
        spec = meta.chunk_spec(coords)
        if complete and value.shape != ():
            merged = value[osel]
            if merged.shape != tuple(spec.shape):
                merged = None
        else:
            merged = None
        if merged is None:
            raw = None if complete else store.get(key)
            if raw is None:
                merged = np.full(spec.shape, meta.fill_value, dtype=meta.dtype)
            else:
                merged = chain_decode(_as_u8(raw), chain, spec).copy()
            merged[csel] = value if value.shape == () else value[osel].reshape(
                merged[csel].shape)
        enc = encode_or_elide(merged, chain, spec)
        if enc is None:
            store.pop(key, None)
        else:
            store[key] = bytes(enc)

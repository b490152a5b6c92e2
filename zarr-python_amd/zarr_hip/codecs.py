"""Codec configuration objects for the fixed-size chain the GPU pipeline runs.

These mirror the reference codecs' *metadata* surface (from_dict / to_dict /
evolve_from_array_spec / resolve_metadata / compute_encoded_size / validate);
their compute lives in the HIP kernels, driven by ``pipeline.HipCodecPipeline``.

  BytesCodec      src/zarr/codecs/bytes.py:42-168
  Crc32cCodec     src/zarr/codecs/crc32c_.py:20-78
  TransposeCodec  src/zarr/codecs/transpose.py:29-128
  ShardingCodec   src/zarr/codecs/sharding.py:402-1756 (configuration + layout rules)

Compression codecs stay on the host (the north star): ``GzipCodec`` (the
``gzip`` name from JSON metadata, stdlib gzip as numcodecs.GZip) and
``HostCodec`` (any bytes->bytes codec INSTANCE a caller hands over -- zarr's
GzipCodec / ZstdCodec / BloscCodec -- driven through its own ``_decode_sync`` /
``_encode_sync``, src/zarr/abc/codec.py:69-96) form the host stage of a chain
(``split_host_tail``); hoststage.py runs it, the GPU runs the rest.
"""

from __future__ import annotations

import sys
from dataclasses import dataclass, field, replace
from typing import Any

import numpy as np

from .spec import ArraySpec

MAX_UINT_64 = 2**64 - 1
SUBCHUNK_WRITE_ORDER = ("morton", "unordered", "lexicographic", "colexicographic")


def _named(data: Any, name: str) -> dict:
    if isinstance(data, str):
        if data != name:
            raise ValueError(f"Expected '{name}'. Got {data} instead.")
        return {}
    if data.get("name") != name:
        raise ValueError(f"Expected '{name}'. Got {data.get('name')} instead.")
    return dict(data.get("configuration") or {})


@dataclass(frozen=True)
class BytesCodec:
    """bytes.py:42-168.  ``endian`` None is legal only for single-byte types."""

    endian: str | None = sys.byteorder
    is_fixed_size = True
    kind = "AB"

    def __post_init__(self):
        if self.endian is not None and self.endian not in ("little", "big"):
            raise ValueError(f"endian must be one of ['little', 'big']. Got {self.endian!r}.")

    @classmethod
    def from_dict(cls, data: Any) -> "BytesCodec":
        conf = _named(data, "bytes")
        e = conf.get("endian")
        return cls(endian=None if e is None else str(getattr(e, "value", e)))

    def to_dict(self) -> dict:
        if self.endian is None:
            return {"name": "bytes"}
        return {"name": "bytes", "configuration": {"endian": self.endian}}

    def evolve_from_array_spec(self, spec: ArraySpec) -> "BytesCodec":
        """bytes.py:74-95 (structured dtypes are outside the GPU path)."""
        if spec.dtype.itemsize == 1:
            return replace(self, endian=None) if self.endian is not None else self
        if self.endian is None:
            raise ValueError(
                "The `endian` configuration needs to be specified for multi-byte data types.")
        return self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        return n

    def validate(self, **kw) -> None:
        return None

    def needs_swap(self, dtype: np.dtype) -> bool:
        """Decoded arrays are native (little-endian on MI355X and its host), so the
        stored bytes need a swap exactly when they are big-endian multi-byte items
        (bytes.py:118-127)."""
        return dtype.itemsize > 1 and self.endian == "big"


@dataclass(frozen=True)
class Crc32cCodec:
    """crc32c_.py:20-78: 4-byte little-endian CRC-32C trailer."""

    is_fixed_size = True
    kind = "BB"

    @classmethod
    def from_dict(cls, data: Any) -> "Crc32cCodec":
        _named(data, "crc32c")
        return cls()

    def to_dict(self) -> dict:
        return {"name": "crc32c"}

    def evolve_from_array_spec(self, spec: ArraySpec) -> "Crc32cCodec":
        return self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        return n + 4

    def validate(self, **kw) -> None:
        return None


@dataclass(frozen=True)
class TransposeCodec:
    """transpose.py:29-128."""

    order: tuple[int, ...]
    is_fixed_size = True
    kind = "AA"

    def __post_init__(self):
        object.__setattr__(self, "order", tuple(int(i) for i in self.order))

    @classmethod
    def from_dict(cls, data: Any) -> "TransposeCodec":
        conf = _named(data, "transpose")
        return cls(order=tuple(conf["order"]))

    def to_dict(self) -> dict:
        return {"name": "transpose", "configuration": {"order": tuple(self.order)}}

    def _check(self, ndim: int) -> None:
        if len(self.order) != ndim:
            raise ValueError(
                "The `order` tuple must have as many entries as there are dimensions in the "
                f"array. Got {self.order}.")
        if len(self.order) != len(set(self.order)):
            raise ValueError(f"There must not be duplicates in the `order` tuple. Got {self.order}.")
        if not all(0 <= x < ndim for x in self.order):
            raise ValueError(
                "All entries in the `order` tuple must be between 0 and the number of dimensions "
                f"in the array. Got {self.order}.")

    def validate(self, *, shape, **kw) -> None:
        self._check(len(shape))

    def evolve_from_array_spec(self, spec: ArraySpec) -> "TransposeCodec":
        self._check(spec.ndim)
        return self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        """transpose.py:89-96."""
        return replace(spec, shape=tuple(spec.shape[self.order[i]] for i in range(spec.ndim)))

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        return n


@dataclass(frozen=True)
class ShardingCodec:
    """sharding.py:402-1756: configuration, index layout and size rules."""

    chunk_shape: tuple[int, ...]
    codecs: tuple = field(default_factory=lambda: (BytesCodec(),))
    index_codecs: tuple = field(default_factory=lambda: (BytesCodec(endian="little"), Crc32cCodec()))
    index_location: str = "end"
    subchunk_write_order: str = "morton"
    is_fixed_size = False
    kind = "AB"

    def __post_init__(self):
        object.__setattr__(self, "chunk_shape", tuple(int(c) for c in self.chunk_shape))
        object.__setattr__(self, "codecs", tuple(parse_codecs(self.codecs)))
        object.__setattr__(self, "index_codecs", tuple(parse_codecs(self.index_codecs)))
        if self.index_location not in ("start", "end"):
            raise ValueError(
                f"index_location must be one of ['start', 'end']. Got {self.index_location!r}.")
        if self.subchunk_write_order not in SUBCHUNK_WRITE_ORDER:
            raise ValueError(
                f"Unrecognized subchunk write order: {self.subchunk_write_order}. "
                f"Only {SUBCHUNK_WRITE_ORDER} are allowed.")

    @classmethod
    def from_dict(cls, data: Any) -> "ShardingCodec":
        conf = _named(data, "sharding_indexed")
        return cls(chunk_shape=tuple(conf["chunk_shape"]),
                   codecs=tuple(conf.get("codecs", ({"name": "bytes"},))),
                   index_codecs=tuple(conf.get("index_codecs", (
                       {"name": "bytes", "configuration": {"endian": "little"}},
                       {"name": "crc32c"}))),
                   index_location=str(getattr(conf.get("index_location", "end"), "value",
                                              conf.get("index_location", "end"))))

    def to_dict(self) -> dict:
        return {"name": "sharding_indexed", "configuration": {
            "chunk_shape": self.chunk_shape,
            "codecs": tuple(c.to_dict() for c in self.codecs),
            "index_codecs": tuple(c.to_dict() for c in self.index_codecs),
            "index_location": self.index_location}}

    def validate(self, *, shape, chunk_shape=None, chunk_grid=None, **kw) -> None:
        """sharding.py:567-593: every distinct edge of the (regular or
        rectilinear) outer grid divisible by the inner chunk size."""
        if len(self.chunk_shape) != len(shape):
            raise ValueError("The shard's `chunk_shape` and array's `shape` need to have the same "
                             "number of dimensions.")
        edges_per_dim = None
        if chunk_shape is not None:
            edges_per_dim = tuple((int(e),) for e in chunk_shape)
        elif chunk_grid is not None:
            dims = getattr(chunk_grid, "dimensions", None)
            if dims is not None:  # zarr_hip.grid.ChunkGrid
                edges_per_dim = tuple(tuple(d.unique_edge_lengths) for d in dims)
            else:  # zarr's Regular / RectilinearChunkGridMetadata
                cs = getattr(chunk_grid, "chunk_shape", None)
                shapes = getattr(chunk_grid, "chunk_shapes", None)
                if cs is not None:
                    edges_per_dim = tuple((int(e),) for e in cs)
                elif shapes is not None:
                    edges_per_dim = tuple((int(s),) if isinstance(s, int) else tuple(s) for s in shapes)
        for i, (edges, inner) in enumerate(zip(edges_per_dim or (), self.chunk_shape)):
            for edge in dict.fromkeys(edges):
                if edge % inner != 0:
                    raise ValueError(f"Chunk edge length {edge} in dimension {i} is not divisible "
                                     f"by the shard's inner chunk size {inner}.")

    def chunks_per_shard(self, shard_shape: tuple[int, ...]) -> tuple[int, ...]:
        """_get_chunks_per_shard (sharding.py:1544-1552)."""
        return tuple(s // c for s, c in zip(shard_shape, self.chunk_shape))

    def inner_spec(self, shard_spec: ArraySpec) -> ArraySpec:
        """_get_chunk_spec (sharding.py:1535-1542)."""
        return replace(shard_spec, shape=self.chunk_shape)

    def shard_index_size(self, n_inner: int) -> int:
        """_shard_index_size (sharding.py:1515-1522)."""
        n = 16 * n_inner
        for c in self.index_codecs:
            n = c.compute_encoded_size(n)
        return n

    @property
    def index_has_crc(self) -> bool:
        return any(isinstance(c, Crc32cCodec) for c in self.index_codecs)

    def evolve_from_array_spec(self, spec: ArraySpec) -> "ShardingCodec":
        inner = self.inner_spec(spec)
        ev = evolve_codecs(self.codecs, inner)
        return replace(self, codecs=ev) if ev != self.codecs else self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        raise NotImplementedError("sharding_indexed output is not fixed-size")


def gzip_member(data, level: int) -> bytes:
    """The bytes ``gzip.compress(data, compresslevel=level, mtime=0)`` returns
    (one member as GzipFile writes it: no name, mtime 0, XFL by level, OS 255,
    raw deflate, CRC-32, ISIZE), built on zlib directly: the deflate runs
    without the GIL, so the host stage's threads compress in parallel
    (gzip.compress in Python 3.10 drives a GzipFile object per call)."""
    import struct
    import zlib

    mv = memoryview(data).cast("B") if not isinstance(data, (bytes, bytearray)) else data
    co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS, zlib.DEF_MEM_LEVEL, 0)
    body = co.compress(mv) + co.flush()
    xfl = b"\002" if level == 9 else b"\004" if level == 1 else b"\000"
    return b"\037\213\010\000\000\000\000\000" + xfl + b"\377" + body + \
        struct.pack("<II", zlib.crc32(mv) & 0xFFFFFFFF, len(mv) & 0xFFFFFFFF)


def gzip_decode(data) -> bytes:
    """numcodecs.GZip.decode over zlib: a gzip member (several members are
    concatenated, as gzip.decompress reads them) or a raw zlib stream; the
    inflate runs without the GIL."""
    import zlib

    b = data if isinstance(data, (bytes, bytearray)) else bytes(data)
    if b[:2] != b"\x1f\x8b":
        return zlib.decompress(b)
    out = []
    while b:
        d = zlib.decompressobj(31)
        out.append(d.decompress(b))
        if not d.eof:
            raise EOFError("Compressed file ended before the end-of-stream marker was reached")
        b = d.unused_data
        if b and b[:2] != b"\x1f\x8b":
            break  # trailing garbage after the last member (gzip.decompress ignores zero padding)
    return b"".join(out)


@dataclass(frozen=True)
class GzipCodec:
    """src/zarr/codecs/gzip.py:31-95 on the host: numcodecs.GZip's stream (a gzip
    member, mtime 0) for encode; decode takes a gzip member or, as
    numcodecs.GZip.decode does, a raw zlib stream."""

    level: int = 5
    is_fixed_size = False
    host = True
    kind = "BB"

    def __post_init__(self):
        lv = self.level
        if isinstance(lv, bool) or not isinstance(lv, int):
            raise TypeError(f"Expected an integer. Got {lv!r} instead.")
        if lv not in range(10):
            raise ValueError(f"Expected an integer from the inclusive range (0, 9). Got {lv} instead.")

    @classmethod
    def from_dict(cls, data: Any) -> "GzipCodec":
        conf = _named(data, "gzip")
        return cls(level=conf.get("level", 5))

    def to_dict(self) -> dict:
        return {"name": "gzip", "configuration": {"level": self.level}}

    def evolve_from_array_spec(self, spec: ArraySpec) -> "GzipCodec":
        return self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        raise NotImplementedError  # gzip.py:89-95

    def validate(self, **kw) -> None:
        return None

    def decode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        return gzip_decode(data)

    def encode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        return gzip_member(data, self.level)


class _HostBuffer:
    """The slice of zarr's Buffer API a bytes->bytes codec uses on the host
    (as_numpy_array / to_bytes / from_bytes, src/zarr/core/buffer/cpu.py), for
    specs that carry no prototype of their own."""

    def __init__(self, data):
        self._a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else \
            np.ascontiguousarray(data).reshape(-1).view(np.uint8)

    @classmethod
    def from_bytes(cls, b) -> "_HostBuffer":
        return cls(b)

    @classmethod
    def from_array_like(cls, a) -> "_HostBuffer":
        return cls(np.asarray(a))

    def as_numpy_array(self) -> np.ndarray:
        return self._a

    def as_array_like(self) -> np.ndarray:
        return self._a

    def to_bytes(self) -> bytes:
        return self._a.tobytes()

    def __len__(self) -> int:
        return int(self._a.size)


class _HostPrototype:
    buffer = _HostBuffer
    nd_buffer = None


HOST_PROTOTYPE = _HostPrototype()


@dataclass(frozen=True)
class HostCodec:
    """A caller-supplied bytes->bytes codec instance (zarr's GzipCodec,
    ZstdCodec, BloscCodec, ... -- nothing of zarr or numcodecs is imported
    here): the pipeline calls its ``_decode_sync`` / ``_encode_sync``
    (SupportsSyncCodec, src/zarr/abc/codec.py:69-96) on the host with a host
    Buffer and the chunk's spec, outside the GPU launch."""

    codec: Any
    is_fixed_size = False
    host = True
    kind = "BB"

    def to_dict(self) -> dict:
        return self.codec.to_dict()

    @property
    def name(self) -> str:
        d = self.to_dict()
        return d if isinstance(d, str) else d.get("name", type(self.codec).__name__)

    def evolve_from_array_spec(self, spec: ArraySpec) -> "HostCodec":
        src = getattr(spec, "source", None)
        ev = getattr(self.codec, "evolve_from_array_spec", None)
        if ev is None or src is None:  # only zarr's own spec type is safe to hand it
            return self
        new = ev(src)
        return self if new is self.codec else HostCodec(new)

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        fn = getattr(self.codec, "compute_encoded_size", None)
        if fn is None:
            raise NotImplementedError
        return fn(n, getattr(spec, "source", None) or spec)

    def validate(self, **kw) -> None:
        return None

    def _spec(self, spec: ArraySpec | None):
        src = getattr(spec, "source", None)
        if src is not None:
            return src
        if spec is None:
            return ArraySpec((0,), np.dtype("u1"), 0, prototype=HOST_PROTOTYPE)
        return spec if spec.prototype is not None and hasattr(getattr(spec.prototype, "buffer", None),
                                                              "from_bytes") else replace(spec, prototype=HOST_PROTOTYPE)

    def decode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        sp = self._spec(spec)
        out = self.codec._decode_sync(sp.prototype.buffer.from_bytes(bytes(data)), sp)
        return _to_bytes(out)

    def encode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        sp = self._spec(spec)
        out = self.codec._encode_sync(sp.prototype.buffer.from_bytes(bytes(data)), sp)
        if out is None:
            raise ValueError(f"host codec {self.name!r} returned no bytes")
        return _to_bytes(out)


@dataclass(frozen=True)
class ForeignArrayCodec:
    """A caller's array->array codec instance other than ``transpose`` (e.g. a
    cast or scale filter).  The pipeline accepts it in a chain and threads the
    chunk spec through it exactly as the reference does
    (``evolve_from_array_spec`` forwards each codec's ``resolve_metadata``,
    chunk_utils.py:18-40; regression test
    tests/test_codec_pipeline.py:189-261), but its compute is not on the GPU
    path: a read or write through such a chain raises NotImplementedError
    (planner.analyze_chain)."""

    codec: Any
    is_fixed_size = True
    kind = "AA"

    def to_dict(self) -> dict:
        return self.codec.to_dict()

    @property
    def name(self) -> str:
        d = self.to_dict()
        return d if isinstance(d, str) else d.get("name", type(self.codec).__name__)

    def evolve_from_array_spec(self, spec: ArraySpec) -> "ForeignArrayCodec":
        ev = getattr(self.codec, "evolve_from_array_spec", None)
        if ev is None:
            return self
        new = ev(getattr(spec, "source", None) or spec)
        return self if new is self.codec else ForeignArrayCodec(new)

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        from .spec import coerce_spec

        return coerce_spec(self.codec.resolve_metadata(getattr(spec, "source", None) or spec))

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        return self.codec.compute_encoded_size(n, getattr(spec, "source", None) or spec)

    def validate(self, **kw) -> None:
        fn = getattr(self.codec, "validate", None)
        if fn is not None:
            fn(**kw)


@dataclass(frozen=True)
class V2Stage:
    """The host half of zarr v2's codec wrapper (V2Codec, src/zarr/codecs/_v2.py:
    19-96): the numcodecs compressor and filters the caller's V2Codec holds run
    on the host, in the reference's order; the raw chunk bytes they produce or
    consume are the fixed-size part the GPU decodes / encodes as a little-endian
    ``bytes`` codec (plus a reversing transpose for ``order="F"``, added when the
    pipeline is evolved against the chunk spec).  Nothing of numcodecs is
    imported: the objects are the caller's."""

    filters: tuple
    compressor: Any
    is_fixed_size = False
    host = True
    kind = "BB"

    def to_dict(self) -> dict:
        return {"name": "v2", "configuration": {"filters": [repr(f) for f in self.filters],
                                                "compressor": repr(self.compressor)}}

    @property
    def name(self) -> str:
        return "v2"

    def evolve_from_array_spec(self, spec: ArraySpec) -> "V2Stage":
        return self

    def resolve_metadata(self, spec: ArraySpec) -> ArraySpec:
        return spec

    def compute_encoded_size(self, n: int, spec: ArraySpec | None = None) -> int:
        raise NotImplementedError  # _v2.py:95-96

    def validate(self, **kw) -> None:
        return None

    def decode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        """_v2.py:25-70 up to the reinterpretation: decompress, filters in reverse,
        then the chunk's bytes in memory order (reshape(-1, order="A"))."""
        chunk = self.compressor.decode(bytes(data)) if self.compressor else data
        for f in reversed(self.filters):
            chunk = f.decode(chunk)
        if isinstance(chunk, (bytes, bytearray, memoryview)):
            return bytes(chunk)
        a = np.asarray(chunk)
        if a.dtype == object:
            raise RuntimeError("cannot read object array without object codec")
        return a.reshape(-1, order="A").view(np.uint8).tobytes()

    def encode_bytes(self, data, spec: ArraySpec | None = None) -> bytes:
        """_v2.py:72-93: the chunk as an array of the native dtype in the spec's
        shape and order, filters, compressor."""
        raw = np.frombuffer(bytes(data), np.uint8)
        chunk = raw
        if spec is not None and raw.size == int(np.prod(spec.shape)) * spec.dtype.itemsize:
            chunk = raw.view(spec.dtype).reshape(spec.shape, order=spec.order)
        for f in self.filters:
            chunk = f.encode(chunk)
        if np.asarray(chunk).dtype == object:
            raise RuntimeError("cannot write object array without object codec")
        cdata = self.compressor.encode(chunk) if self.compressor else chunk
        return _to_bytes(cdata) if not isinstance(cdata, np.ndarray) else \
            np.ascontiguousarray(cdata).reshape(-1).view(np.uint8).tobytes()


def is_v2_codec(c) -> bool:
    """zarr's V2Codec instance (duck-typed: no zarr import)."""
    return type(c).__name__ == "V2Codec" and hasattr(c, "filters") and hasattr(c, "compressor")


def v2_chain(c) -> list:
    """V2Codec(filters, compressor) -> [bytes(little), V2Stage] (the stage only
    when there is something to run on the host)."""
    filters = tuple(c.filters or ())
    out = [BytesCodec(endian="little")]
    if filters or c.compressor is not None:
        out.append(V2Stage(filters, c.compressor))
    return out


def _to_bytes(buf) -> bytes:
    if isinstance(buf, (bytes, bytearray, memoryview)):
        return bytes(buf)
    if hasattr(buf, "to_bytes"):
        return buf.to_bytes()
    return np.ascontiguousarray(buf.as_numpy_array()).reshape(-1).view(np.uint8).tobytes()


def is_host_codec(c) -> bool:
    return getattr(c, "host", False) is True


def split_host_tail(codecs) -> tuple[tuple, tuple]:
    """(GPU part, host stage) of a chain: the bytes->bytes codecs from the
    first host codec on run on the host (a crc32c after a compressor checks
    the compressed bytes, so it stays in that order); every bytes->bytes codec
    after a sharding codec does too (the GPU path reads shard blobs as stored)."""
    codecs = tuple(codecs)
    ab_at = next((i for i, c in enumerate(codecs) if isinstance(c, (BytesCodec, ShardingCodec))), None)
    if ab_at is None:
        return codecs, ()
    cut = len(codecs)
    for i in range(ab_at + 1, len(codecs)):
        if is_host_codec(codecs[i]) or isinstance(codecs[ab_at], ShardingCodec):
            cut = i
            break
    return codecs[:cut], codecs[cut:]


_REGISTRY = {
    "bytes": BytesCodec,
    "crc32c": Crc32cCodec,
    "transpose": TransposeCodec,
    "sharding_indexed": ShardingCodec,
    "gzip": GzipCodec,
}


def parse_codecs(codecs) -> list:
    """Codec configurations -> this package's codec objects.  Accepts its own
    codecs, JSON dicts / names (the zarr.json form), and zarr's Codec instances
    (duck-typed through ``to_dict()``, src/zarr/abc/codec.py:99-225, the form
    ``CodecPipeline.from_codecs`` receives); a sharding codec's write-time
    ``subchunk_write_order`` (not part of its metadata, sharding.py:402-446) is
    carried over from the instance."""
    out = []
    for c in codecs:
        if isinstance(c, (BytesCodec, Crc32cCodec, TransposeCodec, ShardingCodec, GzipCodec, HostCodec, V2Stage,
                          ForeignArrayCodec)):
            out.append(c)
            continue
        if is_v2_codec(c):  # zarr v2's filters + compressor wrapper (an ArrayBytesCodec)
            out.extend(v2_chain(c))
            continue
        conf = c.to_dict() if hasattr(c, "to_dict") and not isinstance(c, dict) else c
        name = conf if isinstance(conf, str) else conf["name"]
        if name != "transpose" and not isinstance(c, (dict, str)) and codec_kind(c) == "AA":
            out.append(ForeignArrayCodec(c))  # spec threading only; not on the GPU path
            continue
        if name not in ("bytes", "crc32c", "transpose", "sharding_indexed") and not isinstance(c, (dict, str)) \
                and hasattr(c, "_decode_sync") and hasattr(c, "_encode_sync"):
            # a compressor instance (zarr's GzipCodec / ZstdCodec / BloscCodec ...):
            # its own sync methods run the host stage, exactly as the reference does
            out.append(HostCodec(c))
            continue
        if name not in _REGISTRY:
            raise NotImplementedError(
                f"codec {name!r} needs its codec object (compression runs on the host through the "
                f"instance zarr passes to from_codecs; no built-in {name!r} implementation here)")
        if name == "sharding_indexed" and not isinstance(c, (dict, str)) and hasattr(c, "codecs"):
            # zarr's ShardingCodec: keep its inner codec INSTANCES (to_dict would
            # flatten a compressor to its JSON name and lose the object that
            # runs it)
            loc = getattr(c, "index_location", "end")
            parsed = ShardingCodec(chunk_shape=tuple(c.chunk_shape), codecs=tuple(c.codecs),
                                   index_codecs=tuple(getattr(c, "index_codecs", None)
                                                      or (BytesCodec(endian="little"), Crc32cCodec())),
                                   index_location=str(getattr(loc, "value", loc)))
        else:
            parsed = _REGISTRY[name].from_dict(conf)
        order = getattr(c, "subchunk_write_order", None)
        if isinstance(parsed, ShardingCodec) and order is not None and not isinstance(c, dict):
            parsed = replace(parsed, subchunk_write_order=str(order))
        out.append(parsed)
    return out


def evolve_codecs(codecs, spec: ArraySpec) -> tuple:
    """chunk_utils.py:18-40: evolve each codec against the spec threaded forward."""
    out = []
    for c in codecs:
        e = c.evolve_from_array_spec(spec)
        out.append(e)
        spec = e.resolve_metadata(spec)
    return tuple(out)


def codec_kind(c) -> str | None:
    """"AA" / "AB" / "BB" for this package's codecs (their ``kind``) and for a
    zarr Codec instance (its base class: ArrayArrayCodec / ArrayBytesCodec /
    BytesBytesCodec, src/zarr/abc/codec.py:228-262, matched by name -- zarr is
    not imported); None for anything else."""
    k = getattr(c, "kind", None)
    if k in ("AA", "AB", "BB"):
        return k
    for base in type(c).__mro__:
        n = base.__name__
        if n == "ArrayArrayCodec":
            return "AA"
        if n == "ArrayBytesCodec":
            return "AB"
        if n == "BytesBytesCodec":
            return "BB"
    return None


def split_codecs(codecs) -> tuple[tuple, Any, tuple]:
    """codecs_from_list_unchecked (codec_pipeline.py:886-944): one left-to-right
    scan over adjacent pairs, so the first structural violation decides the
    error -- an array->array codec after an array->bytes or bytes->bytes one,
    an array->bytes codec right after a bytes->bytes one, and a bytes->bytes
    codec right after an array->array one are TypeErrors; a second
    array->bytes codec, or none at all, is a ValueError."""
    aa, ab, bb = [], None, []
    prev = None
    for c in codecs:
        k = codec_kind(c)
        pk = None if prev is None else codec_kind(prev)
        if k == "AA":
            if pk in ("AB", "BB"):
                raise TypeError(f"Invalid codec order. ArrayArrayCodec {c} must be preceded by another "
                                f"ArrayArrayCodec. Got {type(prev)} instead.")
            aa.append(c)
        elif k == "AB":
            if pk == "BB":
                raise TypeError(f"Invalid codec order. ArrayBytes codec {c} must be preceded by an "
                                f"ArrayArrayCodec. Got {type(prev)} instead.")
            if ab is not None:
                raise ValueError(f"Got two instances of ArrayBytesCodec: {ab} and {c}. "
                                 "Only one array-to-bytes codec is allowed.")
            ab = c
        elif k == "BB":
            if pk == "AA":
                raise TypeError(f"Invalid codec order. BytesBytesCodec {c} must be preceded by either "
                                f"another BytesBytesCodec, or an ArrayBytesCodec. Got {type(prev)} instead.")
            bb.append(c)
        else:
            raise TypeError(f"not a codec: {c!r}")
        prev = c
    if ab is None:
        raise ValueError("Required ArrayBytesCodec was not found.")
    return tuple(aa), ab, tuple(bb)

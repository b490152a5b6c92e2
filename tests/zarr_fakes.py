"""Duck-typed stand-ins for the zarr-python objects a CodecPipeline receives
(test infrastructure).  zarr itself needs Python >= 3.12 and cannot be imported
here, so its interfaces are restated just far enough to drive
HipCodecPipeline the way zarr's Array layer would:

  Codec           to_dict() (src/zarr/abc/codec.py:99-225; bytes.py:68-72,
                  crc32c_.py:31-32, transpose.py:47-48, sharding.py:530-539)
  ZDType          to_native_dtype() (src/zarr/core/dtype/)
  ArrayConfig     order / write_empty_chunks / read_missing_chunks /
                  sharding_coalesce_* (src/zarr/core/array_spec.py:39-119)
  ArraySpec       shape, dtype (a ZDType), fill_value, config, prototype (137-186)
  Buffer          numpy-backed; from_bytes / as_numpy_array / as_array_like
                  (src/zarr/core/buffer/core.py:130-317, cpu.py)
  NDBuffer        numpy-backed; as_ndarray_like / as_numpy_array (core.py:320-567)
  BufferPrototype (buffer, nd_buffer) (core.py:570-586)
  MemoryStore     get_sync(key, *, prototype, byte_range) -> Buffer | None,
                  set_sync(key, Buffer) refusing anything else, delete_sync,
                  get_ranges_sync(..., prototype=...) (src/zarr/storage/_memory.py:110-146,
                  src/zarr/abc/store.py:474-539)
  StorePath       keyword-only get_sync / set_sync / delete_sync
                  (src/zarr/storage/_common.py:247-272)
  RangeByteRequest / SuffixByteRequest  (src/zarr/abc/store.py)
  ArrayV3Metadata codecs / chunk_grid.chunk_shape / data_type / fill_value
  V2Codec         filters + compressor (src/zarr/codecs/_v2.py:19-23), holding
                  numcodecs objects restated from numcodecs' published
                  algorithms (numcodecs is not installed here):
  NumGZip         numcodecs.GZip(level): a gzip member (mtime 0 here, so the
                  bytes are reproducible), decode of a gzip member
  NumDelta        numcodecs.Delta(dtype, astype): out[0] = a[0], out[i] =
                  a[i] - a[i-1] in astype; decode = cumulative sum in dtype
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, NamedTuple

import numpy as np


class FakeCodec:
    def __init__(self, d: dict, **attrs):
        self._d = d
        for k, v in attrs.items():
            setattr(self, k, v)

    def to_dict(self) -> dict:
        return self._d


def zcodecs(codecs: list) -> tuple:
    """JSON codec dicts -> Codec-like objects (sharding keeps its write order attr)."""
    out = []
    for c in codecs:
        if c["name"] == "sharding_indexed":
            conf = dict(c["configuration"])
            order = conf.pop("subchunk_write_order", "morton")
            conf["codecs"] = tuple(x.to_dict() for x in zcodecs(conf.get("codecs", [])))
            conf["index_codecs"] = tuple(x.to_dict() for x in zcodecs(
                conf.get("index_codecs", [{"name": "bytes", "configuration": {"endian": "little"}},
                                          {"name": "crc32c"}])))
            out.append(FakeCodec({"name": "sharding_indexed", "configuration": conf},
                                 subchunk_write_order=order))
        else:
            out.append(FakeCodec(dict(c)))
    return tuple(out)


class ZDType:
    def __init__(self, dtype):
        self._dt = np.dtype(dtype)

    def to_native_dtype(self) -> np.dtype:
        return self._dt

    def __repr__(self):
        return f"ZDType({self._dt})"


@dataclass(frozen=True)
class ArrayConfig:
    order: str = "C"
    write_empty_chunks: bool = False
    read_missing_chunks: bool = True
    sharding_coalesce_max_gap_bytes: int = 1 << 20
    sharding_coalesce_max_bytes: int = 16 << 20


class Buffer:
    def __init__(self, array_like):
        a = np.asarray(array_like)
        assert a.ndim == 1 and a.dtype == np.uint8
        self._data = a

    @classmethod
    def from_bytes(cls, b) -> "Buffer":
        return cls(np.frombuffer(bytes(b), dtype=np.uint8))

    @classmethod
    def from_buffer(cls, b) -> "Buffer":
        return cls(np.asarray(b.as_numpy_array()))

    def as_numpy_array(self) -> np.ndarray:
        return self._data

    def as_array_like(self):
        return self._data

    def to_bytes(self) -> bytes:
        return self._data.tobytes()

    def __getitem__(self, key: slice) -> "Buffer":
        return Buffer(self._data[key])

    def __len__(self) -> int:
        return self._data.size


class NDBuffer:
    def __init__(self, array):
        self._data = array

    @classmethod
    def create(cls, *, shape, dtype, order="C", fill_value=None):
        a = np.empty(shape, dtype=dtype, order=order)
        if fill_value is not None:
            a.fill(fill_value)
        return cls(a)

    @classmethod
    def from_numpy_array(cls, a) -> "NDBuffer":
        return cls(np.asarray(a))

    @classmethod
    def from_ndarray_like(cls, a) -> "NDBuffer":
        return cls(a)

    def as_ndarray_like(self):
        return self._data

    def as_numpy_array(self) -> np.ndarray:
        return np.asarray(self._data)

    @property
    def shape(self):
        return self._data.shape


class BufferPrototype(NamedTuple):
    buffer: type
    nd_buffer: type


cpu_prototype = BufferPrototype(Buffer, NDBuffer)


@dataclass(frozen=True)
class ArraySpec:
    shape: tuple
    dtype: Any
    fill_value: Any
    config: ArrayConfig
    prototype: Any

    @property
    def ndim(self):
        return len(self.shape)


@dataclass(frozen=True)
class RangeByteRequest:
    start: int
    end: int


@dataclass(frozen=True)
class SuffixByteRequest:
    suffix: int


class MemoryStore:
    """zarr MemoryStore's sync surface: Buffers in, Buffers out."""

    def __init__(self, d: dict | None = None):
        self._store_dict = {} if d is None else d
        self.calls = []

    def get_sync(self, key, *, prototype=None, byte_range=None):
        self.calls.append(("get", key, byte_range))
        v = self._store_dict.get(key)
        if v is None:
            return None
        n = len(v)
        if byte_range is None:
            a, b = 0, n
        elif hasattr(byte_range, "suffix"):
            a, b = max(0, n - byte_range.suffix), n
        else:
            a, b = byte_range.start, min(byte_range.end, n)
        return (prototype or cpu_prototype).buffer.from_bytes(v[a:b])

    def set_sync(self, key, value) -> None:
        if not isinstance(value, Buffer):
            raise TypeError(f"MemoryStore.set(): `value` must be a Buffer instance. Got {type(value)}")
        self._store_dict[key] = value.to_bytes()

    def delete_sync(self, key) -> None:
        self._store_dict.pop(key, None)

    def get_ranges_sync(self, key, byte_ranges, *, prototype, max_gap_bytes=1 << 20,
                        max_coalesced_bytes=16 << 20):
        out = []
        for i, r in enumerate(byte_ranges):
            v = self.get_sync(key, prototype=prototype, byte_range=r)
            if v is None:
                raise FileNotFoundError(key)
            out.append((i, v))
        return out


@dataclass(frozen=True)
class StorePath:
    store: MemoryStore
    path: str

    def get_sync(self, *, prototype=None, byte_range=None):
        return self.store.get_sync(self.path, prototype=prototype, byte_range=byte_range)

    def set_sync(self, value) -> None:
        self.store.set_sync(self.path, value)

    def delete_sync(self) -> None:
        self.store.delete_sync(self.path)


@dataclass
class RegularChunkGrid:
    chunk_shape: tuple


@dataclass
class ArrayV3Metadata:
    shape: tuple
    data_type: Any
    chunk_grid: RegularChunkGrid
    fill_value: Any
    codecs: tuple


def batch_for(meta_shape, chunk_shape, selection, store, spec):
    """The batch zarr's Array._get_selection / _set_selection builds
    (array.py:5393-5675): one (StorePath, ArraySpec, chunk_sel, out_sel,
    is_complete) per touched chunk, keys "c/i/j" (chunk_key_encodings.py:87-88)."""
    from oracle import oracle as O

    projections, out_shape = O.basic_indexer(selection if isinstance(selection, tuple) else (selection,),
                                             meta_shape, chunk_shape)
    batch = [(StorePath(store, "/".join(map(str, ("c",) + c))), spec, cs, os_, comp)
             for c, cs, os_, comp in projections]
    return batch, out_shape


class GzipCodec:
    """zarr's GzipCodec (src/zarr/codecs/gzip.py:31-95) as the pipeline sees it:
    a BytesBytesCodec instance whose sync methods run numcodecs.GZip through
    as_numpy_array_wrapper (src/zarr/core/buffer/cpu.py:194-219) -- here over
    the stdlib (numcodecs is absent).  Counts its calls."""

    is_fixed_size = False

    def __init__(self, *, level: int = 5):
        self.level = level
        self.calls = {"decode": 0, "encode": 0}

    def to_dict(self) -> dict:
        return {"name": "gzip", "configuration": {"level": self.level}}

    def evolve_from_array_spec(self, array_spec):
        return self

    def _decode_sync(self, chunk_bytes, chunk_spec):
        import gzip

        self.calls["decode"] += 1
        return chunk_spec.prototype.buffer.from_bytes(gzip.decompress(chunk_bytes.as_numpy_array().tobytes()))

    def _encode_sync(self, chunk_bytes, chunk_spec):
        import gzip

        self.calls["encode"] += 1
        return chunk_spec.prototype.buffer.from_bytes(
            gzip.compress(chunk_bytes.as_numpy_array().tobytes(), compresslevel=self.level, mtime=0))

    def compute_encoded_size(self, n, spec):
        raise NotImplementedError


class LzmaCodec(GzipCodec):
    """A compressor this package has no built-in for (zarr's numcodecs wrapper
    naming, "numcodecs.lzma"): only the instance can run it."""

    def to_dict(self) -> dict:
        return {"name": "numcodecs.lzma", "configuration": {"preset": 1}}

    def _decode_sync(self, chunk_bytes, chunk_spec):
        import lzma

        self.calls["decode"] += 1
        return chunk_spec.prototype.buffer.from_bytes(lzma.decompress(chunk_bytes.as_numpy_array().tobytes()))

    def _encode_sync(self, chunk_bytes, chunk_spec):
        import lzma

        self.calls["encode"] += 1
        return chunk_spec.prototype.buffer.from_bytes(
            lzma.compress(chunk_bytes.as_numpy_array().tobytes(), preset=1))


class ShardingCodec:
    """zarr's ShardingCodec instance surface (sharding.py:402-539): attributes
    holding the inner codec INSTANCES, plus to_dict."""

    def __init__(self, chunk_shape, codecs, index_codecs=None, index_location="end"):
        self.chunk_shape = tuple(chunk_shape)
        self.codecs = tuple(codecs)
        self.index_codecs = tuple(index_codecs or (FakeCodec({"name": "bytes", "configuration": {"endian": "little"}}),
                                                   FakeCodec({"name": "crc32c"})))
        self.index_location = index_location

    def to_dict(self) -> dict:
        return {"name": "sharding_indexed", "configuration": {
            "chunk_shape": list(self.chunk_shape), "codecs": [c.to_dict() for c in self.codecs],
            "index_codecs": [c.to_dict() for c in self.index_codecs], "index_location": self.index_location}}


class NumGZip:
    """numcodecs.GZip (level): encode -> a gzip member, decode -> its payload."""

    codec_id = "gzip"

    def __init__(self, level: int = 1):
        self.level = level

    def encode(self, buf):
        import gzip

        # ensure_contiguous_ndarray: the bytes in memory order (reshape order "A")
        data = np.ascontiguousarray(buf.reshape(-1, order="A")).view(np.uint8).tobytes() \
            if isinstance(buf, np.ndarray) else bytes(buf)
        return gzip.compress(data, compresslevel=self.level, mtime=0)

    def decode(self, buf, out=None):
        import gzip

        return gzip.decompress(bytes(buf))


class NumDelta:
    """numcodecs.Delta (dtype, astype)."""

    codec_id = "delta"

    def __init__(self, dtype, astype=None):
        self.dtype = np.dtype(dtype)
        self.astype = np.dtype(astype) if astype is not None else self.dtype

    def encode(self, buf):
        a = np.asarray(buf).reshape(-1, order="A")  # memory order, as ensure_ndarray + reshape
        a = np.ascontiguousarray(a).view(self.dtype)
        enc = np.empty_like(a, dtype=self.astype)
        if a.size:
            enc[0] = a[0]
            enc[1:] = np.diff(a).astype(self.astype)
        return enc

    def decode(self, buf, out=None):
        enc = np.frombuffer(bytes(buf), self.astype) if not isinstance(buf, np.ndarray) else \
            np.ascontiguousarray(buf).reshape(-1).view(self.astype)
        return np.cumsum(enc, dtype=self.dtype)


class V2Codec:
    """zarr's V2Codec (src/zarr/codecs/_v2.py:19-23): filters + compressor."""

    def __init__(self, filters=None, compressor=None):
        self.filters = tuple(filters) if filters else None
        self.compressor = compressor

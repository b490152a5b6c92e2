"""A thin Array driver over HipCodecPipeline (the caller side of the boundary).

Restates only what the hot path needs from the reference's Array layer:
  ArrayV3Metadata (zarr.json)      src/zarr/core/metadata/v3.py:464-613 (minimal reader/writer)
  create_codec_pipeline             src/zarr/core/array.py:221-265
  _get_selection                    src/zarr/core/array.py:5393-5514
  _set_selection                    src/zarr/core/array.py:5563-5675
  chunk key encodings               src/zarr/core/chunk_key_encodings.py:87-88 (default, "c/0/0"),
                                    103-105 (v2, "0.0"; "0" for 0-d)
"""

from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import buffer
from .codecs import BytesCodec, Crc32cCodec, ShardingCodec, parse_codecs
from .grid import ChunkGrid
from .indexing import basic_projections, chunk_batch
from .pipeline import DecodeProgram, HipCodecPipeline
from .spec import ArrayConfig, ArraySpec
from .store import DeviceStore, StorePath


def _fill_from_json(v, dtype: np.dtype):
    if isinstance(v, str):
        return np.array(float(v), dtype=dtype)[()]
    return np.array(v, dtype=dtype)[()]


def _fill_to_json(v, dtype: np.dtype):
    a = np.asarray(v, dtype=dtype)
    if dtype.kind == "f":
        f = float(a)
        if math.isnan(f):
            return "NaN"
        if math.isinf(f):
            return "Infinity" if f > 0 else "-Infinity"
        return f
    if dtype.kind == "b":
        return bool(a)
    return int(a)


def _selection_key(selection):
    """A hashable image of a basic selection (ints, unit or strided slices,
    Ellipsis), None for anything else (arrays, masks: not memoised)."""
    sel = selection if isinstance(selection, tuple) else (selection,)
    out = []
    for s in sel:
        if s is Ellipsis:
            out.append("...")
        elif isinstance(s, slice):
            if not all(v is None or isinstance(v, (int, np.integer)) for v in (s.start, s.stop, s.step)):
                return None
            out.append(("s", s.start, s.stop, s.step))
        elif isinstance(s, (int, np.integer)) and not isinstance(s, bool):
            out.append(int(s))
        else:
            return None
    return tuple(out)


@dataclass
class ArrayMetadata:
    shape: tuple[int, ...]
    chunk_shape: tuple[int, ...]
    dtype: np.dtype
    fill_value: Any
    codecs: tuple
    separator: str = "/"
    attributes: dict = field(default_factory=dict)
    key_encoding: str = "default"  # or "v2"
    # a rectilinear grid (chunk_grids.py:399-546); None: the regular grid of
    # chunk_shape.  With a rectilinear grid chunk_shape is the placeholder
    # (1,) * ndim zarr evolves the pipeline with (array.py:237-247)
    grid: ChunkGrid | None = None

    @property
    def chunk_grid(self) -> ChunkGrid:
        if self.grid is not None:
            return self.grid
        return ChunkGrid.from_sizes(self.shape, tuple(self.chunk_shape))

    @property
    def is_regular(self) -> bool:
        return self.grid is None or self.grid.is_regular

    def to_json(self) -> dict:
        return {
            "zarr_format": 3, "node_type": "array", "shape": list(self.shape),
            "data_type": np.dtype(self.dtype).name,
            "chunk_grid": self.chunk_grid.to_json() if self.grid is not None else
            {"name": "regular", "configuration": {"chunk_shape": list(self.chunk_shape)}},
            "chunk_key_encoding": {"name": self.key_encoding, "configuration": {"separator": self.separator}},
            "fill_value": _fill_to_json(self.fill_value, np.dtype(self.dtype)),
            "codecs": [c.to_dict() for c in self.codecs],
            "attributes": self.attributes,
        }

    @classmethod
    def from_json(cls, d: dict) -> "ArrayMetadata":
        if d.get("zarr_format") != 3 or d.get("node_type") != "array":
            raise ValueError("not a zarr v3 array")
        g = ChunkGrid.from_json(tuple(d["shape"]), d["chunk_grid"])
        dt = np.dtype(d["data_type"])
        cke = d.get("chunk_key_encoding", {"name": "default"})
        name = cke.get("name", "default")
        if name not in ("default", "v2"):
            raise NotImplementedError(f"chunk key encoding {name!r}")
        sep = (cke.get("configuration") or {}).get("separator", "/" if name == "default" else ".")
        chunk_shape = g.chunk_shape if g.is_regular else (1,) * g.ndim
        return cls(tuple(d["shape"]), chunk_shape, dt, _fill_from_json(d["fill_value"], dt),
                   tuple(parse_codecs(d["codecs"])), sep, d.get("attributes", {}), name,
                   None if g.is_regular else g)

    def chunk_key(self, coords) -> str:
        if self.key_encoding == "v2":
            k = self.separator.join(str(int(c)) for c in coords)
            return k or "0"
        return self.separator.join(map(str, ("c",) + tuple(int(c) for c in coords)))

    @property
    def grid_shape(self) -> tuple[int, ...]:
        if self.grid is not None:
            return self.grid.grid_shape
        return tuple(-(-s // c) for s, c in zip(self.shape, self.chunk_shape))


class Array:
    """zarr v3 array on a store, read/written through HipCodecPipeline."""

    def __init__(self, store_path: StorePath, metadata: ArrayMetadata,
                 config: ArrayConfig = ArrayConfig()):
        self.store_path = store_path
        self.metadata = metadata
        self.config = config
        # (rectilinear grids: the pipeline is evolved with the placeholder
        # shape, every chunk then carries its own spec -- array.py:237-247,
        # 5373-5390)
        self.spec = ArraySpec(metadata.chunk_shape, metadata.dtype, metadata.fill_value, config)
        self.codec_pipeline = HipCodecPipeline.from_codecs(metadata.codecs).evolve_from_array_spec(
            self.spec)
        if metadata.is_regular:
            self.codec_pipeline.validate(shape=metadata.shape, chunk_shape=metadata.chunk_shape)
        else:
            self.codec_pipeline.validate(shape=metadata.shape, chunk_grid=metadata.grid)
        self._programs: dict = {}

    # ------------------------------------------------------------ construction
    @classmethod
    def create(cls, store, shape, chunks, dtype, fill_value=0, codecs=None, *, shards=None,
               inner_codecs=None, index_location="end", path: str = "",
               config: ArrayConfig = ArrayConfig()) -> "Array":
        dtype = np.dtype(dtype)
        if codecs is None:
            codecs = (BytesCodec(endian="little" if dtype.itemsize > 1 else None),)
        codecs = tuple(parse_codecs(codecs))
        chunk_shape = tuple(c if isinstance(c, int) else tuple(c) for c in chunks)
        if shards is not None:
            inner = tuple(parse_codecs(inner_codecs)) if inner_codecs is not None else codecs
            codecs = (ShardingCodec(chunk_shape=chunk_shape, codecs=inner,
                                    index_location=index_location),)
            chunk_shape = tuple(c if isinstance(c, int) else tuple(c) for c in shards)
        # nested edge lists: a rectilinear grid (regular when they reduce to one)
        grid = None
        if any(not isinstance(c, int) for c in chunk_shape):
            grid = ChunkGrid.from_sizes(tuple(shape), chunk_shape)
            chunk_shape = grid.chunk_shape if grid.is_regular else (1,) * len(chunk_shape)
            grid = None if grid.is_regular else grid
        md = ArrayMetadata(tuple(shape), chunk_shape, dtype, np.array(fill_value, dtype)[()],
                           codecs, grid=grid)
        sp = StorePath(store, path)
        key = f"{path}/zarr.json" if path else "zarr.json"
        store.set_sync(key, json.dumps(md.to_json()).encode())
        return cls(sp, md, config)

    @classmethod
    def open(cls, store, path: str = "", config: ArrayConfig = ArrayConfig()) -> "Array":
        key = f"{path}/zarr.json" if path else "zarr.json"
        raw = store.get_sync(key)
        if raw is None:
            raise FileNotFoundError(key)
        d = json.loads(bytes(raw))
        return cls(StorePath(store, path), ArrayMetadata.from_json(d), config)

    # ---------------------------------------------------------------- helpers
    @property
    def shape(self):
        return self.metadata.shape

    @property
    def dtype(self):
        return self.metadata.dtype

    @property
    def chunks(self):
        """The chunk shape; only defined for regular chunk grids -- a
        rectilinear grid raises NotImplementedError, as the reference's
        Array.chunks does (src/zarr/core/array.py:849-862, 2024-2036)."""
        if not self.metadata.is_regular:
            raise NotImplementedError("chunks is only defined for arrays using a regular chunk grid; "
                                      "this array uses a rectilinear chunk grid")
        return self.metadata.chunk_shape

    def _key(self, coords) -> str:
        k = self.metadata.chunk_key(coords)
        return f"{self.store_path.path}/{k}" if self.store_path.path else k

    def batch_info(self, selection):
        """The CodecPipeline batch of a selection (BasicIndexer's chunk
        projections, src/zarr/core/indexing.py:365-621).  Depends only on the
        metadata and the selection, so basic selections are memoised per array
        (a repeated read skips the indexer: the per-call path)."""
        key = _selection_key(selection)
        cache = self.__dict__.setdefault("_batches", {})
        if key is not None:
            hit = cache.get(key)
            if hit is not None:
                return list(hit[0]), hit[1]
        batch, out_shape = self._batch_info(selection)
        if key is not None:
            if len(cache) >= 64:
                cache.pop(next(iter(cache)))
            cache[key] = (tuple(batch), out_shape)
        return batch, out_shape

    def _batch_info(self, selection):
        md = self.metadata
        if not md.is_regular:
            return self._batch_info_rectilinear(selection)
        rows, out_shape = chunk_batch(selection, self.metadata.shape, self.metadata.chunk_shape)
        store, spec, sep = self.store_path.store, self.spec, self.metadata.separator
        if self.metadata.key_encoding == "v2":
            pre = f"{self.store_path.path}/" if self.store_path.path else ""
            batch = [(StorePath(store, pre + (sep.join(map(str, co)) or "0")), spec, csel, osel, comp)
                     for co, csel, osel, comp in rows]
            return batch, out_shape
        prefix = f"{self.store_path.path}/c" if self.store_path.path else "c"
        batch = [(StorePath(store, sep.join([prefix, *map(str, co)])), spec, csel, osel, comp)
                 for co, csel, osel, comp in rows]
        return batch, out_shape

    def _batch_info_rectilinear(self, selection):
        """_get_selection's batch for a rectilinear grid: one ArraySpec per
        chunk, shape = ChunkGrid[coords].codec_shape (_get_chunk_spec,
        array.py:5373-5390, 5469-5486); specs of equal shape are shared."""
        md = self.metadata
        g = md.grid
        rows, out_shape = chunk_batch(selection, md.shape, g)
        store, sep = self.store_path.store, md.separator
        specs: dict = {}
        batch = []
        for co, csel, osel, comp in rows:
            cs = g.codec_shape(co)
            sp = specs.get(cs)
            if sp is None:
                sp = specs[cs] = ArraySpec(cs, md.dtype, md.fill_value, self.config)
            batch.append((StorePath(store, self._key(co)), sp, csel, osel, comp))
        return batch, out_shape

    # ------------------------------------------------------------------- read
    def prepare_read(self, selection=Ellipsis, out=None, device=None) -> tuple[DecodeProgram, Any]:
        """Plan a selection once; the returned program re-launches without re-planning."""
        import torch

        batch, out_shape = self.batch_info(selection)
        if out is None:
            dev = device or getattr(self.store_path.store, "device", None) or torch.device("cuda:0")
            out = buffer.empty(out_shape, self.metadata.dtype, dev, self.config.order)
        prog = self.codec_pipeline.prepare_read(batch, out)
        return prog, out

    def get(self, selection=Ellipsis, out=None, device=None):
        """Device-resident read: returns a torch tensor on the GPU."""
        batch, out_shape = self.batch_info(selection)
        import torch

        if out is None:
            dev = device or getattr(self.store_path.store, "device", None) or torch.device("cuda:0")
            out = buffer.empty(out_shape, self.metadata.dtype, dev, self.config.order)
        if not batch:
            return out
        results = self.codec_pipeline.read_sync(batch, out)
        if not self.config.read_missing_chunks:
            for (bg, *_), r in zip(batch, results):
                if r["status"] == "missing":
                    raise ChunkNotFoundError(f"chunk {bg.path!r} is missing")
        return out

    def __getitem__(self, selection) -> np.ndarray:
        """Host result.  Host-resident stores read into a pinned numpy array:
        the pipeline streams slabs back while later slabs still decode
        (HipCodecPipeline._read_slabs); HBM-resident stores decode on the
        device and copy the result back once."""
        st = self.store_path.store
        if isinstance(st, DeviceStore):
            return buffer.to_numpy(self.get(selection), self.metadata.dtype)
        batch, out_shape = self.batch_info(selection)
        out = buffer.empty_pinned(out_shape, self.metadata.dtype, self.config.order)
        if not batch:
            return out
        results = self.codec_pipeline.read_sync(batch, out)
        if not self.config.read_missing_chunks:
            for (bg, *_), r in zip(batch, results):
                if r["status"] == "missing":
                    raise ChunkNotFoundError(f"chunk {bg.path!r} is missing")
        return out

    # ------------------------------------------------------------------ write
    def set(self, selection, value) -> None:
        """Array._set_selection (array.py:5563-5675): value may be a device
        tensor, a numpy array or a scalar."""
        batch, out_shape = self.batch_info(selection)
        if not batch:
            return
        import torch

        if not isinstance(value, torch.Tensor):
            a = np.asarray(value, dtype=self.metadata.dtype)
            if a.shape not in ((), tuple(out_shape)):
                a = np.broadcast_to(a, out_shape)
            value = a
        self.codec_pipeline.write_sync(batch, value)

    def __setitem__(self, selection, value) -> None:
        self.set(selection, value)


class ChunkNotFoundError(KeyError):
    """array.py:5496-5511 (read_missing_chunks=False)."""

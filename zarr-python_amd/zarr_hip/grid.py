"""Chunk grids: regular and rectilinear (src/zarr/core/chunk_grids.py).

zarr builds one ArraySpec per chunk from ``ChunkGrid[coords].codec_shape``
when the grid is not regular (``_get_chunk_spec``, src/zarr/core/array.py:
5373-5390, 5469-5486), so a batch handed to ``HipCodecPipeline.read`` can
carry chunks of different shapes.  This module restates the grid the host
side needs to build such batches (the package's own ``Array``) and to check
the indexer's projections:

  FixedDimension     chunk_grids.py:73-164   (boundary chunks encoded at full size)
  VaryingDimension   chunk_grids.py:167-293  (explicit edges, prefix sums)
  ChunkSpec          chunk_grids.py:319-341  (slices + codec_shape)
  ChunkGrid          chunk_grids.py:399-546  (from_sizes, __getitem__, grid_shape)
  expand_rle         src/zarr/core/common.py:272-295
  rectilinear JSON   src/zarr/core/metadata/v3.py:276-366
"""

from __future__ import annotations

import bisect
import itertools
from dataclasses import dataclass
from typing import Sequence


def _ceildiv(a: int, b: int) -> int:
    return -(-a // b)


@dataclass(frozen=True)
class FixedDimension:
    """Uniform chunk size; the last chunk's data is clipped at the extent but it
    is encoded at full size (chunk_grids.py:73-130)."""

    size: int
    extent: int

    def __post_init__(self):
        if self.size < 0:
            raise ValueError(f"FixedDimension size must be >= 0, got {self.size}")
        if self.extent < 0:
            raise ValueError(f"FixedDimension extent must be >= 0, got {self.extent}")

    @property
    def nchunks(self) -> int:
        return 0 if self.size == 0 else _ceildiv(self.extent, self.size)

    def index_to_chunk(self, idx: int) -> int:
        if idx < 0:
            raise IndexError(f"Negative index {idx} is not allowed")
        if idx >= self.extent:
            raise IndexError(f"Index {idx} is out of bounds for extent {self.extent}")
        return 0 if self.size == 0 else idx // self.size

    def chunk_offset(self, ix: int) -> int:
        return ix * self.size

    def chunk_size(self, ix: int) -> int:
        return self.size

    def data_size(self, ix: int) -> int:
        if self.size == 0:
            return 0
        return max(0, min(self.size, self.extent - ix * self.size))

    @property
    def unique_edge_lengths(self) -> tuple[int, ...]:
        return (self.size,)


@dataclass(frozen=True, init=False)
class VaryingDimension:
    """Explicit per-chunk edges (chunk_grids.py:167-293).  The last chunk may
    reach past the extent: data_size clips, chunk_size does not."""

    edges: tuple[int, ...]
    cumulative: tuple[int, ...]
    extent: int

    def __init__(self, edges: Sequence[int], extent: int):
        e = tuple(int(x) for x in edges)
        if not e:
            raise ValueError("VaryingDimension edges must not be empty")
        if any(x <= 0 for x in e):
            raise ValueError(f"All edge lengths must be > 0, got {e}")
        cum = tuple(itertools.accumulate(e))
        if extent < 0:
            raise ValueError(f"VaryingDimension extent must be >= 0, got {extent}")
        if extent > cum[-1]:
            raise ValueError(f"VaryingDimension extent {extent} exceeds sum of edges {cum[-1]}")
        object.__setattr__(self, "edges", e)
        object.__setattr__(self, "cumulative", cum)
        object.__setattr__(self, "extent", int(extent))

    @property
    def nchunks(self) -> int:
        # chunks that overlap [0, extent) (chunk_grids.py:199-205)
        return 0 if self.extent == 0 else bisect.bisect_left(self.cumulative, self.extent) + 1

    def index_to_chunk(self, idx: int) -> int:
        if idx < 0 or idx >= self.extent:
            raise IndexError(f"Index {idx} out of bounds for dimension with extent {self.extent}")
        return bisect.bisect_right(self.cumulative, idx)

    def chunk_offset(self, ix: int) -> int:
        return self.cumulative[ix - 1] if ix > 0 else 0

    def chunk_size(self, ix: int) -> int:
        return self.edges[ix]

    def data_size(self, ix: int) -> int:
        off = self.cumulative[ix - 1] if ix > 0 else 0
        return max(0, min(self.edges[ix], self.extent - off))

    def indices_to_chunks(self, indices):
        import numpy as np

        return np.searchsorted(self.cumulative, indices, side="right")

    @property
    def unique_edge_lengths(self) -> tuple[int, ...]:
        return tuple(dict.fromkeys(self.edges))


@dataclass(frozen=True)
class ChunkSpec:
    """chunk_grids.py:319-341: the chunk's data region and its codec shape."""

    slices: tuple
    codec_shape: tuple[int, ...]

    @property
    def shape(self) -> tuple[int, ...]:
        return tuple(s.stop - s.start for s in self.slices)

    @property
    def is_boundary(self) -> bool:
        return self.shape != self.codec_shape


def expand_rle(data) -> list[int]:
    """common.py:272-295: bare edge lengths and [size, count] runs."""
    out: list[int] = []
    for item in data:
        if isinstance(item, (int, float)) and not isinstance(item, bool):
            v = int(item)
            if v < 1:
                raise ValueError(f"Chunk edge length must be >= 1, got {v}")
            out.append(v)
        elif isinstance(item, (list, tuple)) and len(item) == 2:
            size, count = int(item[0]), int(item[1])
            if size < 1:
                raise ValueError(f"Chunk edge length must be >= 1, got {size}")
            if count < 1:
                raise ValueError(f"RLE repeat count must be >= 1, got {count}")
            out.extend([size] * count)
        else:
            raise ValueError(f"RLE entries must be an integer or [size, count], got {item}")
    return out


def compress_rle(sizes: Sequence[int]) -> list:
    """common.py:298-320: runs of length > 1 as [value, count]."""
    out: list = []
    for v, grp in itertools.groupby(int(s) for s in sizes):
        n = len(list(grp))
        out.append([v, n] if n > 1 else v)
    return out


@dataclass(frozen=True)
class ChunkGrid:
    """chunk_grids.py:399-546 (the parts the hot path and its host planner use)."""

    dimensions: tuple

    @classmethod
    def from_sizes(cls, array_shape, chunk_sizes) -> "ChunkGrid":
        """chunk_grids.py:448-487: an int per dim is regular; a list of edges is
        regular when every edge is equal and they cover the extent, else
        varying."""
        extents = tuple(int(s) for s in array_shape)
        if len(extents) != len(chunk_sizes):
            raise ValueError(f"array_shape has {len(extents)} dimensions but chunk_sizes "
                             f"has {len(chunk_sizes)} dimensions")
        dims = []
        for spec, extent in zip(chunk_sizes, extents):
            if isinstance(spec, int):
                dims.append(FixedDimension(int(spec), extent))
                continue
            edges = [int(e) for e in spec]
            if not edges:
                raise ValueError("Each dimension must have at least one chunk")
            if edges[0] > 0 and all(e == edges[0] for e in edges) and (
                    extent == sum(edges) or len(edges) == _ceildiv(extent, edges[0])):
                dims.append(FixedDimension(edges[0], extent))
            else:
                dims.append(VaryingDimension(edges, extent))
        return cls(tuple(dims))

    @classmethod
    def from_json(cls, shape, grid: dict) -> "ChunkGrid":
        """A v3 ``chunk_grid`` object: "regular" (chunk_shape) or "rectilinear"
        (kind "inline", chunk_shapes of ints / RLE lists; metadata/v3.py:350-366)."""
        name, conf = grid["name"], grid.get("configuration") or {}
        if name == "regular":
            return cls.from_sizes(shape, tuple(int(c) for c in conf["chunk_shape"]))
        if name == "rectilinear":
            kind = conf.get("kind")
            if kind not in (None, "inline"):
                raise ValueError(f"Unsupported rectilinear chunk grid kind: {kind!r}")
            dims = []
            for d in conf["chunk_shapes"]:
                if isinstance(d, int):
                    if d < 1:
                        raise ValueError(f"Integer chunk edge length must be >= 1, got {d}")
                    dims.append(d)
                elif isinstance(d, list):
                    dims.append(tuple(expand_rle(d)))
                else:
                    raise TypeError(f"Invalid chunk_shapes entry: expected int or list, got {type(d)}")
            return cls.from_sizes(shape, dims)
        raise NotImplementedError(f"chunk grid {name!r}")

    def to_json(self) -> dict:
        if self.is_regular:
            return {"name": "regular", "configuration": {"chunk_shape": list(self.chunk_shape)}}
        dims = []
        for d in self.dimensions:
            if isinstance(d, FixedDimension):
                dims.append(d.size)
            else:
                rle = compress_rle(d.edges)
                dims.append(rle if len(rle) < len(d.edges) else list(d.edges))
        return {"name": "rectilinear", "configuration": {"kind": "inline", "chunk_shapes": dims}}

    @property
    def ndim(self) -> int:
        return len(self.dimensions)

    @property
    def is_regular(self) -> bool:
        return all(isinstance(d, FixedDimension) for d in self.dimensions)

    @property
    def grid_shape(self) -> tuple[int, ...]:
        return tuple(d.nchunks for d in self.dimensions)

    @property
    def chunk_shape(self) -> tuple[int, ...]:
        if not self.is_regular:
            raise ValueError("chunk_shape is only available for regular chunk grids. "
                             "Use grid[coords] for per-chunk sizes.")
        return tuple(d.size for d in self.dimensions)

    @property
    def shape(self) -> tuple[int, ...]:
        return tuple(d.extent for d in self.dimensions)

    def __getitem__(self, coords) -> ChunkSpec | None:
        """chunk_grids.py:528-546: None out of bounds."""
        if isinstance(coords, int):
            coords = (coords,)
        if len(coords) != self.ndim:
            raise ValueError(f"Expected {self.ndim} coordinate(s) for a {self.ndim}-d chunk grid, "
                             f"got {len(coords)}.")
        slices, cshape = [], []
        for d, ix in zip(self.dimensions, coords):
            if ix < 0 or ix >= d.nchunks:
                return None
            off = d.chunk_offset(ix)
            slices.append(slice(off, off + d.data_size(ix), 1))
            cshape.append(d.chunk_size(ix))
        return ChunkSpec(tuple(slices), tuple(cshape))

    def codec_shape(self, coords) -> tuple[int, ...]:
        return tuple(d.chunk_size(int(ix)) for d, ix in zip(self.dimensions, coords))

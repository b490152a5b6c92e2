"""Rectilinear chunk grids on the CPU: zarr_hip.grid and the oracle's grid
restatement against the reference's literal cases
(tests/test_unified_chunk_grid.py:207-260, 340-400), the reference's
rectilinear metadata fixture (packages/zarr-metadata/tests/v3/array/
rectilinear_grid.json), the package's indexer against the oracle's over
varying dimensions, and the pipeline's grouping of a batch by chunk spec
(src/zarr/core/array.py:5373-5390, 5469-5486).  GPU reads and writes of the
same grids: tests/test_gpu_rectilinear.py."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.join(os.path.dirname(__file__), "golden", "metadata")


def test_varying_dimension_construction():
    from zarr_hip.grid import VaryingDimension

    d = VaryingDimension([10, 20, 30], extent=60)
    assert d.edges == (10, 20, 30)
    assert d.cumulative == (10, 30, 60)
    assert d.nchunks == 3
    assert d.extent == 60
    o = O.VaryingDim([10, 20, 30], 60)
    assert o.cumulative == (10, 30, 60) and o.nchunks == 3


@pytest.mark.parametrize("ix,off,size,data,first", [(0, 0, 10, 10, 0), (1, 10, 20, 20, 1), (2, 30, 30, 30, 2)])
def test_varying_dimension(ix, off, size, data, first):
    from zarr_hip.grid import VaryingDimension

    for d in (VaryingDimension([10, 20, 30], extent=60), O.VaryingDim([10, 20, 30], 60)):
        assert d.chunk_offset(ix) == off
        assert d.chunk_size(ix) == size
        assert d.data_size(ix) == data
        assert d.index_to_chunk(off) == first


def test_varying_dimension_indices_to_chunks():
    from zarr_hip.grid import VaryingDimension

    d = VaryingDimension([10, 20, 30], extent=60)
    np.testing.assert_array_equal(d.indices_to_chunks(np.array([0, 9, 10, 29, 30, 59])), [0, 0, 1, 1, 2, 2])
    o = O.VaryingDim([10, 20, 30], 60)
    assert [o.index_to_chunk(i) for i in (0, 9, 10, 29, 30, 59)] == [0, 0, 1, 1, 2, 2]


@pytest.mark.parametrize("edges,extent,match", [([], 0, "must not be empty"), ([10, 0, 5], 15, "must be > 0")])
def test_varying_dimension_rejects_invalid(edges, extent, match):
    from zarr_hip.grid import VaryingDimension

    with pytest.raises(ValueError, match=match):
        VaryingDimension(edges, extent=extent)
    with pytest.raises(ValueError, match=match):
        O.VaryingDim(edges, extent)


def test_varying_dimension_extent_past_edges():
    """The last chunk may reach past the extent: data_size clips, chunk_size
    (the codec shape) does not (chunk_grids.py:167-173)."""
    from zarr_hip.grid import VaryingDimension

    for d in (VaryingDimension([10, 20, 30], extent=45), O.VaryingDim([10, 20, 30], 45)):
        assert d.nchunks == 3 and d.data_size(2) == 15 and d.chunk_size(2) == 30
    for d in (VaryingDimension([10, 20, 30], extent=25), O.VaryingDim([10, 20, 30], 25)):
        assert d.nchunks == 2 and d.data_size(1) == 15


@pytest.mark.parametrize("shape,chunks,grid_shape", [
    ((100, 200), (10, 20), (10, 10)),
    ((95, 200), (10, 20), (10, 10)),
    ((60, 100), [[10, 20, 30], [25, 25, 25, 25]], (3, 4)),
])
def test_chunk_grid_shape(shape, chunks, grid_shape):
    from zarr_hip.grid import ChunkGrid

    assert ChunkGrid.from_sizes(shape, chunks).grid_shape == grid_shape
    assert tuple(d.nchunks for d in O.grid_dims(shape, chunks)) == grid_shape


@pytest.mark.parametrize("shape,chunks,coords,exp_shape,exp_codec,boundary", [
    ((100, 200), (10, 20), (0, 0), (10, 20), (10, 20), False),
    ((95, 200), (10, 20), (9, 0), (5, 20), (10, 20), True),
    ((60, 100), [[10, 20, 30], [25, 25, 25, 25]], (0, 0), (10, 25), (10, 25), False),
    ((60, 100), [[10, 20, 30], [25, 25, 25, 25]], (1, 0), (20, 25), (20, 25), False),
    ((60, 100), [[10, 20, 30], [25, 25, 25, 25]], (2, 3), (30, 25), (30, 25), False),
])
def test_chunk_grid_getitem(shape, chunks, coords, exp_shape, exp_codec, boundary):
    from zarr_hip.grid import ChunkGrid

    spec = ChunkGrid.from_sizes(shape, chunks)[coords]
    assert spec.shape == exp_shape and spec.codec_shape == exp_codec and spec.is_boundary == boundary
    sl, cs = O.grid_getitem(O.grid_dims(shape, chunks), coords)
    assert tuple(s.stop - s.start for s in sl) == exp_shape and cs == exp_codec


@pytest.mark.parametrize("shape,chunks,coords", [((100, 200), (10, 20), (99, 0)),
                                                 ((60, 100), [[10, 20, 30], [25, 25, 25, 25]], (3, 0))])
def test_chunk_grid_getitem_oob(shape, chunks, coords):
    from zarr_hip.grid import ChunkGrid

    assert ChunkGrid.from_sizes(shape, chunks)[coords] is None
    assert O.grid_getitem(O.grid_dims(shape, chunks), coords) is None


def test_equal_edges_collapse_to_regular():
    """chunk_grids.py:476-487: equal edges covering the extent are a FixedDimension."""
    from zarr_hip.grid import ChunkGrid, FixedDimension, VaryingDimension

    g = ChunkGrid.from_sizes((100, 100), [[25, 25, 25, 25], [30, 30, 30, 30]])
    assert isinstance(g.dimensions[0], FixedDimension) and isinstance(g.dimensions[1], FixedDimension)
    assert g.is_regular and g.chunk_shape == (25, 30)
    g = ChunkGrid.from_sizes((100,), [[30, 30, 40]])
    assert isinstance(g.dimensions[0], VaryingDimension) and not g.is_regular


def test_rle():
    """common.py:272-320."""
    from zarr_hip.grid import compress_rle, expand_rle

    assert expand_rle([[10, 3], 5]) == [10, 10, 10, 5]
    assert compress_rle([10, 10, 10, 5]) == [[10, 3], 5]
    with pytest.raises(ValueError):
        expand_rle([[0, 2]])


def test_rectilinear_fixture():
    """The reference's rectilinear metadata document: 100 x 100 f64, rows
    10/20/30/40, columns 50."""
    from zarr_hip import ArrayMetadata

    with open(os.path.join(HERE, "rectilinear_grid.json")) as fh:
        d = json.load(fh)
    md = ArrayMetadata.from_json(d)
    g = md.grid
    assert md.shape == (100, 100) and md.dtype == np.dtype("float64") and not md.is_regular
    assert md.grid_shape == (4, 2)
    assert [g.codec_shape((i, 0)) for i in range(4)] == [(10, 50), (20, 50), (30, 50), (40, 50)]
    assert g[(2, 1)].slices == (slice(30, 60, 1), slice(50, 100, 1))
    back = ArrayMetadata.from_json(md.to_json())
    assert back.grid == md.grid
    assert md.to_json()["chunk_grid"] == {"name": "rectilinear", "configuration": {
        "kind": "inline", "chunk_shapes": [[10, 20, 30, 40], 50]}}


SELECTIONS = [(Ellipsis,), (slice(5, 77), slice(None)), (slice(3, 97, 7), slice(1, 99, 3)), (33, slice(None)),
              (slice(None), 49), (slice(29, 31), slice(50, 51)), (slice(60, 60), slice(None))]


@pytest.mark.parametrize("sel", SELECTIONS)
@pytest.mark.parametrize("chunks", [[[10, 20, 30, 40], 50], [[10, 20, 30, 40], [7, 93]], [[1, 99], [[3, 30], 10]]])
def test_projections_match_oracle(sel, chunks):
    """zarr_hip.indexing.chunk_batch over a rectilinear grid == the oracle's
    BasicIndexer restatement (indexing.py:369-468 over DimensionGrid)."""
    from zarr_hip.grid import ChunkGrid, expand_rle
    from zarr_hip.indexing import chunk_batch

    chunks = [c if isinstance(c, int) else expand_rle(c) for c in chunks]
    g = ChunkGrid.from_sizes((100, 100), chunks)
    rows, out_shape = chunk_batch(sel, (100, 100), g)
    want, want_shape = O.basic_indexer(sel, (100, 100), O.grid_dims((100, 100), chunks))
    assert out_shape == want_shape

    def norm(sel):  # the same index sets (the package writes tight slice stops)
        return tuple(s if isinstance(s, int) else tuple(range(s.start, s.stop, s.step or 1)) for s in sel)
    assert [(tuple(r[0]), norm(r[1]), norm(r[2]), r[3]) for r in rows] == \
        [(w[0], norm(w[1]), norm(w[2]), w[3]) for w in want]


def test_spec_groups():
    """A batch is grouped by chunk spec in first-seen order; one shared spec
    (a regular grid) is not grouped at all, nor are equal specs that are
    different objects."""
    from zarr_hip.pipeline import normalize_batch, spec_groups
    from zarr_hip.spec import ArraySpec

    a = ArraySpec((10, 50), np.dtype("f8"), 0.0)
    b = ArraySpec((20, 50), np.dtype("f8"), 0.0)
    a2 = ArraySpec((10, 50), np.dtype("f8"), 0.0)
    c = ArraySpec((10, 50), np.dtype("f8"), 1.0)
    sel = (slice(0, 1),) * 2
    mk = lambda sp: (None, sp, sel, sel, True)  # noqa: E731
    assert spec_groups([mk(a), mk(a), mk(a)]) is None
    assert spec_groups([mk(a), mk(a2)]) is None
    assert spec_groups([mk(a), mk(b), mk(a2), mk(b), mk(c)]) == [[0, 2], [1, 3], [4]]
    # zarr's spec objects are coerced once per object
    import zarr_fakes as Z

    zs = Z.ArraySpec((10, 50), Z.ZDType("float64"), 0.0, Z.ArrayConfig(), None)
    nb = normalize_batch([mk(zs), mk(zs)])
    assert nb[0][1] is nb[1][1]


def test_oracle_rectilinear_roundtrip():
    """The oracle writes and reads a rectilinear array: every chunk encoded at
    its own codec shape (the last past the extent at full edge)."""
    meta = O.ArrayMeta((100, 95), ([10, 20, 30, 40], [50, 50]), np.dtype("float64"), 0.0,
                       codecs=[{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}])
    rng = np.random.default_rng(0)
    data = rng.standard_normal((100, 95))
    store: dict = {}
    O.write(store, meta, (Ellipsis,), data)
    assert len(store["c/2/1"]) == 30 * 50 * 8 + 4
    assert len(store["c/0/0"]) == 10 * 50 * 8 + 4
    np.testing.assert_array_equal(O.read(store, meta), data)
    np.testing.assert_array_equal(O.read(store, meta, (slice(5, 66, 3), slice(40, 60))), data[5:66:3, 40:60])


def test_array_chunks_raises_for_rectilinear():
    """Array.chunks is defined for regular grids only; a rectilinear grid
    raises NotImplementedError (src/zarr/core/array.py:849-862), where it
    used to return the internal placeholder (1,) * ndim (advisor round 5)."""
    import zarr_hip

    store = zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, (30, 30), ([10, 20], [20, 10]), "float32", 0.0)
    with pytest.raises(NotImplementedError):
        arr.chunks
    reg = zarr_hip.Array.create(zarr_hip.MemoryStore(), (30, 30), (10, 10), "float32", 0.0)
    assert reg.chunks == (10, 10)

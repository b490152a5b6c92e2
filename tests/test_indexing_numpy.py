"""The host indexer (zarr_hip.indexing.chunk_batch, BasicIndexer's projections)
against numpy's own basic indexing, which zarr's BasicIndexer follows
(src/zarr/core/indexing.py:333-468: negative integers wrap, slices normalise
through slice.indices, Ellipsis and missing trailing dims expand): for random
shapes, regular and rectilinear chunk grids and selections with negative
integers, negative or out-of-range slice bounds, None bounds and steps, the
result assembled chunk by chunk from the projections equals full[selection];
out-of-bounds integers, negative and zero steps raise as the reference does
(BoundsCheckError / NegativeStepError are IndexErrors; a zero step is
slice.indices' ValueError).  CPU only."""

import numpy as np
import pytest

from zarr_hip.indexing import chunk_batch


def _bound(rng, n):
    r = rng.random()
    if r < 0.2:
        return None
    return int(rng.integers(-n - 3, n + 4))


def _dim_sel(rng, n):
    r = rng.random()
    if r < 0.25:
        return int(rng.integers(-n, n))
    step = None if rng.random() < 0.4 else int(rng.choice([1, 2, 3, 5]))
    return slice(_bound(rng, n), _bound(rng, n), step)


def _selection(rng, shape):
    sel = [_dim_sel(rng, n) for n in shape]
    r = rng.random()
    if r < 0.15 and len(sel) > 1:
        return tuple(sel[: int(rng.integers(1, len(sel)))])  # trailing dims implied
    if r < 0.3:
        k = int(rng.integers(0, len(sel) + 1))
        return tuple(sel[:k]) + (Ellipsis,) + tuple(sel[k + 1:])
    return tuple(sel)


def _assemble(full, batch, out_shape, grid_offsets):
    out = np.empty(out_shape, full.dtype)
    for coords, csel, osel, _ in batch:
        region = tuple(slice(o[c], o[c + 1]) for c, o in zip(coords, grid_offsets))
        out[osel] = full[region][csel]
    return out


def _offsets(shape, chunks):
    offs = []
    for n, c in zip(shape, chunks):
        if isinstance(c, int):
            offs.append(list(range(0, n, c)) + [n])
        else:
            o = [0]
            for e in c:
                o.append(min(n, o[-1] + e))
            offs.append(o)
    return offs


@pytest.mark.parametrize("seed", range(300))
def test_chunk_batch_matches_numpy(seed):
    rng = np.random.default_rng(31000 + seed)
    nd = int(rng.integers(1, 4))
    shape = tuple(int(rng.integers(1, 41)) for _ in range(nd))
    full = np.arange(int(np.prod(shape)), dtype=np.int32).reshape(shape)
    rect = seed % 3 == 2
    if rect:
        chunks = []
        for n in shape:
            e, t = [], 0
            while t < n:
                e.append(int(rng.integers(1, 9)))
                t += e[-1]
            chunks.append(tuple(e))
        from zarr_hip.grid import ChunkGrid

        grid = ChunkGrid.from_sizes(shape, tuple(chunks))
        offs = _offsets(shape, chunks)
    else:
        chunks = tuple(int(rng.integers(1, 13)) for _ in range(nd))
        grid = chunks
        offs = _offsets(shape, chunks)
    for _ in range(8):
        sel = _selection(rng, shape)
        want = full[sel]
        batch, out_shape = chunk_batch(sel, shape, grid)
        assert tuple(out_shape) == want.shape, (sel, shape, chunks)
        got = _assemble(full, batch, out_shape, offs)
        assert np.array_equal(got, want), (sel, shape, chunks)


@pytest.mark.parametrize("sel,exc", [
    ((10,), IndexError), ((-11,), IndexError), ((slice(None, None, -1),), IndexError),
    ((slice(2, 8, -2),), IndexError), ((slice(None, None, 0),), ValueError),
    ((1, 2), IndexError),  # too many indices for a 1-d array
])
def test_chunk_batch_errors_as_reference(sel, exc):
    with pytest.raises(exc):
        chunk_batch(sel, (10,), (4,))


def test_out_of_bounds_message():
    """BoundsCheckError's text (indexing.py:342-344)."""
    with pytest.raises(IndexError, match="index out of bounds for dimension with length 10"):
        chunk_batch((12,), (10,), (4,))

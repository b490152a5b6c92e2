"""Selection -> per-chunk projections for regular chunk grids (host planner input).

Semantics follow the reference's BasicIndexer (src/zarr/core/indexing.py:571-621),
IntDimIndexer (365-385) and SliceDimIndexer (388-468), with boundary chunks
stored at full size (FixedDimension.data_size, src/zarr/core/chunk_grids.py:119-130).
The projections are produced per dimension as numpy arrays and combined by a
cartesian product, so planning 10^4-10^5 chunks stays vectorised.
"""

from __future__ import annotations

import itertools
from dataclasses import dataclass

import numpy as np


def _ceildiv(a, b):
    return -(-a // b)


@dataclass
class DimProjection:
    """Projections of one selection item onto one chunked dimension."""

    chunk_ix: np.ndarray   # int64[k]
    sel_start: np.ndarray  # int64[k]   first selected index inside the chunk
    sel_count: np.ndarray  # int64[k]
    step: int
    out_start: np.ndarray  # int64[k]   position along the out dim (0 for int selections)
    complete: np.ndarray   # bool[k]
    dropped: bool          # integer selection: the dim is absent from out
    nitems: int


def normalize_selection(selection, shape: tuple[int, ...]) -> tuple:
    """replace_ellipsis (indexing.py:458-496) + integer normalisation."""
    if not isinstance(selection, tuple):
        selection = (selection,)
    sel = list(selection)
    n_ell = sum(1 for s in sel if s is Ellipsis)
    if n_ell > 1:
        raise IndexError("an index can only have a single ellipsis ('...')")
    if n_ell == 1:
        i = sel.index(Ellipsis)
        fill = len(shape) - (len(sel) - 1)
        sel = sel[:i] + [slice(None)] * max(fill, 0) + sel[i + 1:]
    if len(sel) > len(shape):
        raise IndexError(f"too many indices for array; expected {len(shape)}, got {len(sel)}")
    sel += [slice(None)] * (len(shape) - len(sel))
    out = []
    for s, n in zip(sel, shape):
        if isinstance(s, (int, np.integer)):
            i = int(s)
            if i < 0:
                i += n
            if not 0 <= i < n:
                raise IndexError(f"index out of bounds for dimension with length {n}")
            out.append(i)
        elif isinstance(s, slice):
            if s.step == 0:  # slice.indices raises first (indexing.py:408)
                raise ValueError("slice step cannot be zero")
            if s.step is not None and s.step < 1:
                raise IndexError("only slices with step >= 1 are supported.")
            out.append(slice(*s.indices(n)))
        else:
            raise IndexError(
                "unsupported selection item for basic indexing; expected integer or slice, "
                f"got {type(s)!r}")
    return tuple(out)


def project_dim(sel, dim_len: int, chunk_len: int) -> DimProjection:
    if isinstance(sel, int):
        ix = sel // chunk_len
        data_size = min(chunk_len, dim_len - ix * chunk_len)
        a = np.array([ix], np.int64)
        return DimProjection(a, np.array([sel - ix * chunk_len], np.int64), np.ones(1, np.int64), 1,
                             np.zeros(1, np.int64), np.array([data_size == 1]), True, 1)
    start, stop, step = sel.start, sel.stop, sel.step
    nitems = max(0, _ceildiv(stop - start, step))
    if start >= stop:
        e = np.zeros(0, np.int64)
        return DimProjection(e, e, e, step, e, np.zeros(0, bool), False, 0)
    ix_from = start // chunk_len
    ix_to = (stop - 1) // chunk_len + 1
    ix = np.arange(ix_from, ix_to, dtype=np.int64)
    off = ix * chunk_len
    clen = np.minimum(chunk_len, dim_len - off)
    limit = off + clen
    before = start < off
    rem = np.where(before, (off - start) % step, 0)
    s0 = np.where(before, np.where(rem > 0, step - rem, 0), start - off)
    out_off = np.where(before, -((start - off) // step), 0)  # ceildiv(off-start, step)
    s1 = np.where(stop > limit, clen, stop - off)
    cnt = np.maximum(0, -((s0 - s1) // step))
    complete = (s0 == 0) & (stop >= limit) & (step == 1)
    keep = cnt > 0
    return DimProjection(ix[keep], s0[keep], cnt[keep], step, out_off[keep], complete[keep],
                         False, nitems)


@dataclass
class Projections:
    """Cartesian product of per-dim projections: one row per touched chunk."""

    coords: np.ndarray      # int64[n, ndim]
    sel_start: np.ndarray   # int64[n, ndim]
    sel_count: np.ndarray   # int64[n, ndim]
    step: np.ndarray        # int64[ndim]
    out_start: np.ndarray   # int64[n, ndim]  (0 in dropped dims)
    complete: np.ndarray    # bool[n]
    dropped: tuple[bool, ...]
    out_shape: tuple[int, ...]


def basic_projections(selection, shape: tuple[int, ...], chunk_shape: tuple[int, ...]) -> Projections:
    sel = normalize_selection(selection, shape)
    dims = [project_dim(s, n, c) for s, n, c in zip(sel, shape, chunk_shape)]
    nd = len(dims)
    counts = [len(d.chunk_ix) for d in dims]
    n = int(np.prod(counts)) if counts else 1
    grids = np.indices(counts, dtype=np.int64).reshape(nd, -1) if nd else np.zeros((0, 1), np.int64)

    def take(attr):
        return np.stack([getattr(d, attr)[grids[i]] for i, d in enumerate(dims)], axis=1) \
            if nd else np.zeros((1, 0), np.int64)

    coords = take("chunk_ix")
    complete = np.all(take("complete").astype(bool), axis=1) if nd else np.ones(1, bool)
    return Projections(
        coords=coords.reshape(n, nd), sel_start=take("sel_start").reshape(n, nd),
        sel_count=take("sel_count").reshape(n, nd), step=np.array([d.step for d in dims], np.int64),
        out_start=take("out_start").reshape(n, nd), complete=complete.reshape(n),
        dropped=tuple(d.dropped for d in dims),
        out_shape=tuple(d.nitems for d in dims if not d.dropped))


def to_chunk_selection(p: Projections, i: int) -> tuple:
    """Row i as the reference's (chunk_selection, out_selection) tuples."""
    csel, osel = [], []
    for d in range(p.coords.shape[1]):
        s0 = int(p.sel_start[i, d])
        if p.dropped[d]:
            csel.append(s0)
            continue
        st = int(p.step[d])
        cnt = int(p.sel_count[i, d])
        csel.append(slice(s0, s0 + (cnt - 1) * st + 1, st))
        o = int(p.out_start[i, d])
        osel.append(slice(o, o + cnt))
    return tuple(csel), tuple(osel)


def _project_dim_lists(sel, dim_len: int, chunk_len: int):
    """project_dim as Python lists (ix, sel_start, sel_count, out_start,
    complete, step, dropped, nitems); numpy only for long dims."""
    if isinstance(sel, int):
        ix = sel // chunk_len
        return ([ix], [sel - ix * chunk_len], [1], [0], [min(chunk_len, dim_len - ix * chunk_len) == 1], 1,
                True, 1)
    start, stop, step = sel.start, sel.stop, sel.step
    nitems = max(0, -((start - stop) // step))
    if start >= stop:
        return [], [], [], [], [], step, False, 0
    ix_from, ix_to = start // chunk_len, (stop - 1) // chunk_len + 1
    if ix_to - ix_from > 256:
        d = project_dim(sel, dim_len, chunk_len)
        return (d.chunk_ix.tolist(), d.sel_start.tolist(), d.sel_count.tolist(), d.out_start.tolist(),
                d.complete.tolist(), step, False, nitems)
    ixs, s0s, cnts, oos, cps = [], [], [], [], []
    for ix in range(ix_from, ix_to):
        off = ix * chunk_len
        clen = min(chunk_len, dim_len - off)
        limit = off + clen
        if start < off:
            rem = (off - start) % step
            s0 = step - rem if rem else 0
            oo = -((start - off) // step)
        else:
            s0, oo = start - off, 0
        s1 = clen if stop > limit else stop - off
        cnt = max(0, -((s0 - s1) // step))
        if cnt > 0:
            ixs.append(ix)
            s0s.append(s0)
            cnts.append(cnt)
            oos.append(oo)
            cps.append(s0 == 0 and stop >= limit and step == 1)
    return ixs, s0s, cnts, oos, cps, step, False, nitems


def _project_dim_grid(sel, dim_len: int, g):
    """IntDimIndexer / SliceDimIndexer.__iter__ over any dimension grid
    (indexing.py:369-468 with DimensionGrid's index_to_chunk / chunk_offset /
    data_size): a VaryingDimension of a rectilinear grid (zarr_hip.grid)."""
    if isinstance(sel, int):
        ix = g.index_to_chunk(sel)
        return [ix], [sel - g.chunk_offset(ix)], [1], [0], [g.data_size(ix) == 1], 1, True, 1
    start, stop, step = sel.start, sel.stop, sel.step
    nitems = max(0, -((start - stop) // step))
    if start >= stop:
        return [], [], [], [], [], step, False, 0
    ix_from = g.index_to_chunk(start) if start > 0 else 0
    ix_to = g.index_to_chunk(stop - 1) + 1 if stop > 0 else 0
    ixs, s0s, cnts, oos, cps = [], [], [], [], []
    for ix in range(ix_from, ix_to):
        off = g.chunk_offset(ix)
        clen = g.data_size(ix)
        limit = off + clen
        if start < off:
            rem = (off - start) % step
            s0 = step - rem if rem else 0
            oo = -((start - off) // step)
        else:
            s0, oo = start - off, 0
        s1 = clen if stop > limit else stop - off
        cnt = max(0, -((s0 - s1) // step))
        if cnt > 0:
            ixs.append(ix)
            s0s.append(s0)
            cnts.append(cnt)
            oos.append(oo)
            cps.append(s0 == 0 and stop >= limit and step == 1)
    return ixs, s0s, cnts, oos, cps, step, False, nitems


def chunk_batch(selection, shape: tuple[int, ...], chunk_shape):
    """basic_projections + chunk_selections for a batch: per-dim projections,
    then their Cartesian product (C order over chunk coordinates, as
    basic_projections) built from Python lists.  Returns
    ([(coords, chunk_selection, out_selection, complete)], out_shape).
    `chunk_shape` is a regular chunk shape or a zarr_hip.grid.ChunkGrid
    (rectilinear grids: per-dim projections over the varying edges)."""
    import itertools

    from .grid import ChunkGrid, FixedDimension

    sel = normalize_selection(selection, shape)
    if isinstance(chunk_shape, ChunkGrid):
        dims = chunk_shape.dimensions
        chunk_shape = tuple(d.size if isinstance(d, FixedDimension) else d for d in dims)
    ixs, csels, osels, cps = [], [], [], []
    out_shape = []
    for s, n, c in zip(sel, shape, chunk_shape):
        if isinstance(c, int):
            ix, s0, cnt, oo, cp, st, dropped, nitems = _project_dim_lists(s, n, c)
        else:
            ix, s0, cnt, oo, cp, st, dropped, nitems = _project_dim_grid(s, n, c)
        ixs.append(ix)
        cps.append(cp)
        if dropped:
            csels.append(s0)
        else:
            out_shape.append(nitems)
            csels.append([slice(a, a + (k - 1) * st + 1, st) for a, k in zip(s0, cnt)])
            osels.append([slice(o, o + k) for o, k in zip(oo, cnt)])
    P = itertools.product
    out = list(zip(P(*ixs), P(*csels), P(*osels), map(all, P(*cps))))
    return out, tuple(out_shape)


def chunk_selections(p: Projections) -> list:
    """to_chunk_selection for every row, from Python lists (one pass)."""
    nd = p.coords.shape[1]
    ss, cc, oo = p.sel_start.tolist(), p.sel_count.tolist(), p.out_start.tolist()
    steps = p.step.tolist()
    drop = p.dropped
    out = []
    for s_row, c_row, o_row in zip(ss, cc, oo):
        csel, osel = [], []
        for d in range(nd):
            s0 = s_row[d]
            if drop[d]:
                csel.append(s0)
                continue
            st, cnt, o = steps[d], c_row[d], o_row[d]
            csel.append(slice(s0, s0 + (cnt - 1) * st + 1, st))
            osel.append(slice(o, o + cnt))
        out.append((tuple(csel), tuple(osel)))
    return out


# --- Morton / lexicographic orders (src/zarr/core/indexing.py:1524-1643) -------

def morton_order(shape: tuple[int, ...]) -> np.ndarray:
    """Coordinates of a grid in Morton (Z) order: codes of the ceiling power-of-2
    hypercube decoded (bit-interleaving over the dims that still have bits) and
    filtered to the grid, as _morton_order does (indexing.py:1578-1630)."""
    n_total = int(np.prod(shape)) if shape else 1
    nd = len(shape)
    if n_total == 0:
        return np.zeros((0, nd), np.int64)
    bits = [(c - 1).bit_length() for c in shape]
    total = sum(bits)
    z = np.arange(1 << total, dtype=np.int64)
    out = np.zeros((len(z), nd), np.int64)
    ib = 0
    for cb in range(max(bits) if bits else 0):
        for d in range(nd):
            if cb < bits[d]:
                out[:, d] |= ((z >> ib) & 1) << cb
                ib += 1
    keep = np.all(out < np.array(shape, np.int64), axis=1)
    return out[keep]


def lexicographic_order(shape: tuple[int, ...]) -> np.ndarray:
    if not shape:
        return np.zeros((1, 0), np.int64)
    return np.indices(shape, dtype=np.int64).reshape(len(shape), -1).T


def colexicographic_order(shape: tuple[int, ...]) -> np.ndarray:
    return lexicographic_order(tuple(shape[::-1]))[:, ::-1]


def subchunk_order(shape: tuple[int, ...], order: str) -> np.ndarray:
    """ShardingCodec._subchunk_order_iter (sharding.py:1090-1107)."""
    if order == "morton":
        return morton_order(shape)
    if order in ("lexicographic", "unordered"):
        return lexicographic_order(shape)
    if order == "colexicographic":
        return colexicographic_order(shape)
    raise ValueError(f"Unrecognized subchunk write order: {order!r}.")


def iter_coords(shape):
    return itertools.product(*(range(s) for s in shape))

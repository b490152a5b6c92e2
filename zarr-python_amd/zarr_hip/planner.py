"""Host planner: a batch of (source, chunk_selection, out_selection) items plus an
evolved codec chain  ->  one zhip_layout and flat chunk / selection tables.

This is where zarr semantics stay on the host: the codec chain
is reduced to (stored-dim permutation, byteswap, crc, sharding geometry); the
transpose codec (transpose.py:89-104) disappears into a permutation of the
out strides, so the kernels only ever walk the *stored* byte order.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import struct as _struct

import numpy as np

from . import _native as N
from .codecs import BytesCodec, Crc32cCodec, ShardingCodec, TransposeCodec, is_host_codec, split_codecs, \
    split_host_tail
from .indexing import basic_projections
from .indexing import morton_order
from .spec import ArraySpec

CHUNK_DT, SEL_DT, STATUS_DT = N._np_dtypes()


@dataclass(frozen=True)
class ChainInfo:
    """The GPU-relevant content of an evolved fixed-size codec chain."""

    perm: tuple[int, ...]         # stored dim i is decoded dim perm[i]
    swap: bool                    # bytes codec endian != native
    crc: bool                     # trailing crc32c
    endian: str | None
    shard: ShardingCodec | None = None      # the sharding codec with its GPU inner chain
    inner: "ChainInfo | None" = None
    # the inner chain's host stage (compressors, anything after them): inner
    # chunks pass through it on the host before their fixed-size part decodes
    # on the GPU (hoststage.py)
    inner_host: tuple = ()


def analyze_chain(codecs, spec: ArraySpec) -> ChainInfo:
    aa, ab, bb = split_codecs(codecs)
    if any(is_host_codec(c) for c in bb):
        raise NotImplementedError("the host stage of this chain must be split off first "
                                  "(HipCodecPipeline runs it on the host: hoststage.py)")
    if len(bb) > 1 or any(not isinstance(c, Crc32cCodec) for c in bb):
        raise NotImplementedError("only a single trailing crc32c bytes->bytes codec is supported")
    perm = tuple(range(spec.ndim))
    for t in aa:
        if not isinstance(t, TransposeCodec):
            raise NotImplementedError(f"array->array codec {getattr(t, 'name', t)!r} is not on the GPU path "
                                      "(transpose is the only array->array codec it runs)")
        t.evolve_from_array_spec(ArraySpec(tuple(spec.shape[p] for p in perm), spec.dtype,
                                           spec.fill_value))
        perm = tuple(perm[t.order[i]] for i in range(len(perm)))
    if isinstance(ab, ShardingCodec):
        # transposes around the sharding codec permute the shard it sees
        # (perm = the outer permutation; the pipeline maps batches into that
        # space, HipCodecPipeline._shard_space); bytes->bytes codecs after it
        # would hide the index and are not on the GPU path
        if bb:
            raise NotImplementedError(
                "bytes->bytes codecs around sharding_indexed are not on the GPU path")
        inner_spec = ab.inner_spec(spec)
        fixed, tail = split_host_tail(ab.codecs)
        if tail:
            from dataclasses import replace as _replace

            ab = _replace(ab, codecs=fixed)
        inner = analyze_chain(fixed, inner_spec)
        if inner.shard is not None:
            raise NotImplementedError("nested sharding is not on the GPU path yet")
        ia, iab, ibb = split_codecs(ab.index_codecs)
        if ia or not isinstance(iab, BytesCodec) or iab.endian not in (None, "little") or \
                len(ibb) > 1 or any(not isinstance(c, Crc32cCodec) for c in ibb):
            raise NotImplementedError("shard index codecs must be [bytes(little)] + optional crc32c")
        return ChainInfo(tuple(perm), False, False, None, ab, inner, tuple(tail))
    assert isinstance(ab, BytesCodec)
    ab = ab.evolve_from_array_spec(spec)
    return ChainInfo(perm, ab.needs_swap(spec.dtype), len(bb) == 1, ab.endian)


def _sel_fields(csel, ndim):
    start = np.zeros(ndim, np.int64)
    count = np.ones(ndim, np.int64)
    step = np.ones(ndim, np.int64)
    is_int = np.zeros(ndim, bool)
    for d, s in enumerate(csel):
        if isinstance(s, (int, np.integer)):
            start[d] = int(s)
            is_int[d] = True
        else:
            a, b, st = s.start or 0, s.stop, s.step or 1
            start[d] = a
            step[d] = st
            count[d] = max(0, -((a - b) // st))
    return start, count, step, is_int


def _sel_lists(csel):
    """_sel_fields as Python lists (the per-item planning loop)."""
    st, ct, sp = [], [], []
    for s in csel:
        if isinstance(s, slice):
            a, k = s.start or 0, s.step or 1
            st.append(a)
            sp.append(k)
            ct.append(max(0, -((a - s.stop) // k)))
        else:
            st.append(int(s))
            ct.append(1)
            sp.append(1)
    return st, ct, sp


def out_dim_strides(ndim: int, is_int, drop_axes, out_strides_bytes) -> list:
    """Per decoded dim: the out byte stride (0 for dims absent from out)."""
    kept = [d for d in range(ndim) if not is_int[d]]
    if drop_axes:
        drop = set(int(a) for a in drop_axes)
        kept = [d for k, d in enumerate(kept) if k not in drop]
    st = [0] * ndim
    if len(kept) != len(out_strides_bytes):
        raise ValueError(f"selection has {len(kept)} output dims, out has {len(out_strides_bytes)}")
    for j, d in enumerate(kept):
        st[d] = int(out_strides_bytes[j])
    return st


def _out_offset(osel, out_strides_bytes) -> int:
    off = 0
    for j, s in enumerate(osel):
        a = s if isinstance(s, (int, np.integer)) else (s.start or 0)
        off += int(a) * int(out_strides_bytes[j])
    return off


@dataclass
class Tables:
    layout: N.Layout
    chunks: np.ndarray            # CHUNK_DT[n]
    sels: np.ndarray              # SEL_DT[m]
    fast: bool
    item_of_chunk: np.ndarray     # int64[n]: batch item of each chunk entry
    tile: bool = False            # tiled-transpose decode (ZHIP_DF_TILE)
    tile_prefix: bool = False     # tiled-transpose encode of prefix-box selections (ZHIP_DF_TILE_PREFIX)
    rows: bool = False            # affine whole-row decode (ZHIP_DF_ROWS, k_decode_rows)
    index_layout: N.Layout | None = None
    index_chunks: np.ndarray | None = None
    index_item: np.ndarray | None = None
    predict: "N.Predict | None" = None  # load-address prediction (rows batches, zhip_predict)
    extra: dict = field(default_factory=dict)


def _make_layout(shape_stored, itemsize, ostride_stored, flags, fill: bytes, n_inner=0,
                 index_size=0) -> N.Layout:
    L = N.Layout()
    nd = len(shape_stored)
    L.ndim = nd
    L.itemsize = itemsize
    for i in range(N.MAX_DIMS):
        L.shape[i] = int(shape_stored[i]) if i < nd else 1
        L.out_stride[i] = int(ostride_stored[i]) if i < nd else 0
    L.nbytes = int(np.prod(shape_stored, dtype=np.int64)) * itemsize if nd else itemsize
    L.flags = flags
    L.n_inner = n_inner
    L.index_size = index_size
    fb = (fill * (16 // max(len(fill), 1) + 1))[:16]
    ctypes.memmove(L.fill, fb, 16)
    return L


def _pack_sels(start, count, step) -> tuple[np.ndarray, np.ndarray]:
    """Dedup selection rows; returns (SEL_DT table, row index per entry)."""
    n, nd = start.shape
    key = np.concatenate([start, count, step], axis=1)
    if n and (key == key[0]).all():  # the common case: every chunk selected alike
        uniq, inv = key[:1], np.zeros(n, np.int64)
    else:
        uniq, inv = np.unique(key, axis=0, return_inverse=True)
    sels = np.zeros(len(uniq), SEL_DT)
    for r, row in enumerate(uniq):
        st, ct, sp = row[:nd], row[nd:2 * nd], row[2 * nd:]
        sels["start"][r, :nd] = st
        sels["count"][r, :nd] = ct
        sels["step"][r, :nd] = sp
        sels["step"][r, nd:] = 1
        sels["count"][r, nd:] = 1
        for d in range(N.MAX_DIMS):
            m, s = N.fdiv(int(sp[d]) if d < nd else 1)
            sels["div"][r, d, 0] = m
            sels["div"][r, d, 1] = s
    return sels, inv.reshape(-1).astype(np.uint32)


def _fast_ok(layout: N.Layout, start, count, step, out_offs, out_base_ptr: int) -> bool:
    nd = layout.ndim
    it = layout.itemsize
    last = nd - 1
    row_bytes = layout.shape[last] * it
    if layout.out_stride[last] != it or row_bytes % 16 != 0:
        return False
    if out_base_ptr % 16 != 0 or np.any(out_offs % 16 != 0):
        return False
    for d in range(last):
        if layout.out_stride[d] % 16 != 0:
            return False
    return bool(np.all(start[:, last] == 0) and np.all(count[:, last] == layout.shape[last])
                and np.all(step[:, last] == 1))


def _split_1d(n_items: int, itemsize: int, ostride: int, start, count, step) -> int:
    """A 1-D chunk read into contiguous out as whole rows of R items (the bytes
    unchanged, viewed as (n/R, R)), so the row decode applies: the largest R
    (a power of two, rows of 16..4096 bytes) dividing the chunk length and every
    selection's start and count, with (n/R) a multiple of the rows one 4 KiB
    workgroup step covers.  0 when none (int selections, steps, odd bounds)."""
    if ostride != itemsize or not len(start) or not np.all(step[:, 0] == 1):
        return 0
    r = 4096 // itemsize
    while r * itemsize >= 16:
        if n_items % r == 0 and np.all(start[:, 0] % r == 0) and np.all(count[:, 0] % r == 0) and \
                np.all(count[:, 0] > 0) and (n_items // r) % (4096 // (r * itemsize)) == 0:
            return r
        r //= 2
    return 0


def _rows_ok(layout: N.Layout, count, step) -> bool:
    """ZHIP_DF_ROWS preconditions (on top of _fast_ok): unit steps wherever more
    than one index is selected, rows of 2^k <= 4096 bytes, and shape[ndim-2] a
    multiple of the rows one 4 KiB workgroup step covers."""
    nd = layout.ndim
    if nd < 2:
        return False
    rb = layout.shape[nd - 1] * layout.itemsize
    if rb < 16 or rb > 4096 or rb & (rb - 1):
        return False
    if layout.shape[nd - 2] % (4096 // rb):
        return False
    return bool(np.all((step == 1) | (count <= 1)))


def _tiled_layout(layout: N.Layout) -> bool:
    """A stored dim other than the innermost is contiguous in the array / out
    and innermost rows are 16-byte multiples (zhip_plan.tq >= 0)."""
    nd = layout.ndim
    it = layout.itemsize
    last = nd - 1
    if nd < 2 or layout.out_stride[last] == it or (layout.shape[last] * it) % 16:
        return False
    return any(layout.out_stride[d] == it and layout.shape[d] > 1 for d in range(last))


def _tile_ok(layout: N.Layout, start, count, step, out_offs, out_base_ptr: int) -> bool:
    """Transposed layouts: a stored dim other than the innermost is contiguous in
    out, every chunk is fully selected and out is 16-byte aligned."""
    nd = layout.ndim
    it = layout.itemsize
    last = nd - 1
    if nd < 2 or layout.out_stride[last] == it or (layout.shape[last] * it) % 16:
        return False
    tq = [d for d in range(last) if layout.out_stride[d] == it and layout.shape[d] > 1]
    if not tq:
        return False
    if out_base_ptr % 16 or np.any(out_offs % 16):
        return False
    if any(layout.out_stride[d] % 16 for d in range(nd) if d != tq[0]):
        return False
    shp = np.array([layout.shape[d] for d in range(nd)], np.int64)
    return bool(np.all(start == 0) and np.all(step == 1) and np.all(count == shp[None, :]))


def plan_encode(chain: ChainInfo, spec: ArraySpec, items: list, arr_strides_bytes,
                arr_base_ptr: int) -> Tables:
    """items: list of (dst_off, chunk_selection, arr_selection_start) for whole
    chunks (unsharded chain).  chunk_selection is over decoded dims; elements
    outside it are encoded as the fill value."""
    ndim = spec.ndim
    itemsize = spec.dtype.itemsize
    perm = chain.perm
    shape_st = [spec.shape[p] for p in perm]
    ost = np.asarray(arr_strides_bytes, np.int64)
    ost_st = [int(ost[p]) for p in perm]
    flags = (N.LF_CRC if chain.crc else 0) | (N.LF_SWAP if chain.swap else 0) | \
        (N.LF_FLOAT if spec.dtype.kind == "f" else 0)
    layout = _make_layout(shape_st, itemsize, ost_st, flags, spec.fill_bytes())
    n = len(items)
    chunks = np.zeros(n, CHUNK_DT)
    start = np.zeros((n, ndim), np.int64)
    count = np.zeros((n, ndim), np.int64)
    step = np.ones((n, ndim), np.int64)
    for i, (dst, csel, astart) in enumerate(items):
        st, ct, sp, _ = _sel_fields(csel, ndim)
        start[i], count[i], step[i] = st[list(perm)], ct[list(perm)], sp[list(perm)]
        chunks["src"][i] = dst
        chunks["out_off"][i] = int(sum(int(a) * int(o) for a, o in zip(astart, ost)))
    sels, inv = _pack_sels(start, count, step)
    chunks["sel"] = inv
    fast = _fast_ok(layout, start, count, step, chunks["out_off"], arr_base_ptr)
    rows = fast and _rows_ok(layout, count, step)
    tile = not fast and _tile_ok(layout, start, count, step, chunks["out_off"], arr_base_ptr)
    # transposed chunks whose selections are prefix boxes (edge chunks): the
    # general tiled encode (k_encode_tile) writes the rest of the chunk as fill
    tile_prefix = not fast and not tile and _tiled_layout(layout) and bool(np.all(start == 0)) and \
        bool(np.all(step == 1))
    return Tables(layout, chunks, sels, fast, np.arange(n), rows=rows, tile=tile, tile_prefix=tile_prefix)


def plan_decode(chain: ChainInfo, spec: ArraySpec, items: list, out_strides_bytes,
                out_base_ptr: int, drop_axes=(), resolved: list | None = None,
                item_out_extra=None) -> Tables:
    """items: list of (src_off, src_len, missing, chunk_selection, out_selection).
    item_out_extra: optional per-item byte offset added to the item's out
    position (one launch decoding into the slices of a stacked out).

    Sharded chains: by default every inner chunk is located by the kernel
    through the shard index in HBM.  With `resolved` (host-staged partial
    shard reads, staging.gather_sharded_partial) the host has already fetched
    the touched inner chunks: resolved[i] = (src_by_slot, len_by_slot,
    miss_by_slot, index_src) and the data launch is a plain (unsharded) one
    over those inner chunks; the staged index bytes still get their CRC
    verified by the index launch."""
    ndim = spec.ndim
    itemsize = spec.dtype.itemsize
    fill = spec.fill_bytes()
    if not items:
        raise ValueError("empty batch")
    is_int0 = [not isinstance(s, slice) for s in items[0][3]]
    ost_dec = out_dim_strides(ndim, is_int0, drop_axes, out_strides_bytes)
    if NATIVE_PLANNER and (ndim > 1 or chain.shard is not None) and (resolved is None or chain.shard is not None):
        t = _plan_native(chain, spec, items, out_strides_bytes, out_base_ptr, ost_dec, item_out_extra, fill,
                         resolved)
        if t is not None:
            return t

    if chain.shard is None:
        perm = chain.perm
        shape_st = [spec.shape[p] for p in perm]
        ost_st = [ost_dec[p] for p in perm]
        flags = (N.LF_CRC if chain.crc else 0) | (N.LF_SWAP if chain.swap else 0)
        layout = _make_layout(shape_st, itemsize, ost_st, flags, fill)
        n = len(items)
        chunks = np.zeros(n, CHUNK_DT)
        S, C, P, oo = [], [], [], []
        ostr = [int(x) for x in out_strides_bytes]
        for so, sl, miss, csel, osel in items:
            st, ct, sp = _sel_lists(csel)
            S.append(st)
            C.append(ct)
            P.append(sp)
            oo.append(sum(((s.start or 0) if isinstance(s, slice) else int(s)) * o for s, o in zip(osel, ostr)))
        pl = list(perm)
        start = np.array(S, np.int64).reshape(n, ndim)[:, pl]
        count = np.array(C, np.int64).reshape(n, ndim)[:, pl]
        step = np.array(P, np.int64).reshape(n, ndim)[:, pl]
        chunks["src"] = [it[0] for it in items]
        chunks["src_len"] = [it[1] for it in items]
        chunks["flags"] = [N.CF_MISSING if it[2] else 0 for it in items]
        oo = np.array(oo, np.int64)
        if item_out_extra is not None:
            oo += np.asarray(item_out_extra, np.int64)
        chunks["out_off"] = oo
        if ndim == 1:
            split = _split_1d(shape_st[0], itemsize, ost_st[0], start, count, step)
            if split:  # the same chunk bytes viewed as (N/R, R): whole rows of R items
                R = split
                layout = _make_layout([shape_st[0] // R, R], itemsize, [ost_st[0] * R, ost_st[0]], flags, fill)
                start = np.stack([start[:, 0] // R, np.zeros(n, np.int64)], axis=1)
                count = np.stack([count[:, 0] // R, np.full(n, R, np.int64)], axis=1)
                step = np.ones((n, 2), np.int64)
        sels, inv = _pack_sels(start, count, step)
        chunks["sel"] = inv
        fast = _fast_ok(layout, start, count, step, chunks["out_off"], out_base_ptr)
        tile = not fast and _tile_ok(layout, start, count, step, chunks["out_off"], out_base_ptr)
        rows = fast and _rows_ok(layout, count, step)
        return Tables(layout, chunks, sels, fast, np.arange(n), tile=tile, rows=rows)

    # ---- sharded: expand every shard item into its inner chunks ----
    sh = chain.shard
    inner = chain.inner
    cps = sh.chunks_per_shard(spec.shape)
    n_inner = int(np.prod(cps))
    inner_shape = sh.chunk_shape
    perm = inner.perm
    shape_st = [inner_shape[p] for p in perm]
    ost_st = [ost_dec[p] for p in perm]
    index_size = sh.shard_index_size(n_inner)
    flags = (N.LF_CRC if inner.crc else 0) | (N.LF_SWAP if inner.swap else 0)
    if resolved is None:
        flags |= N.LF_SHARDED | (N.LF_INDEX_START if sh.index_location == "start" else 0)
        layout = _make_layout(shape_st, itemsize, ost_st, flags, fill, n_inner, index_size)
    else:
        layout = _make_layout(shape_st, itemsize, ost_st, flags, fill)
    cps_strides = np.array([int(np.prod(cps[d + 1:])) for d in range(ndim)], np.int64)
    proj_cache: dict = {}
    parts = []
    for i, (so, sl, miss, csel, osel) in enumerate(items):
        if resolved is None and not miss and sl < index_size:
            # the kernels locate the index at blob end - index_size (or the
            # start): a short blob must never reach them (staging.py raises the same)
            raise ValueError("shard blob is shorter than its index")
        key = tuple((s.start, s.stop, s.step) if isinstance(s, slice) else int(s) for s in csel)
        pr = proj_cache.get(key)
        if pr is None:
            pr = basic_projections(tuple(csel), spec.shape, inner_shape)
            proj_cache[key] = pr
        base = _out_offset(osel, out_strides_bytes) + \
            (0 if item_out_extra is None else int(item_out_extra[i]))
        m = len(pr.coords)
        oo = base + (pr.out_start * np.asarray(ost_dec, np.int64)[None, :]).sum(axis=1)
        parts.append((i, so, sl, miss, pr, oo, m))
    total = sum(p[-1] for p in parts)
    chunks = np.zeros(total, CHUNK_DT)
    start = np.zeros((total, ndim), np.int64)
    count = np.zeros((total, ndim), np.int64)
    step = np.zeros((total, ndim), np.int64)
    item_of = np.zeros(total, np.int64)
    pos = 0
    idx_rows = []
    idx_seen: set = set()
    for i, so, sl, miss, pr, oo, m in parts:
        sl_ = slice(pos, pos + m)
        slots = (pr.coords * cps_strides[None, :]).sum(axis=1)
        chunks["out_off"][sl_] = oo
        chunks["slot"][sl_] = slots
        if resolved is not None:
            r = resolved[i]
            if r is None or miss:
                chunks["flags"][sl_] = N.CF_MISSING
            else:
                src_by, len_by, miss_by, isrc = r
                chunks["src"][sl_] = src_by[slots]
                chunks["src_len"][sl_] = len_by[slots]
                chunks["flags"][sl_] = np.where(miss_by[slots], N.CF_MISSING, 0)
                if isrc >= 0 and isrc not in idx_seen:
                    idx_seen.add(isrc)
                    idx_rows.append((i, isrc, index_size))
        else:
            chunks["src"][sl_] = so
            chunks["src_len"][sl_] = sl
            chunks["flags"][sl_] = N.CF_MISSING if miss else 0
            chunks["slot"][sl_] = slots
        start[sl_] = pr.sel_start[:, list(perm)]
        count[sl_] = pr.sel_count[:, list(perm)]
        step[sl_] = np.broadcast_to(pr.step[list(perm)], (m, ndim))
        item_of[sl_] = i
        if resolved is None and not miss and sh.index_has_crc and so not in idx_seen:
            idx_seen.add(so)
            ipos = 0 if sh.index_location == "start" else sl - index_size
            idx_rows.append((i, so + ipos, index_size))
        pos += m
    sels, inv = _pack_sels(start, count, step)
    chunks["sel"] = inv
    fast = _fast_ok(layout, start, count, step, chunks["out_off"], out_base_ptr)
    tile = not fast and _tile_ok(layout, start, count, step, chunks["out_off"], out_base_ptr)
    rows = fast and _rows_ok(layout, count, step)
    t = Tables(layout, chunks, sels, fast, item_of, tile=tile, rows=rows)
    if idx_rows:
        L2 = _make_layout([16 * n_inner], 1, [0], N.LF_CRC | N.LF_NO_WRITE, b"\0")
        ic = np.zeros(len(idx_rows), CHUNK_DT)
        ic["src"] = [r[1] for r in idx_rows]
        ic["src_len"] = [r[2] for r in idx_rows]
        t.index_layout = L2
        t.index_chunks = ic
        t.index_item = np.array([r[0] for r in idx_rows], np.int64)
    return t


# the native host planner (zhip_plan_batch) for basic-selection batches;
# ZARR_HIP_NATIVE_PLANNER=0 keeps the Python loop (tests compare the two)
NATIVE_PLANNER = __import__("os").environ.get("ZARR_HIP_NATIVE_PLANNER", "1") != "0"


_NATIVE_CTX: dict = {}


def _native_ctx(chain: ChainInfo, spec: ArraySpec, ost_dec, fill, staged: bool = False):
    """Per-geometry constants of the native planner (layouts, the
    zhip_batch_geom record, the layout halves of the kernel choice), built
    once per (chain, chunk spec, out strides)."""
    # (the chain by identity, held by the entry: pipelines memoise their
    # chains, and hashing one walks its codecs)
    key = (id(chain), spec.shape, spec.dtype.str, fill, tuple(ost_dec), staged)
    hit = _NATIVE_CTX.get(key)
    if hit is not None and hit[0] is chain:
        return hit[1]
    ndim = spec.ndim
    shape = spec.shape
    g = np.zeros(1, N.GEOM_DT)
    g["ndim"] = ndim
    sh = chain.shard
    inner = chain.inner if sh is not None else chain
    perm = list(inner.perm)
    g["perm"][0, :ndim] = perm
    g["shape"][0, :ndim] = shape
    g["ost"][0, :ndim] = ost_dec
    flags = (N.LF_CRC if inner.crc else 0) | (N.LF_SWAP if inner.swap else 0)
    n_inner, index_layout = 1, None
    if sh is not None:
        inner_shape = sh.chunk_shape
        n_inner = int(np.prod(sh.chunks_per_shard(shape)))
        index_size = sh.shard_index_size(n_inner)
        g["inner"][0, :ndim] = inner_shape
        g["index_size"] = index_size
        g["index_start"] = 1 if sh.index_location == "start" else 0
        g["index_crc"] = 1 if sh.index_has_crc else 0
        if staged:  # host-staged inner chunks: a plain launch over them (plan_decode's `resolved`)
            layout = _make_layout([inner_shape[p] for p in perm], spec.dtype.itemsize,
                                  [ost_dec[p] for p in perm], flags, fill)
        else:
            flags |= N.LF_SHARDED | (N.LF_INDEX_START if sh.index_location == "start" else 0)
            layout = _make_layout([inner_shape[p] for p in perm], spec.dtype.itemsize,
                                  [ost_dec[p] for p in perm], flags, fill, n_inner, index_size)
        index_layout = _make_layout([16 * n_inner], 1, [0], N.LF_CRC | N.LF_NO_WRITE, b"\0")
    else:
        layout = _make_layout([shape[p] for p in perm], spec.dtype.itemsize, [ost_dec[p] for p in perm],
                              flags, fill)
    # the layout halves of _fast_ok / _rows_ok / _tile_ok
    nd, isz, last = layout.ndim, layout.itemsize, layout.ndim - 1
    fast_l = (layout.out_stride[last] == isz and (layout.shape[last] * isz) % 16 == 0
              and all(layout.out_stride[d] % 16 == 0 for d in range(last)))
    tile_l = False
    if nd >= 2 and layout.out_stride[last] != isz and (layout.shape[last] * isz) % 16 == 0:
        tq = [d for d in range(last) if layout.out_stride[d] == isz and layout.shape[d] > 1]
        tile_l = bool(tq) and all(layout.out_stride[d] % 16 == 0 for d in range(nd) if d != tq[0])
    rows_l = False
    if nd >= 2:
        rb = layout.shape[last] * isz
        rows_l = 16 <= rb <= 4096 and not rb & (rb - 1) and layout.shape[nd - 2] % (4096 // rb) == 0
    ctx = (g, g.ctypes.data, layout, index_layout, n_inner, fast_l, tile_l, rows_l)
    if len(_NATIVE_CTX) > 256:
        _NATIVE_CTX.clear()
    _NATIVE_CTX[key] = (chain, ctx)
    return ctx


_CH_SZ, _SEL_SZ = CHUNK_DT.itemsize, SEL_DT.itemsize


def _plan_native(chain: ChainInfo, spec: ArraySpec, items: list, out_strides_bytes, out_base_ptr: int,
                 ost_dec, item_out_extra, fill, resolved=None) -> "Tables | None":
    """plan_decode through zhip_plan_batch: the per-item projections, inner-chunk
    expansion, selection dedup and index list in one native call; the kernel
    choice from the layout (cached per geometry) and the call's aggregate
    flags.  None when an item is not a basic selection (the Python loop then
    plans)."""
    ndim = spec.ndim
    n = len(items)
    shape = spec.shape
    ostr = [int(x) for x in out_strides_bytes]
    # zhip_item records as int64 rows: src, src_len, out_off, missing | res << 32,
    # start[MAX_DIMS], stop[MAX_DIMS], step[MAX_DIMS]
    MD = N.MAX_DIMS
    o_st, o_sp, o_sk = 4, 4 + MD, 4 + 2 * MD
    blank = [0] * (4 + 3 * MD)
    recs = []
    for so, sl, miss, csel, osel in items:
        if len(csel) != ndim:
            return None
        row = blank.copy()
        row[0], row[1], row[3] = so, sl, 1 if miss else 0
        for d, s in enumerate(csel):
            if type(s) is slice:
                a, b, k = s.indices(shape[d])
                if k < 1:
                    return None
                row[o_st + d], row[o_sp + d], row[o_sk + d] = a, b, k
            elif isinstance(s, (int, np.integer)):
                v = int(s)
                row[o_st + d] = v + shape[d] if v < 0 else v  # stop = step = 0: an integer index
            else:
                return None
        oo = 0
        for o, w in zip(osel, ostr):
            oo += (o.start or 0) * w if type(o) is slice else int(o) * w
        row[2] = oo
        recs.append(row)
    g, gp, layout, index_layout, n_inner, fast_l, tile_l, rows_l = _native_ctx(chain, spec, ost_dec, fill,
                                                                               resolved is not None)
    res_p, keep = None, None
    if resolved is not None:  # one zhip_resolved row per distinct staged shard
        rows, row_of = [], {}
        rix = []
        for r in resolved:
            if r is None:
                rix.append(-1)
                continue
            j = row_of.get(id(r))
            if j is None:
                j = row_of[id(r)] = len(rows)
                rows.append(r)
            rix.append(j)
        R = max(len(rows), 1)
        rs = np.zeros((R, n_inner), np.uint64)
        rl = np.zeros((R, n_inner), np.uint64)
        rm = np.ones((R, n_inner), np.uint8)
        ri = np.full(R, -1, np.int64)
        for j, (src_by, len_by, miss_by, isrc) in enumerate(rows):
            rs[j] = src_by
            rl[j] = len_by
            rm[j] = miss_by
            ri[j] = isrc
        rr = np.zeros(1, N.RESOLVED_DT)
        rr["src"], rr["len"], rr["missing"], rr["index_src"] = rs.ctypes.data, rl.ctypes.data, rm.ctypes.data, \
            ri.ctypes.data
        rr["n_rows"], rr["n_inner"] = len(rows), n_inner
        res_p, keep = rr.ctypes.data, (rs, rl, rm, ri, rr)
    it = np.array(recs, np.int64).view(N.ITEM_DT).reshape(n)
    if item_out_extra is not None:
        it["out_off"] += np.asarray(item_out_extra, np.int64)
    if resolved is not None:
        it["res"] = rix
    cap = n * n_inner
    ni = n if chain.shard is not None else 0
    # one buffer: [counts 32 B][chunks cap][sels cap][item_of cap][index chunks ni][index items ni]
    o_ch = 32
    o_se = o_ch + cap * _CH_SZ
    o_io = o_se + cap * _SEL_SZ
    o_ix = o_io + 4 * cap + (-(4 * cap) % 16)
    o_ii = o_ix + ni * _CH_SZ
    buf = np.empty(o_ii + 4 * ni + 16, np.uint8)
    buf[:32] = 0
    b = buf.ctypes.data
    rc = N.lib().zhip_plan_batch(gp, it.ctypes.data, n, res_p, b + o_ch, cap, b, b + o_se, cap, b + 8,
                                 b + o_io, b + o_ix, b + o_ii, b + 12, b + 16)
    del keep
    nc, c1, n_sels, n_idx, agg = _struct.unpack_from("<5I", buf, 0)
    if rc == N.E_BOUNDS and nc == 0 and c1 == 0 and chain.shard is not None and resolved is None:
        raise ValueError("shard blob is shorter than its index")
    N.check(rc, "zhip_plan_batch")
    chunks = np.frombuffer(buf, CHUNK_DT, nc, o_ch)
    sels = np.frombuffer(buf, SEL_DT, n_sels, o_se)
    item_of = np.frombuffer(buf, np.uint32, nc, o_io).astype(np.int64)
    al = out_base_ptr % 16 == 0 and bool(agg & N.AGG_OUT_ALIGNED)
    fast = fast_l and al and bool(agg & N.AGG_LAST_FULL)
    tile = not fast and tile_l and al and bool(agg & N.AGG_ALL_FULL)
    rows = fast and rows_l and bool(agg & N.AGG_UNIT_STEPS)
    t = Tables(layout, chunks, sels, fast, item_of, tile=tile, rows=rows)
    if n_idx:
        t.index_layout = index_layout
        t.index_chunks = np.frombuffer(buf, CHUNK_DT, n_idx, o_ix)
        t.index_item = np.frombuffer(buf, np.uint32, n_idx, o_ii).astype(np.int64)
    return t


_MORTON_RANK: dict = {}


def _morton_rank(cps: tuple) -> np.ndarray:
    """Morton rank of every C-order inner-chunk slot of a shard (memoised)."""
    r = _MORTON_RANK.get(cps)
    if r is None:
        morton = morton_order(cps)
        cstr = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
        r = np.zeros(int(np.prod(cps)), np.int64)
        r[(morton * cstr[None, :]).sum(axis=1)] = np.arange(len(morton))
        if len(_MORTON_RANK) < 64:
            _MORTON_RANK[cps] = r
    return r


def predict_rows(t: Tables, chain: ChainInfo, spec: ArraySpec, src_size: int) -> None:
    """Load-address prediction for a whole-row batch (zhip_decode_predicted).

    Predicts each entry's payload address with the writers' default packing --
    unsharded: the blob itself; sharded: inner chunks in Morton order
    (ShardingCodec._subchunk_order_iter, sharding.py:1090-1107), each
    `encoded size` bytes, after the index when it is at the start -- sorts the
    entries by that address and, when the sorted addresses follow
    base + (c // per) * outer + (c % per) * inner, records the prediction in
    `t.predict`.  Every predicted range is checked to lie inside its entry's
    blob and inside src, so a wrong guess (another writer's packing, elided
    inner chunks) only costs the kernel a reload, never a wild read.  The
    kernel always checks the guess against the live index."""
    if not t.rows or len(t.chunks) == 0:
        return
    ch = t.chunks
    if np.any(ch["flags"] & N.CF_MISSING):
        return
    L = t.layout
    nbytes = int(L.nbytes)
    E = (nbytes + 15) & ~15
    if L.flags & N.LF_SHARDED:
        sh = chain.shard
        cps = tuple(int(c) for c in sh.chunks_per_shard(spec.shape))
        rank_of_slot = _morton_rank(cps)
        elen = nbytes + (4 if chain.inner.crc else 0)
        start = int(L.index_size) if L.flags & N.LF_INDEX_START else 0
        pred = ch["src"].astype(np.int64) + start + rank_of_slot[ch["slot"].astype(np.int64)] * elen
        blob_end = ch["src"].astype(np.int64) + ch["src_len"].astype(np.int64)
        if np.any(pred + E > blob_end):
            return
    else:
        pred = ch["src"].astype(np.int64)
    if np.any(pred < 0) or np.any(pred + E > src_size):
        return
    order = np.argsort(pred, kind="stable")
    ps = pred[order]
    n = len(ps)
    inner = int(ps[1] - ps[0]) if n > 1 else 0
    per = 1
    while per < n and int(ps[per] - ps[per - 1]) == inner:
        per += 1
    outer = int(ps[per] - ps[0]) if per < n else 0
    c = np.arange(n, dtype=np.int64)
    if inner < 0 or outer < 0 or not np.array_equal(ps, ps[0] + (c // per) * outer + (c % per) * inner):
        return
    t.chunks = ch[order]
    t.item_of_chunk = t.item_of_chunk[order]
    t.predict = N.Predict(int(ps[0]), outer, inner, per, 0)

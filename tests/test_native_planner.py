"""The native host planner (zhip_plan_batch, zarr-python_amd/csrc/planner.cpp)
against the Python planner it replaces on the per-call path
(zarr_hip.planner.plan_decode with ZARR_HIP_NATIVE_PLANNER off): for seeded
random geometries -- 1- to 4-d, edge chunks, sharded or not, either index
location, transposes, C / F outs, strided and integer selections, missing
items, stacked outs -- both must produce the same tables byte for byte
(chunk records, deduplicated selections, index checks, kernel flags).  CPU
only: nothing is launched."""

import numpy as np
import pytest

from oracle import oracle as O


def _tables(native: bool, chain, spec, items, ostr, base, drop_axes=(), extra=None):
    from zarr_hip import planner

    keep = planner.NATIVE_PLANNER
    planner.NATIVE_PLANNER = native
    try:
        return planner.plan_decode(chain, spec, items, ostr, base, drop_axes, None, extra)
    finally:
        planner.NATIVE_PLANNER = keep


def _same(a, b):
    assert bytes(a.layout) == bytes(b.layout)
    assert a.chunks.tobytes() == b.chunks.tobytes()
    assert a.sels.tobytes() == b.sels.tobytes()
    assert (a.fast, a.tile, a.rows) == (b.fast, b.tile, b.rows)
    assert np.array_equal(np.asarray(a.item_of_chunk, np.int64), np.asarray(b.item_of_chunk, np.int64))
    assert (a.index_chunks is None) == (b.index_chunks is None)
    if a.index_chunks is not None:
        assert a.index_chunks.tobytes() == b.index_chunks.tobytes()
        assert np.array_equal(a.index_item, b.index_item)
        assert bytes(a.index_layout) == bytes(b.index_layout)


def _rand_sel(rng, shape):
    sel = []
    for n in shape:
        r = rng.random()
        if r < 0.15:
            sel.append(int(rng.integers(0, n)))
        elif r < 0.35:
            a = int(rng.integers(0, n))
            sel.append(slice(a, int(rng.integers(a, n + 1)), int(rng.integers(1, 4))))
        elif r < 0.6:
            a = int(rng.integers(0, n))
            sel.append(slice(a, int(rng.integers(a + 1, n + 1))))
        else:
            sel.append(slice(None))
    return tuple(sel)


@pytest.mark.parametrize("seed", range(60))
def test_native_planner_matches_python(seed):
    from zarr_hip import HipCodecPipeline, planner
    from zarr_hip.spec import ArraySpec

    rng = np.random.default_rng(seed)
    ndim = int(rng.integers(1, 5))
    sharded = bool(rng.integers(0, 2)) or ndim == 1
    dtype = np.dtype(["u1", "<i2", "<f4", "<f8"][int(rng.integers(0, 4))])
    inner = tuple(int(rng.choice([2, 4, 8, 16])) for _ in range(ndim))
    if sharded:
        chunk = tuple(i * int(rng.integers(1, 4)) for i in inner)
    else:
        chunk = tuple(int(rng.integers(2, 20)) for _ in range(ndim))
    shape = tuple(c * int(rng.integers(1, 4)) - int(rng.integers(0, c)) for c in chunk)
    le = {"name": "bytes", "configuration": {"endian": "little" if rng.random() < 0.7 else "big"}}
    crc = [{"name": "crc32c"}] if rng.random() < 0.7 else []
    aa = []
    if ndim > 1 and rng.random() < 0.4:
        aa = [{"name": "transpose", "configuration": {"order": [int(x) for x in rng.permutation(ndim)]}}]
    if sharded:
        codecs = [{"name": "sharding_indexed", "configuration": {
            "chunk_shape": list(inner), "codecs": aa + [le] + crc,
            "index_location": "start" if rng.random() < 0.3 else "end",
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}]
            + ([{"name": "crc32c"}] if rng.random() < 0.8 else [])}}]
    else:
        codecs = aa + [le] + crc
    spec = ArraySpec(chunk, dtype, 0)
    pipe = HipCodecPipeline.from_codecs(codecs).evolve_from_array_spec(spec)
    chain = planner.analyze_chain(pipe.codecs, spec)
    for trial in range(4):
        sel = _rand_sel(rng, shape)
        projections, out_shape = O.basic_indexer(sel, shape, chunk)
        if not projections:
            continue
        order = "F" if rng.random() < 0.3 else "C"
        isz = dtype.itemsize
        strides = []
        acc = isz
        dims = list(range(len(out_shape)))
        for d in (reversed(dims) if order == "C" else dims):
            strides.append(acc)
            acc *= max(out_shape[d], 1)
        ostr = list(reversed(strides)) if order == "C" else strides
        items = []
        top = 0
        for k, (coords, csel, osel, _) in enumerate(projections):
            n = int(rng.integers(200, 5000)) + (16 * int(np.prod([c // i for c, i in zip(chunk, inner)])) + 4
                                                 if sharded else 0)
            items.append((top, n, bool(rng.random() < 0.15), csel, osel))
            top += n + 64
        base = 256 * int(rng.integers(0, 4)) + (16 if rng.random() < 0.1 else 0)
        extra = None
        if rng.random() < 0.2:
            extra = [int(x) * 4096 for x in rng.integers(0, 8, size=len(items))]
        a = _tables(True, chain, spec, items, ostr, base, (), extra)
        b = _tables(False, chain, spec, items, ostr, base, (), extra)
        _same(a, b)


def test_native_planner_headline_and_short_blob():
    import workloads as W
    from zarr_hip import HipCodecPipeline, planner
    from zarr_hip.spec import ArraySpec

    g = W.HEADLINE
    spec = ArraySpec(g["shards"], np.dtype("float32"), 0.0)
    codecs = [{"name": "sharding_indexed", "configuration": {"chunk_shape": list(g["inner"]),
                                                             "codecs": [W.LE, W.CRC]}}]
    pipe = HipCodecPipeline.from_codecs(codecs).evolve_from_array_spec(spec)
    chain = planner.analyze_chain(pipe.codecs, spec)
    blob = 8 * (1048576 + 4) + 8 * 16 + 4
    projections, out_shape = O.basic_indexer((Ellipsis,), g["shape"], g["shards"])
    items = [(k * (blob + 256), blob, False, cs, os_) for k, (_, cs, os_, _) in enumerate(projections)]
    ostr = [256 * 256 * 4, 256 * 4, 4]
    a = _tables(True, chain, spec, items, ostr, 0)
    _same(a, _tables(False, chain, spec, items, ostr, 0))
    assert a.fast and a.rows and len(a.chunks) == 64 and len(a.sels) == 1 and len(a.index_chunks) == 8
    short = [(0, 100, False) + items[0][3:]]
    for native in (True, False):
        with pytest.raises(ValueError, match="shorter than its index"):
            _tables(native, chain, spec, short, ostr, 0)


@pytest.mark.parametrize("seed", range(30))
def test_native_planner_host_staged_matches_python(seed):
    """Host-staged partial shard reads (plan_decode's `resolved`: inner chunks
    fetched and staged by staging.gather_sharded_partial): items are inner-chunk
    selections sharing their shards' staged tables, some shards absent, some
    inner chunks absent, with and without an index check."""
    from zarr_hip import HipCodecPipeline, planner
    from zarr_hip.spec import ArraySpec

    rng = np.random.default_rng(1000 + seed)
    ndim = int(rng.integers(2, 4))
    inner = tuple(int(rng.choice([2, 4, 8])) for _ in range(ndim))
    cps = tuple(int(rng.integers(1, 4)) for _ in range(ndim))
    shard = tuple(i * c for i, c in zip(inner, cps))
    n_inner = int(np.prod(cps))
    crc_ix = bool(rng.random() < 0.7)
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(inner), "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                               {"name": "crc32c"}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}]
        + ([{"name": "crc32c"}] if crc_ix else [])}}]
    spec = ArraySpec(shard, np.dtype("<f4"), 0.0)
    pipe = HipCodecPipeline.from_codecs(codecs).evolve_from_array_spec(spec)
    chain = planner.analyze_chain(pipe.codecs, spec)
    n_shards = int(rng.integers(1, 6))
    tables = []
    top = 0
    for s in range(n_shards):
        if rng.random() < 0.15:
            tables.append(None)
            continue
        src_by = np.zeros(n_inner, np.int64)
        len_by = np.zeros(n_inner, np.int64)
        miss_by = rng.random(n_inner) < 0.2
        for j in range(n_inner):
            if not miss_by[j]:
                src_by[j], len_by[j] = top, 4 * int(np.prod(inner)) + 4
                top += int(len_by[j]) + 16
        tables.append((src_by, len_by, miss_by, top if crc_ix else -1))
        top += 256
    items, resolved = [], []
    out_rows = 0
    for k in range(int(rng.integers(3, 20))):
        s = int(rng.integers(0, n_shards))
        c = [int(rng.integers(0, x)) for x in cps]
        csel = tuple(slice(ci * i, ci * i + i, 1) for ci, i in zip(c, inner))
        osel = (slice(out_rows, out_rows + inner[0]),) + tuple(slice(0, i) for i in inner[1:])
        out_rows += inner[0]
        items.append((0, 0, tables[s] is None, csel, osel))
        resolved.append(tables[s])
    isz = 4
    ostr = []
    acc = isz
    oshape = (out_rows,) + inner[1:]
    for d in reversed(range(ndim)):
        ostr.append(acc)
        acc *= oshape[d]
    ostr = list(reversed(ostr))
    keep = planner.NATIVE_PLANNER
    try:
        planner.NATIVE_PLANNER = True
        a = planner.plan_decode(chain, spec, items, ostr, 0, (), resolved, None)
        planner.NATIVE_PLANNER = False
        b = planner.plan_decode(chain, spec, items, ostr, 0, (), resolved, None)
    finally:
        planner.NATIVE_PLANNER = keep
    _same(a, b)

"""Host planner checks (CPU): projections equal the oracle's BasicIndexer
restatement; chain analysis folds transposes into a stored-dim permutation;
Morton orders match the reference's literal vectors."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from zarr_hip import codecs as C
from zarr_hip.indexing import basic_projections, chunk_batch, morton_order, subchunk_order, to_chunk_selection
from zarr_hip.planner import analyze_chain
from zarr_hip.spec import ArraySpec

SELECTIONS = [
    (Ellipsis,), (slice(None),), (slice(3, 17), slice(None, None, 3)), (5, slice(2, 30, 7)),
    (slice(0, 0),), (slice(30, 5),), (-1, -2), (slice(1, 40, 13), 0), (slice(None), slice(9, 10)),
]


@pytest.mark.parametrize("sel", SELECTIONS)
@pytest.mark.parametrize("shape,chunks", [((37, 29), (8, 10)), ((16, 16), (16, 16)),
                                          ((40, 31), (7, 31))])
def test_projections_match_oracle(sel, shape, chunks):
    pr = basic_projections(sel, shape, chunks)
    want, want_shape = O.basic_indexer(sel, shape, chunks)
    assert pr.out_shape == want_shape
    got = []
    for i in range(len(pr.coords)):
        csel, osel = to_chunk_selection(pr, i)
        got.append((tuple(int(c) for c in pr.coords[i]), csel, osel, bool(pr.complete[i])))

    def norm(rows):
        out = []
        for coords, csel, osel, comp in rows:
            cs = tuple(s if isinstance(s, int) else tuple(range(*s.indices(10**6))) for s in csel)
            os_ = tuple(tuple(range(*s.indices(10**6))) for s in osel)
            out.append((coords, cs, os_, comp))
        return sorted(out)

    assert norm(got) == norm(want)
    # the batch builder (lists, Array.batch_info) gives the same rows in the same order
    rows, shape_b = chunk_batch(sel, shape, chunks)
    assert shape_b == pr.out_shape
    assert [(tuple(c), cs, os_, cp) for c, cs, os_, cp in rows] == got


def test_chunk_batch_long_dims_match_projections():
    rng = np.random.default_rng(3)
    for _ in range(40):
        n = int(rng.integers(1, 5000))
        c = int(rng.integers(1, 9))
        a, b = sorted(int(x) for x in rng.integers(0, n + 1, 2))
        st = int(rng.integers(1, 6))
        sel = (slice(a, b, st),)
        pr = basic_projections(sel, (n,), (c,))
        rows, out_shape = chunk_batch(sel, (n,), (c,))
        assert out_shape == pr.out_shape
        assert [(co, cs, os_, cp) for co, cs, os_, cp in rows] == [
            ((int(pr.coords[i][0]),), *to_chunk_selection(pr, i), bool(pr.complete[i]))
            for i in range(len(pr.coords))]


def test_morton_matches_reference_vectors():
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "morton_exact.json")))
    for case in d["cases"]:
        assert morton_order(tuple(case["shape"])).tolist() == case["order"]


@pytest.mark.parametrize("shape", [(3, 2), (5, 5, 5), (2, 9, 2), (4, 3, 6, 2, 7), (1,)])
@pytest.mark.parametrize("order", ["morton", "lexicographic", "colexicographic"])
def test_subchunk_orders_match_oracle(shape, order):
    assert [tuple(c) for c in subchunk_order(shape, order).tolist()] == \
        O.subchunk_order(shape, order)


def test_chain_analysis_permutation():
    spec = ArraySpec((4, 5, 6), "float32", 0.0)
    ch = analyze_chain(C.parse_codecs([{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                       {"name": "bytes", "configuration": {"endian": "big"}},
                                       {"name": "crc32c"}]), spec)
    # stored shape (6, 4, 5): stored dim i is decoded dim perm[i]
    assert ch.perm == (2, 0, 1) and ch.swap and ch.crc
    a = np.arange(120, dtype="f4").reshape(4, 5, 6)
    stored = O.transpose_encode(a, (2, 0, 1))
    assert stored.shape == tuple(a.shape[p] for p in ch.perm)
    two = analyze_chain(C.parse_codecs([{"name": "transpose", "configuration": {"order": [1, 2, 0]}},
                                        {"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                        {"name": "bytes", "configuration": {"endian": "little"}}]),
                        spec)
    s = O.transpose_encode(O.transpose_encode(a, (1, 2, 0)), (2, 0, 1))
    assert s.shape == tuple(a.shape[p] for p in two.perm)


def test_codec_order_errors():
    with pytest.raises(ValueError):
        C.split_codecs(C.parse_codecs([{"name": "bytes"}, {"name": "bytes"}]))
    with pytest.raises(ValueError):
        C.split_codecs(C.parse_codecs([{"name": "transpose", "configuration": {"order": [0]}}]))
    with pytest.raises(TypeError):
        C.split_codecs(C.parse_codecs([{"name": "crc32c"}, {"name": "bytes"}]))
    with pytest.raises(NotImplementedError):
        C.parse_codecs([{"name": "zstd", "configuration": {"level": 1}}])
    with pytest.raises(TypeError):  # a compressor is a BytesBytesCodec too
        C.split_codecs(C.parse_codecs([{"name": "gzip", "configuration": {"level": 1}}, {"name": "bytes"}]))
    with pytest.raises(ValueError):
        C.parse_codecs([{"name": "gzip", "configuration": {"level": 11}}])


def test_split_host_tail():
    """The host stage starts at the first compressor; a crc32c after it stays
    on the host (it checks the compressed bytes); every bytes->bytes codec
    after a sharding codec is host-side."""
    LE = {"name": "bytes", "configuration": {"endian": "little"}}
    GZ = {"name": "gzip", "configuration": {"level": 1}}
    CRC = {"name": "crc32c"}
    T = {"name": "transpose", "configuration": {"order": [1, 0]}}
    SH = {"name": "sharding_indexed", "configuration": {"chunk_shape": [2, 2], "codecs": [LE, GZ]}}

    def names(cs):
        return [c.to_dict()["name"] for c in cs]

    for chain, gpu, host in [([LE, CRC], ["bytes", "crc32c"], []),
                             ([LE, GZ], ["bytes"], ["gzip"]),
                             ([T, LE, CRC, GZ], ["transpose", "bytes", "crc32c"], ["gzip"]),
                             ([LE, GZ, CRC], ["bytes"], ["gzip", "crc32c"]),
                             ([SH, CRC], ["sharding_indexed"], ["crc32c"])]:
        g, h = C.split_host_tail(C.parse_codecs(chain))
        assert names(g) == gpu and names(h) == host, chain
    sh = C.parse_codecs([SH])[0]
    assert names(C.split_host_tail(sh.codecs)[1]) == ["gzip"]


def _sharded_headline_tables(loc="end", shape=(256, 256, 256), shards=(128, 128, 128),
                             inner=(64, 64, 64)):
    """Plan the headline-shaped full read exactly as prepare_read would, with the
    shard blobs where a DeviceStore written in key order puts them (256-aligned,
    consecutive) -- host logic only, no device."""
    import zarr_hip.planner as P
    from zarr_hip.codecs import parse_codecs

    LE = {"name": "bytes", "configuration": {"endian": "little"}}
    codecs = parse_codecs([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(inner), "codecs": [LE, {"name": "crc32c"}],
        "index_codecs": [LE, {"name": "crc32c"}], "index_location": loc}}])
    spec = ArraySpec(shards, "float32", 0.0)
    chain = analyze_chain(codecs, spec)
    n_inner = int(np.prod([s // c for s, c in zip(shards, inner)]))
    elen = int(np.prod(inner)) * 4 + 4
    blob = n_inner * elen + 16 * n_inner + 4
    stride = (blob + 255) // 256 * 256
    grid = [s // k for s, k in zip(shape, shards)]
    items = []
    for i, sc in enumerate(np.ndindex(*grid)):
        csel = tuple(slice(0, k, 1) for k in shards)
        osel = tuple(slice(c * k, (c + 1) * k, 1) for c, k in zip(sc, shards))
        items.append((i * stride, blob, False, csel, osel))
    ostr = [shape[1] * shape[2] * 4, shape[2] * 4, 4]
    t = P.plan_decode(chain, spec, items, ostr, 0, ())
    return P, t, chain, spec, stride, elen, len(items) * stride


@pytest.mark.parametrize("loc", ["end", "start"])
def test_predict_rows_fits_default_packing(loc):
    """planner.predict_rows: entries sorted by predicted address follow one
    2-level progression (shards x Morton-ranked inner chunks) and every
    prediction lies inside its blob (zhip_predict contract)."""
    P, t, chain, spec, stride, elen, size = _sharded_headline_tables(loc)
    assert t.rows
    items_before = sorted(t.item_of_chunk.tolist())
    P.predict_rows(t, chain, spec, size)
    pr = t.predict
    assert pr is not None
    assert (pr.per, pr.inner, pr.outer) == (8, elen, stride)
    assert pr.base == (16 * 8 + 4 if loc == "start" else 0)
    c = np.arange(len(t.chunks))
    pred = pr.base + (c // pr.per) * pr.outer + (c % pr.per) * pr.inner
    # the sorted entries' own blob + Morton rank give exactly the prediction
    from zarr_hip.indexing import morton_order

    m = morton_order((2, 2, 2))
    rank_of_slot = np.zeros(8, np.int64)
    rank_of_slot[(m * np.array([4, 2, 1])[None, :]).sum(axis=1)] = np.arange(8)
    start = 16 * 8 + 4 if loc == "start" else 0
    want = t.chunks["src"].astype(np.int64) + start + rank_of_slot[t.chunks["slot"].astype(np.int64)] * elen
    assert np.array_equal(pred, want)
    assert np.all(pred + elen <= t.chunks["src"].astype(np.int64) + t.chunks["src_len"].astype(np.int64))
    assert sorted(t.item_of_chunk.tolist()) == items_before  # a permutation of the entries


def test_predict_rows_declines_missing_and_irregular():
    P, t, chain, spec, stride, elen, size = _sharded_headline_tables()
    t.chunks["flags"][3] = 1  # a missing shard
    P.predict_rows(t, chain, spec, size)
    assert t.predict is None
    P, t, chain, spec, stride, elen, size = _sharded_headline_tables()
    t.chunks["src"][5:] += 256  # blobs no longer equally spaced
    P.predict_rows(t, chain, spec, size + 256)
    assert t.predict is None
    P, t, chain, spec, stride, elen, size = _sharded_headline_tables()
    P.predict_rows(t, chain, spec, size - 4096)  # a prediction past the end of src
    assert t.predict is None


def test_plan_encode_tile_modes():
    """Transposed encodes: full chunks -> tile (k_encode_tile4 / k_encode_tileg
    by the library), edge chunks with prefix-box selections -> tile_prefix
    (k_encode_tile); strided selections -> neither (persistent k_encode)."""
    from zarr_hip.planner import plan_encode
    from zarr_hip.spec import ArraySpec

    codecs = C.parse_codecs([{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
                             {"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}])
    spec = ArraySpec((64, 48, 32), np.dtype("float32"), 0.0)
    chain = analyze_chain(codecs, spec)
    astr = [72 * 48 * 4, 48 * 4, 4]  # a (100, 72, 48) float32 array, C order, byte strides
    full = tuple(slice(0, n, 1) for n in (64, 48, 32))
    t = plan_encode(chain, spec, [(0, full, [0, 0, 0])], astr, 0)
    assert t.tile and not t.tile_prefix
    edge = (slice(0, 36, 1), slice(0, 48, 1), slice(0, 16, 1))
    t = plan_encode(chain, spec, [(0, full, [0, 0, 0]), (1 << 20, edge, [64, 0, 32])], astr, 0)
    assert t.tile_prefix and not t.tile
    strided = (slice(0, 64, 2), slice(0, 48, 1), slice(0, 32, 1))
    t = plan_encode(chain, spec, [(0, strided, [0, 0, 0])], astr, 0)
    assert not t.tile and not t.tile_prefix

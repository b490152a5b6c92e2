"""Host planner checks (CPU): projections equal the oracle's BasicIndexer
restatement; chain analysis folds transposes into a stored-dim permutation;
Morton orders match the reference's literal vectors."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from zarr_hip import codecs as C
from zarr_hip.indexing import basic_projections, morton_order, subchunk_order, to_chunk_selection
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
        C.parse_codecs([{"name": "gzip", "configuration": {"level": 1}}])

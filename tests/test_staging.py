"""Host-side IO planning for staged reads: byte requests, coalesce_ranges and
Store.get_ranges_sync, restating the reference's cases
(tests/test_coalesce.py:148-268, 549-640 of zarr-python)."""

import numpy as np
import pytest

from zarr_hip.store import (LocalStore, MemoryStore, OffsetByteRequest, RangeByteRequest,
                            SuffixByteRequest, coalesce_ranges)

BLOB = bytes(i % 256 for i in range(10_000))
MERGE_GAP_50 = {"max_gap_bytes": 50, "max_coalesced_bytes": 1 << 20}
CAP_50 = {"max_gap_bytes": 1000, "max_coalesced_bytes": 50}
DEFAULT = {"max_gap_bytes": 1 << 20, "max_coalesced_bytes": 16 << 20}
R = RangeByteRequest

CASES = [
    ("empty-input", [], DEFAULT, []),
    ("single-range", [R(2, 5)], DEFAULT, [1]),
    ("disjoint-3-no-merge", [R(0, 10), R(200, 210), R(500, 510)], MERGE_GAP_50, [1, 1, 1]),
    ("adjacent-3-one-merged-group", [R(0, 5), R(10, 15), R(20, 25)], MERGE_GAP_50, [3]),
    ("two-clusters-one-singleton", [R(0, 10), R(20, 30), R(500, 510)], MERGE_GAP_50, [1, 2]),
    ("shuffled-input-indices-preserved", [R(500, 510), R(0, 10), R(200, 210), R(300, 310)],
     MERGE_GAP_50, [1, 1, 1, 1]),
    ("cap-prevents-merge-of-close-ranges", [R(0, 20), R(40, 60)], CAP_50, [1, 1]),
    ("single-range-larger-than-cap-passes-through", [R(0, 200)], CAP_50, [1]),
]


@pytest.mark.parametrize("name,ranges,opts,sizes", CASES, ids=[c[0] for c in CASES])
def test_coalesce_structure(name, ranges, opts, sizes):
    groups, other = coalesce_ranges(ranges, **opts)
    assert other == []
    assert sorted(len(g) for g in groups) == sorted(sizes)


@pytest.mark.parametrize("name,ranges,opts,sizes", CASES, ids=[c[0] for c in CASES])
def test_get_ranges_contents(name, ranges, opts, sizes):
    st = MemoryStore({"k": BLOB})
    got = dict(st.get_ranges_sync("k", ranges, **opts))
    assert sorted(got) == list(range(len(ranges)))
    for i, r in enumerate(ranges):
        assert bytes(got[i]) == BLOB[r.start:r.end]


def test_uncoalescable_mixed():
    ranges = [R(0, 10), OffsetByteRequest(100), SuffixByteRequest(5), None, R(20, 30)]
    groups, other = coalesce_ranges(ranges, **MERGE_GAP_50)
    assert len(groups) == 1 and [i for i, _ in groups[0]] == [0, 4]
    assert [(i, type(r).__name__ if r else None) for i, r in other] == [
        (1, "OffsetByteRequest"), (2, "SuffixByteRequest"), (3, None)]
    got = dict(MemoryStore({"k": BLOB}).get_ranges_sync("k", ranges, **MERGE_GAP_50))
    assert bytes(got[1]) == BLOB[100:]
    assert bytes(got[2]) == BLOB[-5:]
    assert bytes(got[3]) == BLOB


def test_groups_sorted_by_start_and_overlaps_merge():
    groups, _ = coalesce_ranges([R(500, 510), R(0, 10), R(20, 30), R(200, 210)], **MERGE_GAP_50)
    assert [i for g in groups for i, _ in g] == [1, 2, 3, 0]
    groups, _ = coalesce_ranges([R(0, 100), R(50, 60), R(80, 120)], **MERGE_GAP_50)
    assert len(groups) == 1 and [i for i, _ in groups[0]] == [0, 1, 2]


def test_coverage_random():
    rng = np.random.default_rng(3)
    st = MemoryStore({"k": BLOB})
    for _ in range(20):
        ranges = []
        for _ in range(rng.integers(1, 30)):
            a = int(rng.integers(0, 9900))
            ranges.append(R(a, a + int(rng.integers(0, 100))))
        got = dict(st.get_ranges_sync("k", ranges, max_gap_bytes=int(rng.integers(-1, 500)),
                                      max_coalesced_bytes=int(rng.integers(1, 2000))))
        assert sorted(got) == list(range(len(ranges)))
        for i, r in enumerate(ranges):
            assert bytes(got[i]) == BLOB[r.start:r.end]


def test_missing_key_raises():
    with pytest.raises(FileNotFoundError):
        MemoryStore({}).get_ranges_sync("k", [R(0, 1)])


def test_local_store_byte_requests(tmp_path):
    st = LocalStore(str(tmp_path))
    st.set_sync("a/b", BLOB)
    assert bytes(st.get_sync("a/b", SuffixByteRequest(7))) == BLOB[-7:]
    assert bytes(st.get_sync("a/b", OffsetByteRequest(9990))) == BLOB[9990:]
    assert bytes(st.get_sync("a/b", R(5, 9))) == BLOB[5:9]
    got = dict(st.get_ranges_sync("a/b", [R(0, 4), R(8000, 8010)]))
    assert bytes(got[1]) == BLOB[8000:8010]


def test_staging_layout_alignment():
    from zarr_hip.staging import StagingLayout

    lay = StagingLayout()
    offs = [lay.add(b"x" * n)[0] for n in (1, 300, 0, 256, 7)]
    assert all(o % 256 == 0 for o in offs)
    assert offs == [0, 256, 768, 768, 1024]


# ------------------------------------------- slab groups of host-out reads
def _batch_for(shape, chunks, sel=(Ellipsis,)):
    from zarr_hip.indexing import chunk_batch

    rows, out_shape = chunk_batch(sel, shape, chunks)
    return [(None, None, csel, osel, comp) for _, csel, osel, comp in rows], out_shape


@pytest.mark.parametrize("shape,chunks,sel", [
    ((256, 256, 128), (64, 64, 64), (Ellipsis,)),
    ((256, 256, 128), (64, 64, 64), (slice(5, 250), slice(None), slice(3, 128))),
    ((512, 64, 64), (48, 64, 64), (Ellipsis,)),      # ragged last slab
    ((256, 128, 128), (32, 64, 64), (7, slice(None), slice(None))),
])
def test_slab_groups_partition_out_rows(shape, chunks, sel):
    """HipCodecPipeline._read_slabs' groups: disjoint byte ranges of out in
    row order, every item in exactly one group, each item's rows inside its
    group's range."""
    import torch

    from zarr_hip.pipeline import _slab_groups

    batch, out_shape = _batch_for(shape, chunks, sel)
    out = torch.empty(out_shape, dtype=torch.float32)
    g = _slab_groups(batch, out)
    if out.numel() * 4 < 16 << 20:
        assert g is None
        return
    assert g is not None and len(g) >= 2
    row_bytes = out[0].numel() * 4
    assert sorted(i for _, _, idx in g for i in idx) == list(range(len(batch)))
    for (a0, b0, _), (a1, b1, _) in zip(g, g[1:]):
        assert b0 <= a1
    for a, b, idx in g:
        for i in idx:
            r = batch[i][3][0]
            assert a <= r.start * row_bytes and r.stop * row_bytes <= b


def test_slab_groups_declines():
    import torch

    from zarr_hip.pipeline import _slab_groups

    batch, out_shape = _batch_for((256, 256, 128), (64, 64, 64))
    assert _slab_groups(batch, torch.empty(out_shape, dtype=torch.float32).transpose(0, 1)) is None  # strided
    one_row, shp = _batch_for((64, 512, 512), (64, 64, 64))  # a single chunk row along dim 0
    assert _slab_groups(one_row, torch.empty(shp, dtype=torch.float32)) is None


def test_touched_slots_matches_projection():
    """staging._touched_slots (interval arithmetic for ints and unit-step
    slices) names exactly the inner chunks basic_projections touches; other
    selection forms return None (the caller projects)."""
    import numpy as np

    from zarr_hip.indexing import basic_projections
    from zarr_hip.staging import _touched_slots

    rng = np.random.default_rng(7)
    shape, inner = (12, 20, 9), (4, 5, 3)
    cps = [s // c for s, c in zip(shape, inner)]
    strides = np.array([int(np.prod(cps[d + 1:])) for d in range(3)])
    for _ in range(500):
        sel = []
        for n in shape:
            r = rng.integers(0, 3)
            if r == 0:
                sel.append(int(rng.integers(-n, n)))
            else:
                a = int(rng.integers(0, n))
                b = int(rng.integers(a, n + 1))
                sel.append(slice(a, b, None if r == 1 else 1))
        sel = tuple(sel)
        want = {int(x) for x in (basic_projections(sel, shape, inner).coords * strides).sum(axis=1)}
        assert set(_touched_slots(sel, shape, inner, strides)) == want, sel
    assert _touched_slots((slice(0, 12, 2), slice(None), slice(None)), shape, inner, strides) is None

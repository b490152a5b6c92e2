"""Host half of nested sharding (zarr_hip/nested.py), on the CPU: chain
detection, the cell projection of an item's selection onto the inner shards,
out-selection composition, and the outer-index read with its CRC check (the
GPU half runs in tests/test_gpu_pipeline_suite.py's nested scenarios)."""

import numpy as np
import pytest

from oracle import oracle as O

LE = {"name": "bytes", "configuration": {"endian": "little"}}


def _nest(outer, inner, loc="end"):
    return {"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(outer), "index_location": loc,
        "codecs": [{"name": "sharding_indexed", "configuration": {"chunk_shape": list(inner), "codecs": [LE]}}]}}


def test_nested_split_detects_only_nested_chains():
    from zarr_hip import HipCodecPipeline, nested

    assert nested.nested_split(HipCodecPipeline.from_codecs([LE])) is None
    flat = {"name": "sharding_indexed", "configuration": {"chunk_shape": [4, 4], "codecs": [LE]}}
    assert nested.nested_split(HipCodecPipeline.from_codecs([flat])) is None
    outer = nested.nested_split(HipCodecPipeline.from_codecs([_nest((10, 10), (5, 5))]))
    assert outer is not None and outer.chunk_shape == (10, 10)
    with pytest.raises(NotImplementedError):
        nested.nested_split(HipCodecPipeline.from_codecs([_nest((10, 10), (5, 5)), {"name": "crc32c"}]))


def test_cells_and_composed_out_selection():
    """Each touched inner shard with its own selection and its out region;
    the regions tile the item's out selection exactly."""
    from zarr_hip import HipCodecPipeline, nested
    from zarr_hip.spec import ArraySpec

    outer = nested.nested_split(HipCodecPipeline.from_codecs([_nest((10, 15), (5, 5))]))
    spec = ArraySpec((20, 30), np.dtype("int32"), 0)
    csel = (slice(3, 17), slice(4, 29))
    cps, cells = nested._cells(outer, spec, csel)
    assert cps == (2, 2)
    assert sorted(c[0] for c in cells) == [0, 1, 2, 3]
    cover = np.zeros((14, 25), int)
    for _, c_csel, c_osel, _ in cells:
        o = nested._compose((slice(100, 114), slice(200, 225)), c_osel)
        cover[o[0].start - 100:o[0].stop - 100, o[1].start - 200:o[1].stop - 200] += 1
        assert (o[0].stop - o[0].start, o[1].stop - o[1].start) == tuple(
            s.stop - s.start for s in c_csel)
    assert (cover == 1).all()
    with pytest.raises(NotImplementedError):
        nested._compose((slice(0, 10, 2),), (slice(0, 5),))


@pytest.mark.parametrize("loc", ["end", "start"])
def test_outer_index_read_and_crc_message(loc):
    """The outer index of an oracle-written nested shard, read through a range
    request; a flipped index bit raises the reference's checksum message."""
    from zarr_hip import HipCodecPipeline, MemoryStore, nested
    from zarr_hip.store import StorePath

    codecs = [_nest((10, 10), (5, 5), loc)]
    meta = O.ArrayMeta((20, 20), (20, 20), np.dtype("int32"), 0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), np.arange(400, dtype="int32").reshape(20, 20))
    outer = nested.nested_split(HipCodecPipeline.from_codecs(codecs))
    st = MemoryStore(dict(host))
    idx = nested._read_index(outer, StorePath(st, "c/0/0"), (20, 20))
    assert idx.shape == (4, 2) and int(idx[:, 1].min()) > 0
    blob = bytearray(host["c/0/0"])
    pos = len(blob) - 2 if loc == "end" else 5
    blob[pos] ^= 1
    bad = MemoryStore({"c/0/0": bytes(blob)})
    with pytest.raises(ValueError, match="Stored and computed checksum do not match"):
        nested._read_index(outer, StorePath(bad, "c/0/0"), (20, 20))
    assert nested._read_index(outer, StorePath(MemoryStore({}), "c/0/0"), (20, 20)) is None

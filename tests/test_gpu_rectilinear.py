"""GPU reads and writes of rectilinear chunk grids (row n3): zarr hands the
pipeline one ArraySpec per chunk, shape = ChunkGrid[coords].codec_shape
(_get_chunk_spec, src/zarr/core/array.py:5373-5390, 5469-5486), so a batch
mixes chunk shapes.  HipCodecPipeline groups the items by spec and plans,
stages and launches each group with its own spec (pipeline.spec_groups).

Cases: the reference's rectilinear metadata fixture geometry (100 x 100 f64,
rows 10/20/30/40, columns 50; packages/zarr-metadata/tests/v3/array/
rectilinear_grid.json), chunks of equal byte size but different shape (a 10 x
20 and a 20 x 10 chunk), and a sharded variant (rectilinear shards of regular
inner chunks).  Reads (full, partial, strided, integer) are compared bit for
bit with the CPU oracle, stores byte for byte."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import BE, CRC, LE, SHARD, _data

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(__file__), "golden", "metadata")

SELS = [(Ellipsis,), (slice(5, 77), slice(None)), (slice(3, 97, 7), slice(1, 99, 3)), (33, slice(None)),
        (slice(None), 49), (slice(29, 61), slice(45, 55))]


def _store(kind, device):
    import zarr_hip

    return zarr_hip.MemoryStore() if kind == "memory" else zarr_hip.DeviceStore(device)


def _check(arr, store, meta, data, sels=SELS):
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert got == host
    for sel in sels:
        want = O.read(host, meta, sel)
        assert np.asarray(arr[sel]).tobytes() == np.ascontiguousarray(want).tobytes()
    return host


@pytest.mark.parametrize("kind", ["memory", "device"])
def test_rectilinear_fixture_roundtrip(kind, device):
    """The reference's fixture document opened from a store, written and read."""
    import zarr_hip

    with open(os.path.join(HERE, "rectilinear_grid.json")) as fh:
        doc = json.load(fh)
    store = _store(kind, device)
    store.set_sync("zarr.json", json.dumps(doc).encode())
    arr = zarr_hip.Array.open(store)
    assert not arr.metadata.is_regular
    data = _data((100, 100), "float64")
    arr[...] = data
    meta = O.ArrayMeta((100, 100), ([10, 20, 30, 40], 50), np.dtype("float64"), 0.0, codecs=doc["codecs"])
    _check(arr, store, meta, data)


@pytest.mark.parametrize("codecs", [[LE, CRC], [BE], [BE, CRC]])
@pytest.mark.parametrize("kind", ["memory", "device"])
def test_same_nbytes_different_shape(kind, codecs, device):
    """Chunks of one byte size and different shapes (10 x 20 and 20 x 10):
    decoding one with the other's spec would scatter wrongly without any
    error, so each must be planned with its own."""
    import zarr_hip

    grid = ([10, 20], [20, 10])
    store = _store(kind, device)
    arr = zarr_hip.Array.create(store, (30, 30), grid, "float32", -1.0, codecs=codecs)
    data = _data((30, 30), "float32")
    arr[...] = data
    meta = O.ArrayMeta((30, 30), grid, np.dtype("float32"), -1.0, codecs=codecs)
    host = _check(arr, store, meta, data, SELS[:1] + [(slice(5, 25), slice(7, 29, 2)), (12, slice(None))])
    assert len(host["c/0/0"]) == len(host["c/1/1"])
    # a partial write into two chunks of different shape, then a missing chunk
    arr[8:14, 15:25] = np.full((6, 10), 7.5, np.float32)
    O.write(host, meta, (slice(8, 14), slice(15, 25)), np.full((6, 10), 7.5, np.float32))
    store.delete_sync("c/1/0")
    host.pop("c/1/0")
    assert np.asarray(arr[...]).tobytes() == O.read(host, meta).tobytes()


@pytest.mark.parametrize("kind", ["memory", "device"])
def test_rectilinear_with_extent_past_edges(kind, device):
    """A varying last chunk reaching past the extent is encoded at its full
    edge (chunk_size), read and written clipped (data_size)."""
    import zarr_hip

    grid = ([10, 20, 30, 40], [16, 48])
    store = _store(kind, device)
    arr = zarr_hip.Array.create(store, (85, 60), grid, "int16", 3, codecs=[LE, CRC])
    data = _data((85, 60), "int16")
    arr[...] = data
    meta = O.ArrayMeta((85, 60), grid, np.dtype("int16"), 3, codecs=[LE, CRC])
    host = _check(arr, store, meta, data)
    assert len(host["c/3/1"]) == 40 * 48 * 2 + 4


@pytest.mark.parametrize("kind", ["memory", "device"])
def test_rectilinear_shards(kind, device):
    """Rectilinear shards of regular inner chunks (each shard edge divisible
    by the inner chunk, sharding.py:567-593): the shard index and its CRC, the
    inner chunks' CRC and scatter per shard shape."""
    import zarr_hip

    shards = ([32, 64, 32], [64, 32])
    store = _store(kind, device)
    arr = zarr_hip.Array.create(store, (128, 96), (16, 32), "float32", 0.5, codecs=[LE, CRC], shards=shards)
    data = _data((128, 96), "float32")
    arr[...] = data
    meta = O.ArrayMeta((128, 96), shards, np.dtype("float32"), 0.5, codecs=[SHARD((16, 32), [LE, CRC])])
    host = _check(arr, store, meta, data, [(Ellipsis,), (slice(20, 111), slice(10, 90)),
                                           (slice(1, 128, 5), slice(None, None, 3)), (40, slice(None))])
    # a partial write (partial shard encode per shard shape), then a corrupted inner chunk
    arr[30:70, 50:70] = np.arange(800, dtype=np.float32).reshape(40, 20)
    O.write(host, meta, (slice(30, 70), slice(50, 70)), np.arange(800, dtype=np.float32).reshape(40, 20))
    got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert got == host
    assert np.asarray(arr[...]).tobytes() == O.read(host, meta).tobytes()
    bad = bytearray(host["c/1/0"])
    bad[100] ^= 0x08
    host["c/1/0"] = bytes(bad)
    store.set_sync("c/1/0", bytes(bad))
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    with pytest.raises(ValueError) as got_err:
        arr[...]
    assert str(got_err.value) == str(want.value)


def test_read_sync_with_zarr_per_chunk_specs(device):
    """The boundary as zarr drives it: a batch of (StorePath, zarr ArraySpec per
    chunk, chunk_selection, out_selection, is_complete) with the specs zarr's
    _get_chunk_spec builds, into one out; then prepare_read of the same batch
    (one program per spec group) and a write of the same shape."""
    import torch
    import zarr_fakes as Z
    import zarr_hip
    from zarr_hip.grid import ChunkGrid
    from zarr_hip.indexing import chunk_batch

    shape = (100, 100)
    g = ChunkGrid.from_sizes(shape, [[10, 20, 30, 40], [60, 40]])
    meta = O.ArrayMeta(shape, ([10, 20, 30, 40], [60, 40]), np.dtype("float64"), 0.0, codecs=[LE, CRC])
    host: dict = {}
    data = _data(shape, "float64")
    O.write(host, meta, (Ellipsis,), data)
    store = zarr_hip.DeviceStore.from_host(host, device)
    pipe = zarr_hip.HipCodecPipeline.from_codecs(Z.zcodecs([LE, CRC])).evolve_from_array_spec(
        Z.ArraySpec((1, 1), Z.ZDType("float64"), 0.0, Z.ArrayConfig(), None))
    sel = (slice(7, 93, 2), slice(3, 97))
    rows, out_shape = chunk_batch(sel, shape, g)
    specs = {}
    batch = []
    for co, csel, osel, comp in rows:
        cs = g.codec_shape(co)
        sp = specs.setdefault(cs, Z.ArraySpec(cs, Z.ZDType("float64"), 0.0, Z.ArrayConfig(), None))
        batch.append((zarr_hip.StorePath(store, "c/" + "/".join(map(str, co))), sp, csel, osel, comp))
    assert len({id(it[1]) for it in batch}) > 2
    out = torch.empty(out_shape, dtype=torch.float64, device=device)
    res = pipe.read_sync(batch, out)
    assert [r["status"] for r in res] == ["present"] * len(batch)
    want = np.ascontiguousarray(O.read(host, meta, sel))
    assert out.cpu().numpy().tobytes() == want.tobytes()
    out.zero_()
    prog = pipe.prepare_read(batch, out)
    prog.launch()
    assert len(prog.results()) == len(batch)
    assert out.cpu().numpy().tobytes() == want.tobytes()
    # writes with the same per-chunk specs
    store2 = zarr_hip.DeviceStore(device)
    rows, _ = chunk_batch((Ellipsis,), shape, g)
    wb = [(zarr_hip.StorePath(store2, "c/" + "/".join(map(str, co))), specs.setdefault(
        g.codec_shape(co), Z.ArraySpec(g.codec_shape(co), Z.ZDType("float64"), 0.0, Z.ArrayConfig(), None)),
        csel, osel, comp) for co, csel, osel, comp in rows]
    pipe.write_sync(wb, torch.from_numpy(data).to(device))
    assert {k: bytes(v) for k, v in store2.to_dict().items()} == host


@pytest.mark.parametrize("codecs", [[LE, CRC], [BE]])
def test_many_distinct_edges_one_synchronisation(codecs, device):
    """A 1-D rectilinear grid of 64 distinct edge lengths (1, 2, ..., 64: an
    RLE-free [[1, 2, 3, ...]] grid, chunk_grids.py:167-293) read whole and
    strided into a device out: 64 spec groups, one plan and one launch each,
    launched back to back, and ONE host synchronisation for the whole batch
    (pipeline.SYNCS); bit-exact with the oracle.  Writes (whole, and a strided
    scalar write whose edge chunks merge with their stored bytes) encode every
    group before ONE readback of their checks and non-empty flags; stores
    byte-identical.  A corrupted chunk still raises the reference's message
    from that single readback."""
    import zarr_hip
    from zarr_hip import pipeline as P

    edges = list(range(1, 65))
    n = sum(edges)
    store = zarr_hip.DeviceStore(device)
    arr = zarr_hip.Array.create(store, (n,), (edges,), "float32", -2.0, codecs=codecs)
    data = _data((n,), "float32")
    arr[...] = data
    meta = O.ArrayMeta((n,), (edges,), np.dtype("float32"), -2.0, codecs=codecs)
    host = _check(arr, store, meta, data, [])
    for sel in [(Ellipsis,), (slice(3, n - 5, 3),), (slice(100, 900),)]:
        groups = len({id(it[1]) for it in arr.batch_info(sel)[0]})
        assert groups == 64 or sel != (Ellipsis,)
        arr.get(sel)  # warm: plans and pooled buffers exist
        l0, s0 = P.LAUNCHES[0], P.SYNCS[0]
        got = arr.get(sel)
        assert P.SYNCS[0] - s0 == 1, (sel, P.SYNCS[0] - s0)
        assert P.LAUNCHES[0] - l0 == groups
        want = np.ascontiguousarray(O.read(host, meta, sel))
        assert got.cpu().numpy().tobytes() == want.tobytes()
    # writes: every group's merge reads and encodes first, one readback
    for sel, val in [((Ellipsis,), _data((n,), "float32", seed=5)), ((slice(7, 1500, 2),), np.float32(2.5))]:
        s0 = P.SYNCS[0]
        arr[sel] = val
        assert P.SYNCS[0] - s0 == 1, (sel, P.SYNCS[0] - s0)
        O.write(host, meta, sel, val)
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert got == host
    if CRC in codecs:
        bad = bytearray(host["c/40"])
        bad[17] ^= 0x04
        host["c/40"] = bytes(bad)
        store.set_sync("c/40", bytes(bad))
        with pytest.raises(ValueError) as want:
            O.read(host, meta)
        with pytest.raises(ValueError) as got:
            arr.get((Ellipsis,))
        assert str(got.value) == str(want.value)

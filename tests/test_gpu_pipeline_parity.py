"""The reference's cross-pipeline parity matrix (tests/test_pipeline_parity.py)
restated: there it checks FusedCodecPipeline against BatchedCodecPipeline;
here the GPU pipeline (HipCodecPipeline, HIP kernels through the C ABI) is
checked against the CPU oracle, which restates the reference's read/write
path.  For every (codec config x layout x write sequence x write_empty_chunks)
cell (test_pipeline_parity.py:82-233):

  1. both produce the same array contents,
  2. the same set of store keys,
  3. the same stored bytes (stronger than the reference, which skips byte
     equality only because gzip embeds timestamps -- no gzip here),
  4. each side reads the other side's store correctly.

Cells the device path does not take (gzip compressor, nested sharding,
bytes->bytes codecs around a sharding serializer) are refused loudly; that is
pinned in test_gpu_pipeline_suite.py and test_outer_codecs_around_sharding_refused.
Transposes around a sharding serializer are supported (the shard is sharded in
its permuted space) and checked both ways.
"""

from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

LE = {"name": "bytes", "configuration": {"endian": "little"}}
BE = {"name": "bytes", "configuration": {"endian": "big"}}
CRC = {"name": "crc32c"}

# test_pipeline_parity.py:82-101 (gzip omitted: host-side compression)
CODEC_CONFIGS = [
    ("bytes-only", "float64", [LE]),
    ("bytes-big-endian", "int32", [BE]),
    ("bytes-crc32c", "int32", [LE, CRC]),
]

# test_pipeline_parity.py:107-138 (nested sharding omitted)
LAYOUT_CONFIGS = [
    ("1d-unsharded", (100,), (10,), None),
    ("1d-1chunk-per-shard", (100,), (10,), (10,)),
    ("1d-multi-chunk-per-shard", (100,), (10,), (50,)),
    ("2d-unsharded", (20, 20), (5, 5), None),
    ("2d-sharded", (20, 20), (5, 5), (10, 10)),
]


def _full_overwrite(shape):
    return [((slice(None),) * len(shape), np.arange(int(np.prod(shape))).reshape(shape) + 1)]


def _partial_middle(shape):
    if len(shape) == 1:
        return [((slice(shape[0] // 4, 3 * shape[0] // 4),), 7)]
    return [((slice(shape[0] // 4, 3 * shape[0] // 4), slice(shape[1] // 4, 3 * shape[1] // 4)), 7)]


def _scalar_one_cell(shape):
    return [(tuple(s // 2 for s in shape), 99)]


def _overlapping(shape):
    if len(shape) == 1:
        n = shape[0]
        return [((slice(0, n // 2),), 1), ((slice(n // 4, 3 * n // 4),), 2), ((slice(n // 2, n),), 3)]
    a, b = shape
    return [((slice(0, a // 2), slice(0, b // 2)), 1),
            ((slice(a // 4, 3 * a // 4), slice(b // 4, 3 * b // 4)), 2)]


def _ends_in_fill(shape):
    full = (slice(None),) * len(shape)
    return [(full, 5), (full, 0)]


def _ends_in_partial_fill(shape):
    full = (slice(None),) * len(shape)
    half = (slice(0, shape[0] // 2),) + (slice(None),) * (len(shape) - 1)
    return [(full, 5), (half, 0)]


# test_pipeline_parity.py:143-202
SEQUENCES = [("full-overwrite", _full_overwrite), ("partial-middle", _partial_middle),
             ("scalar-one-cell", _scalar_one_cell), ("overlapping", _overlapping),
             ("ends-in-fill", _ends_in_fill), ("ends-in-partial-fill", _ends_in_partial_fill)]


def _matrix():
    for cid, dtype, codecs in CODEC_CONFIGS:
        for lid, shape, chunks, shards in LAYOUT_CONFIGS:
            for sid, fn in SEQUENCES:
                for wec in (False, True):
                    yield pytest.param(dtype, codecs, shape, chunks, shards, fn, wec,
                                       id=f"{lid}-{cid}-{sid}-wec{wec}")


def _oracle_meta(shape, chunks, shards, dtype, codecs, wec, order="morton", loc="end"):
    if shards is None:
        return O.ArrayMeta(shape, chunks, np.dtype(dtype), 0, codecs=list(codecs), write_empty_chunks=wec)
    return O.ArrayMeta(shape, shards, np.dtype(dtype), 0, codecs=[{
        "name": "sharding_indexed", "configuration": {
            "chunk_shape": list(chunks), "codecs": list(codecs), "index_codecs": [LE, CRC],
            "index_location": loc, "subchunk_write_order": order}}], write_empty_chunks=wec)


def _chunk_bytes(store) -> dict:
    return {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}


@pytest.mark.parametrize("dtype,codecs,shape,chunks,shards,seq,wec", list(_matrix()))
def test_pipeline_parity(device, dtype, codecs, shape, chunks, shards, seq, wec):
    """test_pipeline_parity.py:295-366, GPU pipeline vs the CPU oracle."""
    import zarr_hip
    from zarr_hip.spec import ArrayConfig

    ops = seq(shape)
    store = zarr_hip.DeviceStore(device)
    kw = dict(shards=shards) if shards is not None else {}
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, 0, codecs=list(codecs),
                                config=ArrayConfig(write_empty_chunks=wec), **kw)
    meta = _oracle_meta(shape, chunks, shards, dtype, codecs, wec)
    host: dict = {}
    for sel, val in ops:
        arr[sel] = val
        O.write(host, meta, sel, val)
    got = arr[...]
    want = O.read(host, meta, Ellipsis)
    np.testing.assert_array_equal(got, want)                       # 1. contents
    gpu_bytes = _chunk_bytes(store)
    assert sorted(gpu_bytes) == sorted(host)                        # 2. keys
    for k in host:                                                  # 3. bytes
        assert gpu_bytes[k] == host[k], k
    np.testing.assert_array_equal(O.read(gpu_bytes, meta, Ellipsis), want)      # 4. cross reads
    other = zarr_hip.DeviceStore.from_host(dict(host), device)
    oarr = zarr_hip.Array.create(other, shape, chunks, dtype, 0, codecs=list(codecs), **kw)
    np.testing.assert_array_equal(oarr[...], want)


@pytest.mark.parametrize("order", ["morton", "unordered", "lexicographic", "colexicographic"])
@pytest.mark.parametrize("loc", ["start", "end"])
def test_pipeline_parity_subchunk_write_order(device, order, loc):
    """test_pipeline_parity.py:374-445: a dense shard in every physical order,
    then a partial write into it; contents and stored bytes must match."""
    import zarr_hip
    from zarr_hip.codecs import BytesCodec, ShardingCodec
    from zarr_hip.spec import ArrayConfig

    shape, shard, inner = (12, 8), (6, 4), (2, 2)
    sc = ShardingCodec(chunk_shape=inner, codecs=(BytesCodec(),), index_location=loc,
                       subchunk_write_order=order)
    store = zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, shard, "int32", -1, codecs=[sc],
                                config=ArrayConfig(write_empty_chunks=True))
    ref = np.arange(96, dtype="int32").reshape(shape)
    arr[:] = ref
    arr[3:9, 1:6] = 777
    ref[3:9, 1:6] = 777
    np.testing.assert_array_equal(arr[...], ref)
    meta = O.ArrayMeta(shape, shard, np.dtype("int32"), -1, codecs=[{
        "name": "sharding_indexed", "configuration": {
            "chunk_shape": list(inner), "codecs": [LE], "index_location": loc,
            "subchunk_write_order": order}}], write_empty_chunks=True)
    host: dict = {}
    O.write(host, meta, slice(None), np.arange(96, dtype="int32").reshape(shape))
    O.write(host, meta, (slice(3, 9), slice(1, 6)), 777)
    assert _chunk_bytes(store) == host


def _outer_t(order, inner, inner_codecs=(LE,)):
    return [{"name": "transpose", "configuration": {"order": list(order)}},
            {"name": "sharding_indexed", "configuration": {
                "chunk_shape": list(inner), "codecs": list(inner_codecs)}}]


@pytest.mark.parametrize("direction", ["gpu-write-oracle-read", "oracle-write-gpu-read",
                                       "oracle-write-gpu-read-host-store"])
@pytest.mark.parametrize("shape,chunks,order,inner,inner_codecs,sels", [
    # test_pipeline_parity.py:463-523 ("outer-transpose-around-sharding")
    ((8, 8), (4, 4), (1, 0), (2, 2), (LE,), [np.s_[...], np.s_[1:3, 2:7]]),
    # non-square shards, 3-d, crc inside, int selections (the inner chunk also
    # divides the unpermuted shard: ShardingCodec.validate sees the array's
    # chunk shape, sharding.py:558-590)
    ((12, 8, 8), (6, 8, 4), (2, 0, 1), (2, 2, 4), (BE, CRC),
     [np.s_[...], np.s_[1:11:3, 5, :], np.s_[7, 2:8, 1:5], np.s_[4, 3, 2]]),
])
def test_pipeline_parity_outer_transpose_around_sharding(device, direction, shape, chunks, order, inner,
                                                         inner_codecs, sels):
    """Transposes in front of the sharding codec: the shard is sharded in its
    permuted (stored) space.  Whichever side writes (full write, then a region
    write through the partial-encode branch), the other reads back the same
    contents, full and partial; and both sides write the same bytes."""
    import zarr_hip

    codecs = _outer_t(order, inner, inner_codecs)
    data = (np.arange(int(np.prod(shape))).reshape(shape) + 1).astype("uint16")
    region = tuple(slice(1, min(4, s)) for s in shape)
    expected = data.copy()
    expected[region] = 99
    meta = O.ArrayMeta(shape, chunks, np.dtype("uint16"), 0, codecs=codecs)
    host: dict = {}
    O.write(host, meta, Ellipsis, data)
    O.write(host, meta, region, 99)
    if direction == "gpu-write-oracle-read":
        store = zarr_hip.DeviceStore(device)
        arr = zarr_hip.Array.create(store, shape, chunks, "uint16", 0, codecs=codecs)
        arr[...] = data
        arr[region] = 99
        got = _chunk_bytes(store)
        assert got == host
        for sel in sels:
            np.testing.assert_array_equal(O.read(got, meta, sel), expected[sel])
    else:
        store = zarr_hip.MemoryStore(dict(host)) if direction.endswith("host-store") else \
            zarr_hip.DeviceStore.from_host(dict(host), device)
        arr = zarr_hip.Array.create(store, shape, chunks, "uint16", 0, codecs=codecs)
        for sel in sels:
            np.testing.assert_array_equal(arr[sel], expected[sel])


@pytest.mark.parametrize("kind", ["memory", "device"])
def test_outer_gzip_around_sharding(device, kind):
    """test_pipeline_parity.py:455-523, "outer-gzip-around-sharding": a gzip
    codec after the sharding serializer compresses whole shards, so partial
    reads and writes must go through it (the reference's regression: they
    skipped it).  Here the outer host stage decompresses the whole shard
    before the GPU reads its index and inner chunks, and recompresses after
    the GPU re-packs it; full + region write, full + region read, stored bytes
    equal to the oracle's."""
    import zarr_hip

    codecs = [{"name": "sharding_indexed", "configuration": {"chunk_shape": [2, 2], "codecs": [LE]}},
              {"name": "gzip", "configuration": {"level": 1}}]
    shape = (8, 8)
    data = (np.arange(64).reshape(shape) + 1).astype("uint16")
    store = zarr_hip.MemoryStore() if kind == "memory" else zarr_hip.DeviceStore(device)
    a = zarr_hip.Array.create(store, shape, (4, 4), "uint16", 0, codecs=codecs)
    a[...] = data
    a[2:5, 1:3] = 99
    expected = data.copy()
    expected[2:5, 1:3] = 99
    np.testing.assert_array_equal(a[...], expected)
    np.testing.assert_array_equal(a[1:3, 2:7], expected[1:3, 2:7])
    meta = O.ArrayMeta(shape, (4, 4), np.dtype("uint16"), 0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), data)
    O.write(host, meta, (slice(2, 5), slice(1, 3)), np.full((3, 2), 99, "uint16"))
    got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert got == host

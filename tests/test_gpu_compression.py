"""GPU parity for chains with a host stage (compression stays on the host):
zarr v3's default numeric chain is ``bytes + zstd`` (src/zarr/core/array.py:
4884-4890), so a drop-in pipeline must open such arrays.  The GPU decodes and
encodes the fixed-size part (bytes / crc32c / transpose / sharding index and
extraction), the host runs the compressor -- the built-in gzip for JSON
metadata, or the caller's own codec INSTANCE (zarr's GzipCodec / ZstdCodec /
...) through its ``_decode_sync`` / ``_encode_sync``.

Checked against the oracle (oracle.gzip_* restates numcodecs.GZip over the
stdlib): decoded values bit for bit, and whole stores byte for byte -- same
keys, same compressed bytes (gzip with mtime 0 is deterministic).  The
reference scenarios restated: tests/test_codec_pipeline_suite.py:144-165
(1d-gzip, 1d-zstd: here with a caller-supplied codec the package has no
built-in for) and 294-307 (transpose-gzip)."""

import numpy as np
import pytest

import zarr_fakes as Z
from oracle import oracle as O
from test_gpu_decode import CRC, LE, SHARD, T, _data

pytestmark = pytest.mark.gpu


def GZ(level=1):
    return {"name": "gzip", "configuration": {"level": level}}


def _store(kind, tmp_path, device):
    import zarr_hip

    if kind == "memory":
        return zarr_hip.MemoryStore()
    if kind == "local":
        return zarr_hip.LocalStore(str(tmp_path / "store"))
    return zarr_hip.DeviceStore(device)


def _stored(store) -> dict:
    return {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}


STORES = ("memory", "local", "device")


@pytest.mark.parametrize("kind", STORES)
@pytest.mark.parametrize("codecs,shape,chunks,dtype", [
    ([LE, GZ(1)], (100,), (10,), "float64"),                # suite 1d-gzip
    ([LE, CRC, GZ(5)], (37, 50), (8, 16), "int32"),         # crc on the raw bytes, then compressed
    ([LE, GZ(9), CRC], (37, 50), (8, 16), "float32"),       # crc of the COMPRESSED bytes
    ([T((1, 0)), LE, GZ(1)], (8, 12), (2, 4), "int32"),     # suite transpose-gzip
], ids=["gzip", "crc-gzip", "gzip-crc", "transpose-gzip"])
def test_compressed_chain_roundtrip(kind, codecs, shape, chunks, dtype, tmp_path, device):
    import zarr_hip

    data = _data(shape, dtype)
    dt = data.dtype
    fill = 0.0 if dt.kind == "f" else -1
    store = _store(kind, tmp_path, device)
    arr = zarr_hip.Array.create(store, shape, chunks, dt, fill, codecs=codecs)
    arr[...] = data
    meta = O.ArrayMeta(shape, chunks, dt, fill, codecs=codecs)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    assert _stored(store) == host
    for sel in [(Ellipsis,), tuple(slice(1, s - 1, 2) for s in shape), tuple(s // 2 for s in shape)]:
        got = arr[sel]
        want = O.read(host, meta, sel)
        assert np.asarray(got).tobytes() == np.ascontiguousarray(want).tobytes()
    # a partial write (read-modify-write through the host stage), then all of it again
    sub = tuple(slice(1, max(2, s // 2)) for s in shape)
    val = np.full(tuple(x.stop - x.start for x in sub), 7, dtype=dt)
    arr[sub] = val
    O.write(host, meta, sub, val)
    assert _stored(store) == host
    assert arr[...].tobytes() == O.read(host, meta).tobytes()


@pytest.mark.parametrize("kind", STORES)
@pytest.mark.parametrize("inner", [[LE, GZ(1)], [LE, CRC, GZ(3)], [T((1, 0)), LE, GZ(1)]],
                         ids=["gzip", "crc-gzip", "transpose-gzip"])
def test_sharded_compressed_inner_chunks(kind, inner, tmp_path, device):
    """zarr's default sharded chain compresses every inner chunk: the index and
    the fixed-size inner decode stay on the GPU, touched inner chunks are
    decompressed on the host first; writes re-pack the shard with compressed
    inner chunks (same physical order, index re-encoded)."""
    import zarr_hip

    shape, shards, ichunks = (40, 36), (20, 36), (10, 12)
    data = _data(shape, "float32")
    data[0:10, 0:12] = 0.0  # an empty inner chunk: elided
    store = _store(kind, tmp_path, device)
    arr = zarr_hip.Array.create(store, shape, ichunks, "float32", 0.0, shards=shards, inner_codecs=inner)
    arr[...] = data
    meta = O.ArrayMeta(shape, shards, np.dtype("float32"), 0.0, codecs=[SHARD(ichunks, inner)])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    assert _stored(store) == host
    for sel in [(Ellipsis,), (slice(3, 33, 2), slice(5, 30)), (17, slice(None)), (slice(21, 22), 35)]:
        got = arr[sel]
        want = O.read(host, meta, sel)
        assert np.asarray(got).tobytes() == np.ascontiguousarray(want).tobytes(), sel
    # partial shard write: untouched inner chunks keep their stored state
    val = _data((6, 7), "float32", seed=3)
    arr[12:18, 20:27] = val
    O.write(host, meta, (slice(12, 18), slice(20, 27)), val)
    assert _stored(store) == host
    assert arr[...].tobytes() == O.read(host, meta).tobytes()


def test_compressed_crc_mismatch_message(device):
    """A corrupted crc32c after the compressor raises on the host with the
    reference's message; a corrupted compressed payload raises too."""
    import zarr_hip

    codecs = [LE, GZ(1), CRC]
    meta = O.ArrayMeta((32, 32), (16, 16), np.dtype("float32"), 0.0, codecs=codecs)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data((32, 32), "float32"))
    bad = bytearray(host["c/1/0"])
    bad[-2] ^= 0x01
    host["c/1/0"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), (32, 32), (16, 16), "float32", 0.0,
                                codecs=codecs)
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)


@pytest.mark.parametrize("where", ["offset", "crc"])
def test_sharded_compressed_corrupt_index_message(where, device):
    """A corrupted shard index in front of compressed inner chunks raises the
    reference's checksum message (the index CRC is checked before its
    offsets drive the host decompression, as _decode_shard_index_sync does,
    sharding.py:624-631), not the decompressor's error."""
    import zarr_hip

    inner = [LE, GZ(1)]
    shape, shards, ichunks = (40, 36), (20, 36), (10, 12)
    meta = O.ArrayMeta(shape, shards, np.dtype("float32"), 0.0, codecs=[SHARD(ichunks, inner)])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    bad = bytearray(host["c/1/0"])
    isz = 16 * 6 + 4  # 2 x 3 inner chunks per shard
    bad[len(bad) - isz + (3 if where == "offset" else isz - 3)] ^= 0x40  # an offset byte / the CRC
    host["c/1/0"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), shape, ichunks, "float32", 0.0,
                                shards=shards, inner_codecs=inner)
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)
    assert str(got.value).startswith("Stored and computed checksum do not match")


def _zarr_batch(meta_shape, chunk_shape, sel, store, dtype, fill, prototype=None):
    spec = Z.ArraySpec(tuple(chunk_shape), Z.ZDType(dtype), fill, Z.ArrayConfig(), prototype or Z.cpu_prototype)
    return Z.batch_for(meta_shape, chunk_shape, sel, store, spec)


@pytest.mark.parametrize("codec_cls", [Z.GzipCodec, Z.LzmaCodec], ids=["zarr-gzip", "numcodecs.lzma"])
def test_caller_codec_instances_run_the_host_stage(codec_cls, device):
    """zarr hands from_codecs its codec INSTANCES; the pipeline runs the
    compressor through the instance's own _decode_sync / _encode_sync (the
    suite's 1d-zstd scenario with a compressor the package has no built-in
    for), and the rest on the GPU."""
    import zarr_hip

    comp = codec_cls(level=1)
    codecs = (Z.FakeCodec(LE), comp)
    shape, chunks = (100,), (10,)
    pipe = zarr_hip.HipCodecPipeline.from_codecs(codecs)
    zstore = Z.MemoryStore()
    data = np.arange(1, 101, dtype="float64")
    batch, _ = _zarr_batch(shape, chunks, (slice(None),), zstore, "float64", 0.0)
    pipe.write_sync(batch, data)
    assert comp.calls["encode"] == 10
    # what is stored: the compressor over the oracle's fixed-size chunk bytes
    meta = O.ArrayMeta(shape, chunks, np.dtype("float64"), 0.0, codecs=[LE])
    plain: dict = {}
    O.write(plain, meta, (Ellipsis,), data)
    for k, v in plain.items():
        assert comp._decode_sync(Z.Buffer.from_bytes(zstore._store_dict[k]), Z.ArraySpec(
            chunks, Z.ZDType("float64"), 0.0, Z.ArrayConfig(), Z.cpu_prototype)).to_bytes() == v
    out = Z.NDBuffer(np.zeros(100))
    res = pipe.read_sync(batch, out)
    assert [r["status"] for r in res] == ["present"] * 10
    assert out.as_numpy_array().tobytes() == data.tobytes()
    assert comp.calls["decode"] >= 10
    # device-resident out
    import torch

    dout = torch.zeros(100, dtype=torch.float64, device=device)
    pipe.read_sync(batch, zarr_hip.NDBuffer(dout))
    assert dout.cpu().numpy().tobytes() == data.tobytes()


def test_zarr_sharding_instance_with_compressed_inner(device):
    """zarr's ShardingCodec instance with a compressor instance inside
    (create_array(shards=...)'s default chain): the inner instance runs the
    host stage, stores match the oracle's gzip layout."""
    import zarr_hip

    comp = Z.GzipCodec(level=1)
    sc = Z.ShardingCodec((5, 5), (Z.FakeCodec(LE), comp))
    pipe = zarr_hip.HipCodecPipeline.from_codecs((sc,))
    zstore = Z.MemoryStore()
    data = np.arange(400, dtype="int32").reshape(20, 20)
    batch, _ = _zarr_batch((20, 20), (10, 10), (slice(None), slice(None)), zstore, "int32", -1)
    pipe.write_sync(batch, data)
    meta = O.ArrayMeta((20, 20), (10, 10), np.dtype("int32"), -1, codecs=[SHARD((5, 5), [LE, GZ(1)])])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    assert {k: v for k, v in zstore._store_dict.items()} == host
    out = Z.NDBuffer(np.zeros((20, 20), "int32"))
    pipe.read_sync(batch, out)
    assert out.as_numpy_array().tobytes() == data.tobytes()
    assert comp.calls["decode"] >= 16


def test_json_zstd_without_instance_refused(device):
    """No built-in zstd here (no zstd module in the image): metadata naming it
    without the codec object zarr would pass is refused loudly."""
    import zarr_hip

    with pytest.raises(NotImplementedError, match="zstd"):
        zarr_hip.Array.create(zarr_hip.MemoryStore(), (20,), (10,), "int32", 0,
                              codecs=[LE, {"name": "zstd", "configuration": {"level": 1}}])

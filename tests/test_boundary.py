"""CPU checks of the CodecPipeline boundary with zarr-shaped inputs (duck-typed
stand-ins for zarr's Codec / ArraySpec / ZDType / Buffer / NDBuffer / stores,
tests/zarr_fakes.py), of the HBM arena's free list, and of the oracle's
partial shard encode.  No kernel runs here (tests/test_gpu_boundary.py drives
the same objects through the GPU)."""

import numpy as np
import pytest

from oracle import oracle as O
from tests import zarr_fakes as Z

LE = {"name": "bytes", "configuration": {"endian": "little"}}
BE = {"name": "bytes", "configuration": {"endian": "big"}}
CRC = {"name": "crc32c"}


def SHARD(inner, codecs, loc="end", order="morton"):
    return {"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(inner), "codecs": list(codecs), "index_location": loc,
        "subchunk_write_order": order}}


def test_from_codecs_accepts_zarr_codec_objects():
    from zarr_hip import HipCodecPipeline, ShardingCodec

    js = [{"name": "transpose", "configuration": {"order": [1, 0]}}, LE, CRC]
    a = HipCodecPipeline.from_codecs(Z.zcodecs(js))
    b = HipCodecPipeline.from_codecs(js)
    assert a.codecs == b.codecs
    sh = HipCodecPipeline.from_codecs(Z.zcodecs([SHARD((4, 4), [BE, CRC], "start", "colexicographic")]))
    c = sh.codecs[0]
    assert isinstance(c, ShardingCodec) and c.index_location == "start"
    assert c.subchunk_write_order == "colexicographic"  # write-time attribute carried over
    assert c.codecs[0].endian == "big"
    assert sh.supports_partial_decode and sh.supports_partial_encode


def test_unsupported_codec_is_loud():
    """A compressor named only by its JSON form with no built-in here (zstd:
    no module in this image) is refused; gzip has a built-in host stage; a
    codec INSTANCE with sync methods runs through them (HostCodec)."""
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import GzipCodec, HostCodec

    with pytest.raises(NotImplementedError, match="zstd"):
        HipCodecPipeline.from_codecs([LE, Z.FakeCodec({"name": "zstd", "configuration": {"level": 5}})])
    p = HipCodecPipeline.from_codecs([LE, Z.FakeCodec({"name": "gzip", "configuration": {"level": 5}})])
    assert isinstance(p.bytes_bytes_codecs[0], GzipCodec) and p.bytes_bytes_codecs[0].level == 5
    p = HipCodecPipeline.from_codecs([LE, Z.LzmaCodec()])
    assert isinstance(p.bytes_bytes_codecs[0], HostCodec) and p.bytes_bytes_codecs[0].name == "numcodecs.lzma"


def test_zarr_array_spec_and_zdtype_coerced():
    from zarr_hip import HipCodecPipeline
    from zarr_hip.spec import coerce_spec

    spec = Z.ArraySpec((8, 8), Z.ZDType("int16"), np.int16(-3),
                       Z.ArrayConfig(order="F", write_empty_chunks=True,
                                     sharding_coalesce_max_gap_bytes=7), Z.cpu_prototype)
    s = coerce_spec(spec)
    assert s.dtype == np.dtype("int16") and s.fill_value == -3
    assert s.config.order == "F" and s.config.write_empty_chunks
    assert s.config.sharding_coalesce_max_gap_bytes == 7
    assert s.prototype is Z.cpu_prototype
    p = HipCodecPipeline.from_codecs(Z.zcodecs([LE, CRC])).evolve_from_array_spec(spec)
    assert p.compute_encoded_size(128, spec) == 132


def test_bytes_endian_evolves_from_zdtype():
    from zarr_hip import HipCodecPipeline

    spec = Z.ArraySpec((8,), Z.ZDType("uint8"), 0, Z.ArrayConfig(), Z.cpu_prototype)
    p = HipCodecPipeline.from_codecs(Z.zcodecs([LE])).evolve_from_array_spec(spec)
    assert p.codecs[0].endian is None  # single-byte dtype (bytes.py:74-95)


def test_from_array_metadata_and_store():
    from zarr_hip import HipCodecPipeline

    md = Z.ArrayV3Metadata((64, 64), Z.ZDType("float32"), Z.RegularChunkGrid((32, 32)), np.float32(0),
                           Z.zcodecs([SHARD((16, 16), [LE, CRC])]))
    p = HipCodecPipeline.from_array_metadata_and_store(md, Z.MemoryStore())
    assert p.codecs[0].chunk_shape == (16, 16)
    p.validate(shape=md.shape, dtype=md.data_type, chunk_grid=md.chunk_grid)
    with pytest.raises(ValueError):  # 32 is not divisible by 12
        HipCodecPipeline.from_array_metadata_and_store(
            Z.ArrayV3Metadata((64, 64), Z.ZDType("float32"), Z.RegularChunkGrid((32, 32)), 0,
                              Z.zcodecs([SHARD((12, 16), [LE])])), None).validate(
            shape=(64, 64), chunk_grid=Z.RegularChunkGrid((32, 32)))

    class V2:
        shape = (4,)

    with pytest.raises(NotImplementedError):
        HipCodecPipeline.from_array_metadata_and_store(V2(), None)


def test_interop_conversions():
    from zarr_hip import interop

    b = Z.Buffer.from_bytes(b"\x01\x02\x03")
    assert interop.byte_payload(b).tobytes() == b"\x01\x02\x03"
    assert interop.device_tensor(b) is None
    nd = Z.NDBuffer(np.arange(6, dtype=np.int16).reshape(2, 3))
    assert interop.host_array(nd).shape == (2, 3)
    assert interop.native_dtype(Z.ZDType(">f8")) == np.dtype(">f8")
    assert interop.wrap_for_setter(b"ab", Z.cpu_prototype).to_bytes() == b"ab"
    assert interop.wrap_for_setter(b"ab", None) == b"ab"
    # zarr is not importable here: duck-typed stores get this package's requests
    R, S = interop.request_classes(Z.MemoryStore())
    assert R(1, 2).end == 2 and S(5).suffix == 5

    class Group(Exception):
        def __init__(self, excs):
            self.exceptions = excs

    assert interop.is_missing_key_error(Group([FileNotFoundError("k"), FileNotFoundError("k")]))
    assert not interop.is_missing_key_error(Group([FileNotFoundError("k"), ValueError()]))


def test_own_stores_take_zarr_buffers_and_keyword_requests():
    import zarr_hip
    from zarr_hip.store import _resolve_range

    st = zarr_hip.MemoryStore()
    st.set_sync("k", Z.Buffer.from_bytes(b"0123456789"))
    assert bytes(st.get_sync("k", prototype=None, byte_range=Z.RangeByteRequest(2, 5))) == b"234"
    assert _resolve_range(Z.SuffixByteRequest(3), 10) == (7, 10)


def test_arena_free_list_reuses_and_coalesces():
    from zarr_hip.store import ALIGN, DeviceArena

    a = DeviceArena("cpu", capacity=64 * ALIGN)
    offs = [a.reserve(ALIGN * 2) for _ in range(4)]
    assert offs == [0, 2 * ALIGN, 4 * ALIGN, 6 * ALIGN] and a.top == 8 * ALIGN
    a.free(offs[1], 2 * ALIGN)
    a.free(offs[2], 2 * ALIGN)  # coalesces with the block before it
    assert a._free == [[2 * ALIGN, 4 * ALIGN]]
    assert a.reserve(3 * ALIGN) == 2 * ALIGN  # first fit inside the freed hole
    a.free(offs[3], 2 * ALIGN)
    # [6,8) reaches the top and coalesces with the hole [5,6): the top comes down to 5
    assert a.top == 5 * ALIGN and a._free == []
    a.free(2 * ALIGN, 3 * ALIGN)
    # everything above offs[0] is free and the top came down
    assert a.top == 2 * ALIGN and a._free == []
    assert a.used_bytes == 2 * ALIGN


def test_device_store_overwrite_returns_space():
    import zarr_hip
    from zarr_hip.store import ALIGN

    st = zarr_hip.DeviceStore("cpu", capacity=1 << 16)
    for i in range(50):
        st.set_sync("c/0", bytes([i]) * 1000)
        st.set_sync("c/1", bytes([i]) * 3000)
    assert st.arena.used_bytes <= 5 * ALIGN + 12 * ALIGN
    assert st.to_dict()["c/1"] == bytes([49]) * 3000
    st.delete_sync("c/0")
    st.delete_sync("c/1")
    assert st.arena.used_bytes == 0 and st.arena.top == 0
    off = st.arena.reserve(10 * ALIGN)
    st.commit("x", off, 3 * ALIGN + 1, 10 * ALIGN)  # the unused tail goes back
    assert st.arena.used_bytes == 4 * ALIGN
    st.commit("y", st.arena.reserve(ALIGN), 0, ALIGN)  # elided: nothing kept
    assert "y" not in st and st.arena.used_bytes == 4 * ALIGN


# ------------------------------------------------ oracle: partial shard encode

def _meta(shape, shards, inner, wec=False, fill=0.0, dtype="float32"):
    return O.ArrayMeta(shape, shards, np.dtype(dtype), fill, codecs=[SHARD(inner, [LE, CRC])],
                       write_empty_chunks=wec)


def _present(blob, meta):
    sh = meta.chain.shard
    cps = tuple(s // c for s, c in zip(meta.chunk_shape, sh.chunk_shape))
    return {k for k, v in O.shard_reader(np.frombuffer(blob, np.uint8), sh, cps).items() if v is not None}


def test_oracle_partial_write_keeps_untouched_inner_chunks_absent():
    """wec=True, a first write covering the top-left corner of a shard stores only
    the inner chunks it touches (sharding.py:774-885), not the whole shard."""
    meta = _meta((16, 16), (16, 16), (4, 4), wec=True)
    store = {}
    O.write(store, meta, (slice(0, 6), slice(0, 3)), np.ones((6, 3), np.float32))
    assert _present(store["c/0/0"], meta) == {(0, 0), (1, 0)}
    # a later write elsewhere keeps the earlier inner chunks and adds its own
    O.write(store, meta, (slice(12, 16), slice(12, 16)), np.zeros((4, 4), np.float32))
    assert _present(store["c/0/0"], meta) == {(0, 0), (1, 0), (3, 3)}
    got = O.read(store, meta)
    want = np.zeros((16, 16), np.float32)
    want[:6, :3] = 1
    assert got.tobytes() == want.tobytes()


def test_oracle_edge_shard_never_stores_out_of_array_inner_chunks():
    meta = _meta((20, 16), (16, 16), (4, 4), wec=True)
    store = {}
    O.write(store, meta, (Ellipsis,), np.arange(320, dtype=np.float32).reshape(20, 16))
    # the edge shard c/1/0 holds rows 16..19 = inner row 0 only
    assert _present(store["c/1/0"], meta) == {(0, j) for j in range(4)}
    assert len(_present(store["c/0/0"], meta)) == 16


def test_oracle_complete_shard_write_resets_untouched_state():
    """A write that covers a whole shard re-encodes every inner chunk (the
    existing shard is not read); fill-valued ones are elided without wec."""
    meta = _meta((8, 8), (8, 8), (4, 4), wec=False)
    store = {}
    O.write(store, meta, (Ellipsis,), np.ones((8, 8), np.float32))
    assert len(_present(store["c/0/0"], meta)) == 4
    v = np.ones((8, 8), np.float32)
    v[:4, :4] = 0.0
    O.write(store, meta, (Ellipsis,), v)
    assert _present(store["c/0/0"], meta) == {(0, 1), (1, 0), (1, 1)}

"""CPU checks of the host stage (hoststage.py): the library's host CRC-32C,
the host-side crc32c / gzip steps against the oracle's restatements, and the
shard transcoder (fixed-size inner chunks <-> compressed inner chunks) against
the oracle's shard assembly.  No kernel runs here."""

import numpy as np
import pytest

import zarr_fakes as Z
from oracle import oracle as O

LE = {"name": "bytes", "configuration": {"endian": "little"}}
CRC = {"name": "crc32c"}


def GZ(level=1):
    return {"name": "gzip", "configuration": {"level": level}}


def test_host_crc_matches_oracle_and_kat():
    from zarr_hip import hoststage

    assert hoststage.host_crc32c(b"123456789") == 0xE3069283  # RFC 3720 check value
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 8, 9, 63, 4096, 100003):
        a = rng.integers(0, 256, n, dtype=np.uint8)
        for off in (0, 1, 3):
            if off <= n:
                assert hoststage.host_crc32c(a[off:]) == O.crc32c(a[off:]), (n, off)


@pytest.mark.parametrize("chain", [[CRC], [GZ(1)], [GZ(6), CRC], [CRC, GZ(9)]])
def test_tail_matches_oracle(chain):
    from zarr_hip import hoststage
    from zarr_hip.codecs import parse_codecs

    tail = tuple(parse_codecs(chain))
    data = np.random.default_rng(1).standard_normal(1000).astype("f4").view(np.uint8)
    och = O.Chain(bb=tuple("crc32c" if c["name"] == "crc32c" else ("gzip", c["configuration"]["level"])
                           for c in chain))
    want = bytes(O.chain_encode(data.view("f4"), och, O.Spec((1000,), np.dtype("f4"), 0.0)))
    got = hoststage.encode_tail(data, tail, None)
    assert got == want
    assert hoststage.decode_tail(got, tail, None) == data.tobytes()


def test_tail_crc_error_message_is_the_reference_one():
    from zarr_hip import hoststage
    from zarr_hip.codecs import parse_codecs

    tail = tuple(parse_codecs([GZ(1), CRC]))
    enc = bytearray(hoststage.encode_tail(b"x" * 500, tail, None))
    enc[-1] ^= 0x80
    with pytest.raises(ValueError) as got:
        hoststage.decode_tail(bytes(enc), tail, None)
    with pytest.raises(ValueError) as want:
        O.crc32c_decode(np.frombuffer(bytes(enc), np.uint8))
    assert str(got.value) == str(want.value)


@pytest.mark.parametrize("loc", ["end", "start"])
@pytest.mark.parametrize("inner", [[LE, GZ(1)], [LE, CRC, GZ(4)]])
def test_shard_transcoder_matches_oracle_assembly(loc, inner):
    """The fixed-size shard (what the GPU packer writes) re-packed with the
    inner host stage equals the oracle's shard of the full inner chain, and
    back; Morton order and elided inner chunks survive."""
    from zarr_hip import hoststage
    from zarr_hip.codecs import parse_codecs, split_host_tail
    from zarr_hip.spec import ArraySpec

    shard_shape, ichunks = (8, 12), (4, 4)
    data = np.random.default_rng(2).standard_normal(shard_shape).astype("f4")
    data[4:8, 0:4] = 0.0  # elided
    fixed_inner = [c for c in inner if c["name"] != "gzip"]

    def blob(codecs):
        meta = O.ArrayMeta(shard_shape, shard_shape, np.dtype("f4"), 0.0, codecs=[{
            "name": "sharding_indexed", "configuration": {"chunk_shape": list(ichunks), "codecs": codecs,
                                                          "index_location": loc}}])
        st = {}
        O.write(st, meta, (Ellipsis,), data)
        return st["c/0/0"]

    sh = parse_codecs([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(ichunks), "codecs": inner, "index_location": loc}}])[0]
    from dataclasses import replace

    fixed, tail = split_host_tail(sh.codecs)
    tr = hoststage.ShardTranscoder(replace(sh, codecs=fixed), shard_shape, tail,
                                   ArraySpec(ichunks, "f4", 0.0))
    assert tr.to_stored(blob(fixed_inner)) == blob(inner)
    assert tr.to_fixed(blob(inner)) == blob(fixed_inner)
    bad = bytearray(blob(inner))
    bad[-1 if loc == "end" else 16 * 6 + 1] ^= 1  # the index's crc / one index byte
    with pytest.raises(ValueError, match="checksum"):
        tr.to_fixed(bytes(bad))


def test_host_codec_instance_gets_a_buffer_and_its_spec():
    """HostCodec hands a caller codec a Buffer of the spec's prototype (zarr's
    own when the spec came from zarr) and the caller's spec object."""
    from zarr_hip.codecs import HostCodec
    from zarr_hip.spec import coerce_spec

    c = Z.GzipCodec(level=3)
    zspec = Z.ArraySpec((10,), Z.ZDType("f8"), 0.0, Z.ArrayConfig(), Z.cpu_prototype)
    hc = HostCodec(c)
    spec = coerce_spec(zspec)
    assert spec.source is zspec
    enc = hc.encode_bytes(b"abc" * 100, spec)
    assert hc.decode_bytes(enc, spec) == b"abc" * 100
    assert c.calls == {"decode": 1, "encode": 1}
    assert hc.decode_bytes(enc, None) == b"abc" * 100  # no spec: the package's host prototype
    assert hc.to_dict() == {"name": "gzip", "configuration": {"level": 3}}

"""Pin the CPU oracle (oracle/) against published vectors and the reference's own
test invariants before anything else trusts it.  CPU only."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# --- CRC-32C known-answer vectors (RFC 3720 B.4 + the "check" value) ---------

@pytest.mark.parametrize("impl", ["hw", "slice8", "bitwise"])
def test_crc32c_kats(impl):
    for kat in _load("crc32c_kat.json")["vectors"]:
        data = bytes.fromhex(kat["hex"])
        assert O.crc32c(data, impl) == int(kat["crc"], 16), kat["name"]


def test_crc32c_impls_agree_random():
    rng = np.random.default_rng(0)
    for n in [0, 1, 3, 7, 8, 15, 16, 17, 63, 64, 255, 1000, 4097]:
        buf = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        vals = {O.crc32c(buf, i) for i in ("hw", "slice8", "bitwise")}
        assert len(vals) == 1
        if n <= 64:
            assert vals == {O.crc32c_pure_python(buf)}


# --- Morton order: literal vectors from tests/test_codecs/test_codecs.py:175-206 --

def test_morton_exact_order():
    for case in _load("morton_exact.json")["cases"]:
        shape = tuple(case["shape"])
        assert [list(c) for c in O.morton_order_coords(shape)] == case["order"]


@pytest.mark.parametrize("shape", [(2, 2, 2), (5, 2), (2, 5), (2, 9, 2), (3, 2, 12), (2, 5, 1),
                                   (4, 3, 6, 2, 7), (1,), (1, 1), (5, 1, 3), (5, 5, 5)])
def test_morton_is_permutation(shape):
    """test_codecs.py:208-245: every coordinate exactly once."""
    import itertools
    order = O.morton_order_coords(shape)
    assert len(order) == int(np.prod(shape)) == len(set(order))
    assert set(order) == set(itertools.product(*(range(s) for s in shape)))


@pytest.mark.parametrize("shape", [(2, 2), (4, 4), (2, 2, 2), (4, 4, 4), (2, 2, 2, 2)])
def test_morton_ordering(shape):
    """test_codecs.py:248-266."""
    for i, c in enumerate(O.morton_order_coords(shape)):
        assert c == O.decode_morton(i, shape)


# --- codec invariants from the reference tests --------------------------------

@pytest.mark.parametrize("endian", ["little", "big"])
@pytest.mark.parametrize("dtype", ["float64", ">u2", "<i4", "float32", "int16", "uint8"])
def test_bytes_codec_stored_bytes(endian, dtype):
    """tests/test_codecs/test_bytes.py:90,136: stored == astype(newbyteorder).tobytes()."""
    arr = np.arange(100, dtype=dtype)
    enc = O.bytes_encode(arr, endian)
    want = arr.astype(np.dtype(dtype).newbyteorder("<" if endian == "little" else ">"))
    assert enc.tobytes() == want.tobytes()
    dec = O.bytes_decode(enc, arr.shape, np.dtype(dtype).newbyteorder("="), endian)
    np.testing.assert_array_equal(dec, arr)


def test_crc_encoded_size():
    """tests/test_chunk_transform.py:118-135: 800 -> 804."""
    chain = O.Chain.from_json([{"name": "bytes", "configuration": {"endian": "little"}},
                               {"name": "crc32c"}])
    assert O.chain_encoded_size(800, chain) == 804
    enc = O.crc32c_encode(np.zeros(800, np.uint8))
    assert len(enc) == 804
    assert O.crc32c_decode(enc).size == 800


def test_crc_mismatch_message():
    enc = O.crc32c_encode(np.arange(16, dtype=np.uint8))
    enc[3] ^= 1
    with pytest.raises(ValueError, match="Stored and computed checksum do not match"):
        O.crc32c_decode(enc)


@pytest.mark.parametrize("order", [(2, 1, 0), (1, 2, 0), (0, 2, 1)])
def test_transpose_roundtrip(order):
    """test_transpose.py:51-113 including non-self-inverse orders."""
    a = np.arange(2 * 3 * 4, dtype="f4").reshape(2, 3, 4)
    e = O.transpose_encode(a, order)
    assert e.shape == O.transpose_resolve_shape(a.shape, order)
    np.testing.assert_array_equal(O.transpose_decode(e, order), a)


def test_shard_index_semantics():
    """test_sharding_unit.py:45-170: MAX_UINT_64 sentinel, (offset, length) pairs."""
    sh = O.ShardSpec((4, 4), O.Chain.from_json([{"name": "bytes"}]),
                     O.Chain.from_json([{"name": "bytes", "configuration": {"endian": "little"}},
                                        {"name": "crc32c"}]))
    enc = {(0, 1): np.arange(100, dtype=np.uint8), (1, 0): np.arange(50, dtype=np.uint8)}
    blob = O.assemble_shard(enc, sh, (2, 2))
    r = O.shard_reader(blob, sh, (2, 2))
    assert r[(0, 0)] is None and r[(1, 1)] is None
    np.testing.assert_array_equal(r[(0, 1)], enc[(0, 1)])
    np.testing.assert_array_equal(r[(1, 0)], enc[(1, 0)])
    assert len(blob) == 150 + O.shard_index_size(4, sh.index) == 150 + 68


@pytest.mark.parametrize("order", ["morton", "lexicographic", "colexicographic"])
def test_subchunk_physical_order(order):
    """test_sharding.py:957-975: physical order of subchunks == _subchunk_order_iter."""
    cps = (3, 2)
    sh = O.ShardSpec((4, 4), O.Chain.from_json([{"name": "bytes"}]),
                     O.Chain.from_json([{"name": "bytes", "configuration": {"endian": "little"}},
                                        {"name": "crc32c"}]), subchunk_write_order=order)
    enc = {c: np.full(10, i, np.uint8) for i, c in enumerate(O.lexicographic_order_coords(cps))}
    blob = O.assemble_shard(enc, sh, cps)
    idx = O.decode_shard_index(blob[-(16 * 6 + 4):], cps, sh.index)
    by_off = sorted((int(idx[c][0]), c) for c in O.lexicographic_order_coords(cps))
    assert [c for _, c in by_off] == O.subchunk_order(cps, order)


def test_missing_inner_fills_and_roundtrip():
    meta = O.ArrayMeta((16, 16), (8, 8), np.dtype("int16"), -1, codecs=[{
        "name": "sharding_indexed", "configuration": {
            "chunk_shape": [4, 4],
            "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                       {"name": "crc32c"}],
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                             {"name": "crc32c"}]}}])
    store = {}
    data = np.arange(256, dtype="int16").reshape(16, 16)
    data[0:4, 0:4] = -1  # an inner chunk equal to fill -> elided
    O.write(store, meta, (Ellipsis,), data)
    np.testing.assert_array_equal(O.read(store, meta), data)
    np.testing.assert_array_equal(O.read(store, meta, (slice(1, 15, 3), 5)), data[1:15:3, 5])


def test_fill_equality_rules():
    """buffer/core.py:534-558: fill 0.0 compares bit patterns; NaN fill is NaN-equal."""
    assert not O.all_equal(np.array([-0.0], "f4"), np.float32(0.0))
    assert O.all_equal(np.array([0.0], "f4"), np.float32(0.0))
    nan2 = np.array([0x7FC00001], np.uint32).view("f4")
    assert O.all_equal(nan2, np.float32("nan"))

"""GPU parity for host-sourced batches (MemoryStore / LocalStore bytes staged
through pinned memory into HBM): plain chunks across several staging windows,
and partial shard reads that fetch the index by range request and only the
touched inner chunks (coalesced), as sharding.py:1695-1752 does."""

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import BE, CRC, LE, SHARD, T, _data, _roundtrip

pytestmark = pytest.mark.gpu


class CountingStore:
    """MemoryStore wrapper recording every byte request (IO-shape checks)."""

    def __init__(self, inner):
        self.inner = inner
        self.calls = []

    def get_sync(self, key, byte_range=None):
        v = self.inner.get_sync(key, byte_range)
        self.calls.append((key, byte_range, 0 if v is None else len(v)))
        return v

    def get_ranges_sync(self, key, ranges, **kw):
        from zarr_hip.store import _RangesMixin

        return _RangesMixin.get_ranges_sync(self, key, ranges, **kw)

    def set_sync(self, key, value):
        self.inner.set_sync(key, value)

    def delete_sync(self, key):
        self.inner.delete_sync(key)


def test_host_store_multi_window(device):
    # 32 MiB of chunks -> 4 staging windows, copied by the thread pool
    _roundtrip(device, (256, 256, 128), (64, 64, 64), "float32", [LE, CRC], host_store=True)


@pytest.mark.parametrize("loc", ["end", "start"])
@pytest.mark.parametrize("inner", [[LE, CRC], [BE], [T((2, 0, 1)), LE, CRC]])
@pytest.mark.parametrize("sel", [(Ellipsis,), (slice(3, 29), slice(None, None, 3), 7),
                                 (slice(9, 10), slice(17, 40), slice(0, 40, 9))])
def test_host_sharded_partial(device, loc, inner, sel):
    _roundtrip(device, (48, 40, 40), (24, 20, 20), "float32",
               [SHARD((8, 10, 10), inner, loc)], selection=sel, host_store=True)


def test_host_sharded_missing_inner_and_shard(device):
    import zarr_hip

    codecs = [SHARD((4, 4), [LE, CRC])]
    meta = O.ArrayMeta((16, 24), (8, 8), np.dtype("int16"), -1, codecs=codecs)
    data = _data((16, 24), "int16")
    data[0:4, 4:8] = -1
    data[8:16, 16:24] = -1
    host = {}
    O.write(host, meta, (Ellipsis,), data)
    assert "c/1/2" not in host
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), (16, 24), (8, 8), "int16", -1,
                                codecs=codecs)
    for sel in [(Ellipsis,), (slice(3, 13), slice(2, 23, 3)), (7, slice(None)), (slice(9, 10), 20)]:
        assert arr[sel].tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()


def test_host_sharded_fetches_only_touched_inner_chunks(device):
    import zarr_hip
    from zarr_hip.spec import ArrayConfig

    codecs = [SHARD((16, 16, 16), [LE, CRC])]
    meta = O.ArrayMeta((64, 64, 64), (64, 64, 64), np.dtype("float32"), 0.0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), _data((64, 64, 64), "float32"))
    blob = len(host["c/0/0/0"])
    idx = 64 * 16 + 4
    inner = 16 ** 3 * 4 + 4
    sel = (slice(0, 16), slice(16, 32), slice(40, 50))  # two inner chunks
    want = np.ascontiguousarray(O.read(host, meta, sel)).tobytes()
    # default coalescing (gap <= 1 MiB): index read + ONE merged range read
    st = CountingStore(zarr_hip.MemoryStore(dict(host)))
    arr = zarr_hip.Array.create(st, (64, 64, 64), (16, 16, 16), "float32", 0.0, shards=(64, 64, 64),
                                inner_codecs=[LE, CRC])
    st.calls.clear()
    assert arr[sel].tobytes() == want
    assert len(st.calls) == 2 and st.calls[0][2] == idx
    assert 2 * inner <= st.calls[1][2] < blob // 4
    # coalescing off (the reference's NO_MERGE knob): exactly the two chunks
    arr = zarr_hip.Array.create(st, (64, 64, 64), (16, 16, 16), "float32", 0.0, shards=(64, 64, 64),
                                inner_codecs=[LE, CRC],
                                config=ArrayConfig(sharding_coalesce_max_gap_bytes=-1))
    st.calls.clear()
    assert arr[sel].tobytes() == want
    assert sorted(n for _, _, n in st.calls) == [idx, inner, inner]


def test_host_sharded_index_crc_mismatch(device):
    import zarr_hip

    codecs = [SHARD((4, 4), [LE])]
    meta = O.ArrayMeta((8, 8), (8, 8), np.dtype("float32"), 0.0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), _data((8, 8), "float32"))
    bad = bytearray(host["c/0/0"])
    bad[-6] ^= 1  # inside the index CRC trailer region of entries
    host["c/0/0"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), (8, 8), (8, 8), "float32", 0.0,
                                codecs=codecs)
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)


def test_local_store_sharded(device, tmp_path):
    import zarr_hip

    codecs = [SHARD((8, 8, 8), [LE, CRC])]
    meta = O.ArrayMeta((32, 32, 32), (16, 16, 16), np.dtype("float32"), 0.0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), _data((32, 32, 32), "float32"))
    st = zarr_hip.LocalStore(str(tmp_path))
    arr = zarr_hip.Array.create(st, (32, 32, 32), (8, 8, 8), "float32", 0.0, shards=(16, 16, 16),
                                inner_codecs=[LE, CRC])
    for k, v in host.items():
        st.set_sync(k, v)
    for sel in [(Ellipsis,), (slice(5, 27), 3, slice(None, None, 2))]:
        assert arr[sel].tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()

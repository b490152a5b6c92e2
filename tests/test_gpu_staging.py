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


# ---------------------------------------------------------------- pinned store
def test_pinned_store_multi_window(device):
    # values DMA'd straight from the page-locked arena (merged runs)
    _roundtrip(device, (256, 256, 128), (64, 64, 64), "float32", [LE, CRC], host_store="pinned")


@pytest.mark.parametrize("inner", [[LE, CRC], [T((2, 0, 1)), LE, CRC]])
@pytest.mark.parametrize("sel", [(Ellipsis,), (slice(3, 29), slice(None, None, 3), 7)])
def test_pinned_store_sharded_partial(device, inner, sel):
    _roundtrip(device, (48, 40, 40), (24, 20, 20), "float32",
               [SHARD((8, 10, 10), inner, "end")], selection=sel, host_store="pinned")


def test_pinned_store_rewrites_stay_bounded(device):
    """Overwrites free and reuse the arena (after the staging streams drain);
    every read after a rewrite sees the new bytes."""
    import zarr_hip

    codecs = [SHARD((8, 8), [LE, CRC])]
    meta = O.ArrayMeta((32, 48), (16, 16), np.dtype("float32"), 0.0, codecs=codecs)
    st = zarr_hip.PinnedMemoryStore(capacity=1 << 12)
    arr = zarr_hip.Array.create(st, (32, 48), (8, 8), "float32", 0.0, shards=(16, 16), inner_codecs=[LE, CRC])
    host = {}
    caps = []
    for i in range(10):
        data = _data((32, 48), "float32", seed=i)
        sel = (Ellipsis,) if i % 3 == 0 else (slice(i, 20 + i), slice(3 * i, 3 * i + 17))
        O.write(host, meta, sel, data if sel == (Ellipsis,) else data[sel])
        arr[sel] = data if sel == (Ellipsis,) else data[sel]
        assert arr[...].tobytes() == O.read(host, meta).tobytes()
        stored = st.to_dict()
        assert {k: stored[k] for k in host} == host  # byte-identical shards (metadata aside)
        caps.append(st.arena.capacity)
    assert caps[-1] == caps[3]  # capacity stops growing once the working set fits
    assert st.arena.used_bytes == sum(-(-len(v) // 256) * 256 for v in st.to_dict().values())


def test_stage_mixed_pinned_and_pageable_pieces(device):
    """zhip_stage_h2d with pinned pieces (direct DMA, merged when contiguous)
    interleaved with pageable ones (packed windows): every piece lands at its
    offset; bytes no piece covers are left alone."""
    import torch

    from zarr_hip import _native as N

    rng = np.random.default_rng(5)
    pin = torch.empty(1 << 22, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:] = rng.integers(0, 256, pin.numel(), dtype=np.uint8)
    pageable = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(1, 300000, 24)]
    rows, off, poff, want = [], 0, 0, {}
    for i in range(48):
        if i % 2 == 0 or i % 7 == 0:  # pinned: consecutive ones are contiguous in host and dst order
            n = int(rng.integers(1, 200000))
            poff = (poff + 255) // 256 * 256
            rows.append((pin.data_ptr() + poff, n, off, N.PIECE_PINNED, 0))
            want[off] = pin.numpy()[poff: poff + n].copy()
            poff += n
        else:
            v = pageable[i % len(pageable)]
            rows.append((v.ctypes.data, v.size, off, 0, 0))
            want[off] = v.copy()
            n = v.size
        off = (off + n + 255) // 256 * 256
        if i == 20:
            off += 4096  # a gap no piece covers
    pieces = np.array(rows, N.PIECE_DT)
    host = torch.empty(off + 64, dtype=torch.uint8, pin_memory=True)
    dev = torch.full((off + 64,), 0xA5, dtype=torch.uint8, device=device)
    st = torch.cuda.current_stream(device)
    for window in (4096, 1 << 16, 1 << 20):
        dev.fill_(0xA5)
        rc = N.lib().zhip_stage_h2d(pieces.ctypes.data, len(pieces), host.data_ptr(), dev.data_ptr(), off,
                                    window, 4, st.cuda_stream)
        assert rc == 0
        got = dev.cpu().numpy()
        for o, w in want.items():
            assert got[o: o + w.size].tobytes() == w.tobytes(), (window, o)
        gap_lo = sorted(want)[21] - 4096
        assert (got[gap_lo: gap_lo + 4096] == 0xA5).all()


# ------------------------------------------------- slab-pipelined host reads
@pytest.mark.parametrize("kind", ["memory", "pinned"])
@pytest.mark.parametrize("sel", [(Ellipsis,), (slice(5, 250), slice(None), slice(3, 128)),
                                 (7, slice(None), slice(None))])
def test_slab_pipelined_host_read(device, kind, sel):
    """Outs of >= 16 MiB split into row slabs (H2D / decode / D2H overlap);
    the result equals the oracle's whole read."""
    from zarr_hip.pipeline import _slab_groups

    arr, host, meta = _roundtrip(device, (256, 256, 128), (64, 64, 64), "float32", [LE, CRC],
                                 host_store=kind, selection=sel)
    batch, _ = arr.batch_info(sel)
    import torch

    shape = O.read(host, meta, sel).shape
    twin = torch.empty(shape, dtype=torch.float32, device=device)
    g = _slab_groups(batch, twin)
    if sel[0] == 7:
        assert g is None or len(g) >= 2  # 2-D out (dim 0 dropped): slabs over the next dim
    else:
        assert g is not None and len(g) >= 2
        covered = sorted(i for _, _, idx in g for i in idx)
        assert covered == list(range(len(batch)))


def test_slab_read_into_pageable_strided_out(device):
    """read_sync into a caller's pageable, non-contiguous numpy out that the
    batch only partly covers: slabs go through the pinned bounce, regions no
    chunk writes keep their values."""
    import zarr_hip

    meta = O.ArrayMeta((256, 128, 128), (32, 64, 64), np.dtype("float32"), 0.0, codecs=[LE, CRC])
    host = {}
    O.write(host, meta, (Ellipsis,), _data((256, 128, 128), "float32"))
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), (256, 128, 128), (32, 64, 64), "float32", 0.0,
                                codecs=[LE, CRC])
    sel = (slice(0, 256), slice(0, 128), slice(0, 64))  # half of the last dim's chunks
    batch, out_shape = arr.batch_info(sel)
    big = np.full((256, 128, 128), -7.0, np.float32)
    out = big[:, :, :64]  # strided view
    res = arr.codec_pipeline.read_sync(batch, out)
    assert all(r["status"] == "present" for r in res)
    assert out.tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()
    assert (big[:, :, 64:] == -7.0).all()


def test_slab_read_crc_error_in_later_slab(device):
    import zarr_hip

    meta = O.ArrayMeta((256, 128, 128), (32, 128, 128), np.dtype("float32"), 0.0, codecs=[LE, CRC])
    host = {}
    O.write(host, meta, (Ellipsis,), _data((256, 128, 128), "float32"))
    bad = bytearray(host["c/6/0/0"])
    bad[100] ^= 0x10
    host["c/6/0/0"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.PinnedMemoryStore(dict(host)), (256, 128, 128), (32, 128, 128),
                                "float32", 0.0, codecs=[LE, CRC])
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)


def test_slab_read_sharded_host(device):
    _roundtrip(device, (256, 128, 128), (64, 128, 128), "float32",
               [SHARD((32, 64, 64), [LE, CRC], "end")], host_store="pinned")


# --------------------------------------------- local files: pread by the pool
def test_local_store_file_pieces(device, tmp_path):
    """LocalStore chunks reach HBM as ZHIP_PIECE_FILE pieces (the staging
    pool preads them into the pinned windows): multi-window unsharded reads,
    missing chunks, and a file piece that cannot be read in full."""
    import zarr_hip
    from zarr_hip import staging
    from zarr_hip.store import FileRef

    meta = O.ArrayMeta((256, 128, 128), (64, 64, 64), np.dtype("float32"), 1.5, codecs=[LE, CRC])
    host = {}
    data = _data((256, 128, 128), "float32")
    O.write(host, meta, (Ellipsis,), data)
    host.pop("c/1/0/1")
    st = zarr_hip.LocalStore(str(tmp_path))
    arr = zarr_hip.Array.create(st, (256, 128, 128), (64, 64, 64), "float32", 1.5, codecs=[LE, CRC])
    for k, v in host.items():
        st.set_sync(k, v)
    assert isinstance(st.locate_sync("c/0/0/0"), FileRef) and st.locate_sync("c/1/0/1") is None
    for sel in [(Ellipsis,), (slice(3, 200), 5, slice(None, None, 3))]:
        assert arr[sel].tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()
    # a piece that claims more bytes than its file holds fails loudly
    lay = staging.StagingLayout()
    lay.add(FileRef(st._path("c/0/0/0"), 0, len(host["c/0/0/0"]) + 4096))
    with pytest.raises(Exception):
        _, _, pend = staging.stage(lay, device, defer=True)
        pend.finish()

"""GPU tests of object lifetimes and cached state around the hot path:

* staging jobs end on every error path (a failed slab, a planning error), so
  no library thread keeps writing into buffers Python has dropped;
* a host out read through row slabs keeps the values of rows no item selects;
* the per-call plan cache of HipCodecPipeline.read_sync (repeated reads skip
  planning) sees every write, overwrite and delete between two reads;
* prepared programs and ReadGraphs refuse to launch after the store's
  placements changed (freed regions are reused at once).

Every decoded result is compared with the CPU oracle (test infrastructure)."""

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import CRC, LE, SHARD, _data

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------ staging lifetimes
def _local_array(tmp_path, shape, chunks, fill=0.0):
    import zarr_hip

    meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), fill, codecs=[LE, CRC])
    host = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    st = zarr_hip.LocalStore(str(tmp_path))
    arr = zarr_hip.Array.create(st, shape, chunks, "float32", fill, codecs=[LE, CRC])
    for k, v in host.items():
        st.set_sync(k, v)
    return arr, st, host, meta


def test_slab_read_io_error_ends_every_job(device, tmp_path, monkeypatch):
    """A file piece that cannot be read in full fails its slab with an IO
    error; every later slab's staging job (all begun up front) is ended
    before the exception leaves read_sync, and the next read is exact."""
    from zarr_hip import _native as N
    from zarr_hip.store import FileRef, LocalStore

    arr, st, host, meta = _local_array(tmp_path, (256, 128, 128), (32, 128, 128))
    real = LocalStore.locate_sync

    def short(self, key, byte_range=None):
        r = real(self, key, byte_range)
        if r is not None and key == "c/3/0/0":  # a middle slab: claims more than the file holds
            return FileRef(r.path, r.offset, r.length + 8192)
        return r

    monkeypatch.setattr(LocalStore, "locate_sync", short)
    for _ in range(3):
        with pytest.raises((N.NativeError, ValueError)):
            arr[...]
    monkeypatch.setattr(LocalStore, "locate_sync", real)
    for _ in range(2):
        assert arr[...].tobytes() == O.read(host, meta).tobytes()


def test_planning_error_ends_the_job(device, tmp_path, monkeypatch):
    """An out of the wrong item size is refused before anything is staged;
    a batch whose staging began and whose planning then fails aborts the job."""
    import torch

    import zarr_hip
    from zarr_hip import pipeline as P

    arr, st, host, meta = _local_array(tmp_path, (128, 64, 64), (32, 64, 64))
    batch, shape = arr.batch_info((Ellipsis,))
    bad = torch.empty(shape, dtype=torch.int16, device=device)
    with pytest.raises(TypeError):
        arr.codec_pipeline.prepare_read(batch, bad)
    # planning fails after the staging job began (the job is aborted, not leaked)
    out = torch.empty(shape, dtype=torch.float32, device=device)
    real = P.plan_decode

    def boom(*a, **k):
        raise RuntimeError("planning failed")

    monkeypatch.setattr(P, "plan_decode", boom)
    with pytest.raises(RuntimeError, match="planning failed"):
        arr.codec_pipeline.prepare_read(batch, out)
    monkeypatch.setattr(P, "plan_decode", real)
    assert arr[...].tobytes() == O.read(host, meta).tobytes()
    assert isinstance(st, zarr_hip.LocalStore)


@pytest.mark.parametrize("kind", ["memory", "pinned"])
def test_slab_read_middle_band_keeps_out(device, kind):
    """A >= 16 MiB host out of which the batch covers only a middle band of
    dim-0 rows (in two non-adjacent bands): the rows before, between and after
    keep their values (the slab bounce copies back whole)."""
    import zarr_hip

    shape, chunks = (512, 128, 128), (32, 128, 128)
    meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 0.0, codecs=[LE, CRC])
    host = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    store = zarr_hip.PinnedMemoryStore(dict(host)) if kind == "pinned" else zarr_hip.MemoryStore(dict(host))
    arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=[LE, CRC])
    bands = [(96, 224), (320, 448)]
    batch = []
    for a, b in bands:
        bb, _ = arr.batch_info((slice(a, b),))
        for bg, spec, csel, osel, comp in bb:  # shift into the full-shape out
            o0 = osel[0]
            batch.append((bg, spec, csel, (slice(o0.start + a, o0.stop + a, 1),) + tuple(osel[1:]), comp))
    out = np.full(shape, -3.5, np.float32)
    res = arr.codec_pipeline.read_sync(batch, out)
    assert all(r["status"] == "present" for r in res)
    want = np.full(shape, -3.5, np.float32)
    full = O.read(host, meta)
    for a, b in bands:
        want[a:b] = full[a:b]
    assert out.tobytes() == want.tobytes()


# ------------------------------------------------------------ per-call plan cache
def _device_array(device, shape, chunks, codecs, fill=0.0, shards=None):
    import zarr_hip

    if shards is not None:
        meta = O.ArrayMeta(shape, shards, np.dtype("float32"), fill, codecs=[SHARD(chunks, codecs)])
    else:
        meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), fill, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    store = zarr_hip.DeviceStore.from_host(host, device)
    if shards is not None:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", fill, shards=shards, inner_codecs=codecs)
    else:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", fill, codecs=codecs)
    return arr, store, host, meta


@pytest.mark.parametrize("sharded", [False, True])
def test_cached_read_sees_overwrite_and_delete(device, sharded):
    """Two identical reads: the second is served by the cached program (no
    planning).  An overwrite between two cached reads is seen, and so is a
    delete (fill) and a rewrite that grows the arena."""
    import torch

    arr, store, host, meta = _device_array(device, (128, 64, 64), (32, 32, 32), [LE, CRC],
                                           shards=(64, 64, 64) if sharded else None)
    pipe = arr.codec_pipeline
    out = torch.empty((128, 64, 64), dtype=torch.float32, device=device)
    arr.get((Ellipsis,), out=out)
    assert len(pipe._read_cache) == 1
    prog = next(iter(pipe._read_cache.values()))
    arr.get((Ellipsis,), out=out)
    assert next(iter(pipe._read_cache.values())) is prog  # served by the cached program
    assert out.cpu().numpy().tobytes() == O.read(host, meta).tobytes()
    # overwrite a region through the GPU writer (host oracle mirrors it)
    new = _data((40, 64, 64), "float32", seed=7)
    arr.set((slice(30, 70),), torch.from_numpy(new).to(device))
    O.write(host, meta, (slice(30, 70),), new)
    arr.get((Ellipsis,), out=out)
    assert out.cpu().numpy().tobytes() == O.read(host, meta).tobytes()
    assert next(iter(pipe._read_cache.values())) is not prog  # re-planned
    # delete one stored object -> fill
    key = "c/1/0/0"
    store.delete_sync(key)
    host.pop(key)
    arr.get((Ellipsis,), out=out)
    assert out.cpu().numpy().tobytes() == O.read(host, meta).tobytes()
    # a fresh out tensor of the same geometry reuses the cached program
    prog = next(iter(pipe._read_cache.values()))
    out2 = torch.empty_like(out)
    arr.get((Ellipsis,), out=out2)
    assert next(iter(pipe._read_cache.values())) is prog
    assert out2.cpu().numpy().tobytes() == O.read(host, meta).tobytes()


def test_cached_read_new_store_same_keys(device):
    """One pipeline reads store A, A is dropped, store B with different bytes
    at the same keys is read through the same pipeline: the result is B's
    (the cache keys on the store object, not its address), and A's program
    -- holding A's HBM arena -- leaves the cache."""
    import gc

    import torch

    import zarr_hip

    shape, chunks = (64, 64, 64), (32, 32, 32)
    arr, store, host, meta = _device_array(device, shape, chunks, [LE, CRC])
    pipe = arr.codec_pipeline
    batch, _ = arr.batch_info((Ellipsis,))
    out = torch.empty(shape, dtype=torch.float32, device=device)
    pipe.read_sync(batch, out)
    assert len(pipe._read_cache) == 1
    for _round in range(3):
        host2 = {}
        O.write(host2, meta, (Ellipsis,), _data(shape, "float32", seed=11 + _round))
        del arr, store, batch
        gc.collect()
        store = zarr_hip.DeviceStore.from_host(host2, device)
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=[LE, CRC])
        batch, _ = arr.batch_info((Ellipsis,))
        pipe.read_sync(batch, out)
        assert out.cpu().numpy().tobytes() == O.read(host2, meta).tobytes()
        assert len(pipe._read_cache) == 1  # the dead store's program was dropped


def test_cached_read_crc_error_then_recovery(device):
    """A cached program re-verifies every CRC: bytes corrupted in HBM after
    the first read raise the reference's message, restored bytes read clean."""
    import torch

    arr, store, host, meta = _device_array(device, (64, 64), (32, 32), [LE, CRC])
    out = torch.empty((64, 64), dtype=torch.float32, device=device)
    arr.get((Ellipsis,), out=out)
    ref = store.get_sync("c/1/0")
    ref.arena.buf[ref.offset + 9] ^= 0x40
    bad = bytearray(host["c/1/0"])
    bad[9] ^= 0x40
    with pytest.raises(ValueError) as want:
        O.read({**host, "c/1/0": bytes(bad)}, meta)
    with pytest.raises(ValueError) as got:
        arr.get((Ellipsis,), out=out)
    assert str(got.value) == str(want.value)
    ref.arena.buf[ref.offset + 9] ^= 0x40
    arr.get((Ellipsis,), out=out)
    assert out.cpu().numpy().tobytes() == O.read(host, meta).tobytes()


def test_cached_read_partial_selections(device):
    """Different selections are different cache entries; each stays exact."""
    import torch

    arr, store, host, meta = _device_array(device, (96, 80, 40), (32, 16, 40), [LE, CRC])
    sels = [(Ellipsis,), (slice(5, 90), slice(None, None, 3), 7), (slice(40, 41), slice(3, 77), slice(0, 40, 5))]
    for _ in range(2):
        for sel in sels:
            want = O.read(host, meta, sel)
            out = torch.empty(want.shape, dtype=torch.float32, device=device)
            arr.get(sel, out=out)
            assert out.cpu().numpy().tobytes() == np.ascontiguousarray(want).tobytes()
    assert len(arr.codec_pipeline._read_cache) == len(sels)


# ------------------------------------------------------ stale prepared programs
def test_prepared_program_refuses_stale_offsets(device):
    """A program planned before a write (whose freed region the store may hand
    out again at once) refuses to launch; so does a ReadGraph holding it."""
    import torch

    import zarr_hip

    arr, store, host, meta = _device_array(device, (64, 64), (32, 32), [LE, CRC])
    prog, out = arr.prepare_read((Ellipsis,))
    g = zarr_hip.ReadGraph([prog], 2, device)
    g.replay()
    g.results()
    arr.set((slice(0, 32), slice(0, 32)), torch.zeros((32, 32), dtype=torch.float32, device=device) + 2.0)
    with pytest.raises(RuntimeError, match="changed since this read was planned"):
        prog.launch()
    with pytest.raises(RuntimeError, match="changed since this read was planned"):
        g.replay()
    prog2, out2 = arr.prepare_read((Ellipsis,))
    prog2.launch()
    prog2.results()
    O.write(host, meta, (slice(0, 32), slice(0, 32)), np.full((32, 32), 2.0, np.float32))
    assert out2.cpu().numpy().tobytes() == O.read(host, meta).tobytes()

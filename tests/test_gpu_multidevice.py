"""GPU tests of the single-process multi-device read (zarr_hip.parallel.
DeviceGroup): a batch split round-robin by item over a device list, each
device decoding its sub-batch on its own stream from its own host thread into
its own out.  On the one-GPU box the list is [0, 0] (two workers on one card,
the same code path as eight GPUs of a node); the union of the devices' regions
and the gathered out are compared with the CPU oracle bit for bit."""

import os

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import CRC, LE, SHARD, _data

pytestmark = pytest.mark.gpu


def _arr(device, kind, shape, chunks, codecs, shards=None):
    import zarr_hip

    if shards is not None:
        meta = O.ArrayMeta(shape, shards, np.dtype("float32"), 0.0, codecs=[SHARD(chunks, codecs)])
    else:
        meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 0.0, codecs=codecs)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    store = zarr_hip.DeviceStore.from_host(host, device) if kind == "device" else \
        zarr_hip.PinnedMemoryStore(dict(host)) if kind == "pinned" else zarr_hip.MemoryStore(dict(host))
    if shards is not None:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, shards=shards, inner_codecs=codecs)
    else:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=codecs)
    return arr, host, meta


@pytest.mark.parametrize("kind", ["device", "memory", "pinned"])
@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("n_dev", [2, 3])
def test_device_group_matches_oracle(device, kind, sharded, n_dev):
    import torch

    from zarr_hip.parallel import DeviceGroup, partition

    shape = (128, 96, 64)
    arr, host, meta = _arr(device, kind, shape, (32, 32, 32), [LE, CRC],
                           shards=(64, 96, 64) if sharded else None)
    grp = DeviceGroup([0] * n_dev)
    for sel in [(Ellipsis,), (slice(5, 120, 3), slice(None), slice(7, 60))]:
        batch, out_shape = arr.batch_info(sel)
        outs, res = grp.read_sync(arr.codec_pipeline, batch, out_shape, "float32")
        assert len(outs) == n_dev and len(res) == len(batch)
        assert all(r["status"] == "present" for r in res)
        want = np.ascontiguousarray(O.read(host, meta, sel))
        # every device holds exactly its own items' regions
        for r, out in enumerate(outs):
            o = out.cpu().numpy()
            for j in partition(len(batch), n_dev, r):
                osel = tuple(batch[j][3])
                assert o[osel].tobytes() == want[osel].tobytes()
        # gathered onto one out: the whole selection
        into = torch.empty(out_shape, dtype=torch.float32, device=device)
        prog = grp.prepare_read(arr.codec_pipeline, batch, out_shape, "float32")
        prog.launch()
        prog.results()
        prog.gather(batch, into)
        assert into.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize("keep", [lambda j: j % 3 != 1, lambda j: j < 5, lambda j: j >= 12])
def test_gather_partial_batch_keeps_unselected_regions(device, keep):
    """gather of a batch that does not tile the devices' bands (a subset of
    the chunks) into a pre-filled `into`: only the items' regions change, the
    rest keeps its sentinel (the per-device outs hold garbage there: a band
    copy would overwrite it -- advisor round 5)."""
    import torch

    from zarr_hip.parallel import DeviceGroup

    shape = (128, 96, 64)
    arr, host, meta = _arr(device, "device", shape, (32, 32, 32), [LE, CRC])
    batch, out_shape = arr.batch_info((Ellipsis,))
    sub = [it for j, it in enumerate(batch) if keep(j)]
    want = np.full(out_shape, -5.0, np.float32)
    full = O.read(host, meta)
    for it in sub:
        osel = tuple(it[3])
        want[osel] = full[osel]
    for n_dev in (2, 3):
        grp = DeviceGroup([0] * n_dev)
        prog = grp.prepare_read(arr.codec_pipeline, sub, out_shape, "float32")
        prog.launch()
        prog.results()
        into = torch.full(out_shape, -5.0, dtype=torch.float32, device=device)
        prog.gather(sub, into)
        assert into.cpu().numpy().tobytes() == want.tobytes()


def test_device_group_crc_error_surfaces(device):
    """A corrupted chunk on any device raises the reference's message."""
    import zarr_hip
    from zarr_hip.parallel import DeviceGroup

    meta = O.ArrayMeta((64, 64), (16, 16), np.dtype("float32"), 0.0, codecs=[LE, CRC])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data((64, 64), "float32"))
    bad = bytearray(host["c/3/1"])
    bad[40] ^= 0x04
    host["c/3/1"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.DeviceStore.from_host(host, device), (64, 64), (16, 16), "float32",
                                0.0, codecs=[LE, CRC])
    batch, out_shape = arr.batch_info((Ellipsis,))
    with pytest.raises(ValueError) as got:
        DeviceGroup([0, 0]).read_sync(arr.codec_pipeline, batch, out_shape, "float32")
    assert str(got.value) == str(want.value)


def test_device_group_compressed_chain(device):
    """The host stage runs in each device's thread (gzip inner chunks)."""
    from zarr_hip.parallel import DeviceGroup

    arr, host, meta = _arr(device, "memory", (64, 48), (16, 16),
                           [LE, {"name": "gzip", "configuration": {"level": 1}}], shards=(32, 48))
    batch, out_shape = arr.batch_info((Ellipsis,))
    prog = DeviceGroup([0, 0]).prepare_read(arr.codec_pipeline, batch, out_shape, "float32")
    prog.launch()
    prog.results()
    import torch

    into = torch.empty(out_shape, dtype=torch.float32, device=device)
    prog.gather(batch, into)
    assert into.cpu().numpy().tobytes() == O.read(host, meta).tobytes()


# ------------------------------------------------- HipCodecPipeline(devices=...)
@pytest.mark.parametrize("kind", ["memory", "device"])
@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("devs", ["0,0", "0,0,0"])
def test_pipeline_devices_through_array(device, monkeypatch, kind, sharded, devs):
    """A zarr caller's arr[...] / arr[...] = v with a device list (zarr config
    "hip.devices", env ZARR_HIP__DEVICES): the items split into bands of the
    out over the devices, every band decoded / encoded on its device; reads
    into host and device outs and the written store compared with the oracle."""
    import torch

    import zarr_hip

    monkeypatch.setenv("ZARR_HIP__DEVICES", devs)
    shape, chunks = (128, 96, 64), (32, 32, 32)
    shards = (64, 96, 64) if sharded else None
    if shards is not None:
        meta = O.ArrayMeta(shape, shards, np.dtype("float32"), 0.0, codecs=[SHARD(chunks, [LE, CRC])])
    else:
        meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 0.0, codecs=[LE, CRC])
    store = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
    if shards is not None:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, shards=shards, inner_codecs=[LE, CRC])
    else:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=[LE, CRC])
    assert arr.codec_pipeline.devices == tuple(int(d) for d in devs.split(","))
    host: dict = {}
    data = _data(shape, "float32")
    for sel, val in [((Ellipsis,), data), ((slice(10, 100), slice(5, 90), slice(3, 60)), _data((90, 85, 57), "float32", seed=4)),
                     ((slice(64, 128),), np.float32(2.5))]:
        arr[sel] = val
        O.write(host, meta, sel, val)
        stored = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert stored == host
    for sel in [(Ellipsis,), (slice(5, 120, 3), slice(None), slice(7, 60)), (slice(30, 31), slice(None), 5)]:
        want = np.ascontiguousarray(O.read(host, meta, sel))
        assert np.asarray(arr[sel]).tobytes() == want.tobytes()
    out = torch.empty(shape, dtype=torch.float32, device=device)
    arr.get((Ellipsis,), out=out)
    assert out.cpu().numpy().tobytes() == O.read(host, meta).tobytes()
    outf = torch.empty(tuple(reversed(shape)), dtype=torch.float32, device=device).permute(2, 1, 0)  # F order
    arr.get((Ellipsis,), out=outf)
    assert outf.cpu().numpy().tobytes() == O.read(host, meta).tobytes()


def test_pipeline_devices_crc_error(device, monkeypatch):
    import zarr_hip

    monkeypatch.setenv("ZARR_HIP__DEVICES", "0,0")
    meta = O.ArrayMeta((64, 64), (16, 16), np.dtype("float32"), 0.0, codecs=[LE, CRC])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data((64, 64), "float32"))
    bad = bytearray(host["c/3/1"])
    bad[40] ^= 0x04
    host["c/3/1"] = bytes(bad)
    with pytest.raises(ValueError) as want:
        O.read(host, meta)
    arr = zarr_hip.Array.create(zarr_hip.MemoryStore(dict(host)), (64, 64), (16, 16), "float32", 0.0,
                                codecs=[LE, CRC])
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)


@pytest.mark.parametrize("sharded", [False, True])
def test_device_store_decodes_where_its_bytes_are(device, monkeypatch, sharded):
    """devices=[0, 0] over a DeviceStore on GPU 0: every item decodes on the
    GPU that holds its bytes (parallel.placement) -- no encoded byte is
    staged device to device (staging.D2D_COPIES unchanged) -- for a device
    out on that GPU (the single-device read), a host out (decoded there, one
    copy back) and a strided selection; all exact against the oracle."""
    import torch

    import zarr_hip
    from zarr_hip import staging

    monkeypatch.setenv("ZARR_HIP__DEVICES", "0,0")
    shape, chunks = (128, 96, 64), (32, 32, 32)
    shards = (64, 96, 64) if sharded else None
    codecs = [SHARD(chunks, [LE, CRC])] if sharded else [LE, CRC]
    meta = O.ArrayMeta(shape, shards or chunks, np.dtype("float32"), 0.0, codecs=codecs)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), _data(shape, "float32"))
    store = zarr_hip.DeviceStore.from_host(host, device)
    arr = zarr_hip.Array.create(store, shape, shards or chunks, "float32", 0.0, codecs=codecs)
    assert arr.codec_pipeline.devices == (0, 0)
    before = staging.D2D_COPIES[0]
    for sel in [(Ellipsis,), (slice(5, 120, 3), slice(None), slice(7, 60))]:
        want = np.ascontiguousarray(O.read(host, meta, sel))
        assert np.asarray(arr[sel]).tobytes() == want.tobytes()
        batch, out_shape = arr.batch_info(sel)
        hout = np.full(out_shape, -7.0, np.float32)
        arr.codec_pipeline.read_sync(batch, hout)
        assert hout.tobytes() == want.tobytes()
        dout = torch.empty(out_shape, dtype=torch.float32, device=device)
        arr.codec_pipeline.read_sync(batch, dout)
        assert dout.cpu().numpy().tobytes() == want.tobytes()
    assert staging.D2D_COPIES[0] == before


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_MULTI", "24"))))
def test_random_device_list(device, monkeypatch, seed):
    """Seeded parity of the device-list pipeline (devices [0, 0] or [0, 0, 0]):
    the regular and rectilinear fuzz geometries (test_gpu_fuzz._case /
    _rect_case: sharding, transposes, endianness, crc32c, edge chunks), a whole
    write and a random write, then random reads through arr[sel] and through
    read_sync into pre-filled host and device outs; stores and reads compared
    with the oracle."""
    import torch

    import zarr_hip
    from test_gpu_fuzz import _case, _rand_sel, _rect_case

    monkeypatch.setenv("ZARR_HIP__DEVICES", "0,0" if seed % 2 == 0 else "0,0,0")
    if seed % 3 == 2:
        rng, shape, grid, inner, dtype, chain, fill = _rect_case(seed)
        loc = str(rng.choice(["end", "start"]))
        codecs = chain if inner is None else [SHARD(inner, chain, loc)]
        meta = O.ArrayMeta(shape, grid, np.dtype(dtype), fill, codecs=codecs)
        kw = {"codecs": chain} if inner is None else {"codecs": chain, "shards": grid, "index_location": loc}
        chunks = grid if inner is None else inner
    else:
        rng, shape, chunks, dtype, codecs, fill = _case(seed)
        meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
        kw = {"codecs": codecs}
    store = zarr_hip.DeviceStore(device) if seed % 4 < 2 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, **kw)
    assert len(arr.codec_pipeline.devices) in (2, 3)
    host: dict = {}
    data = _data(shape, dtype, seed)
    sel = _rand_sel(rng, shape)
    wshape = O.read({}, meta, sel).shape
    val = _data(wshape, dtype, seed + 3) if wshape else _data((1,), dtype, seed + 3)[0]
    for s, v in [((Ellipsis,), data), (sel, val)]:
        O.write(host, meta, s, v)
        arr[s] = v
        got = {k: bytes(b) for k, b in store.to_dict().items() if not k.endswith("zarr.json")}
        assert got == host, (s, shape, chunks, codecs)
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        want = np.ascontiguousarray(want)
        assert got.tobytes() == want.tobytes(), (sel, shape, chunks, codecs)
        batch, out_shape = arr.batch_info(sel)
        if not batch or not out_shape:
            continue
        hout = np.full(out_shape, 3, np.dtype(dtype))
        arr.codec_pipeline.read_sync(batch, hout)
        assert hout.tobytes() == want.tobytes(), (sel, shape, chunks, codecs)
        dout = torch.from_numpy(np.full(out_shape, 3, np.dtype(dtype))).to(device)
        arr.codec_pipeline.read_sync(batch, dout)
        assert dout.cpu().numpy().tobytes() == want.tobytes(), (sel, shape, chunks, codecs)

"""Concurrent use of one pipeline from several host threads -- what zarr's
async API does when it runs read_sync / write_sync through asyncio.to_thread
(codec_pipeline.py:1257-1319: `await asyncio.to_thread(self.read_sync, ...)`)
for independent requests: reads of one array from four threads at once
(random selections through arr[sel], arr.get into device outs, the per-call
plan cache and its checkout, pooled buffers, the library's thread-local upload
slots and staging pool) while two more threads write arrays of their own.
Every read is compared with the CPU oracle's, every store byte for byte."""

import os
import threading

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import CRC, LE, SHARD, _data
from test_gpu_fuzz import _rand_sel

pytestmark = pytest.mark.gpu

SHAPE, CHUNKS = (96, 80, 64), (16, 16, 32)
ITERS = int(os.environ.get("ZARR_HIP_CONC_ITERS", "12"))  # reads per thread (stress runs: more)


def _setup(kind, sharded, device):
    import zarr_hip

    store = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
    if sharded:
        codecs = [SHARD(CHUNKS, [LE, CRC])]
        meta = O.ArrayMeta(SHAPE, (32, 80, 64), np.dtype("float32"), 0.0, codecs=codecs)
        arr = zarr_hip.Array.create(store, SHAPE, CHUNKS, "float32", 0.0, shards=(32, 80, 64),
                                    inner_codecs=[LE, CRC])
    else:
        meta = O.ArrayMeta(SHAPE, CHUNKS, np.dtype("float32"), 0.0, codecs=[LE, CRC])
        arr = zarr_hip.Array.create(store, SHAPE, CHUNKS, "float32", 0.0, codecs=[LE, CRC])
    return store, arr, meta


def _run(threads):
    errs: list = []

    def wrap(fn):
        def go():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001 -- reported below with its thread
                errs.append(e)
        return go

    ts = [threading.Thread(target=wrap(fn)) for fn in threads]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    if errs:
        raise errs[0]


@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("kind", ["device", "memory"])
def test_concurrent_reads_and_writes(kind, sharded, device):
    import torch

    store, arr, meta = _setup(kind, sharded, device)
    data = _data(SHAPE, "float32", seed=3)
    arr[...] = data
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    full = O.read(host, meta)

    def reader(r):
        def go():
            rng = np.random.default_rng(100 + r)
            repeat = _rand_sel(rng, SHAPE)  # read again and again: the plan cache
            for i in range(ITERS):
                sel = repeat if i % 3 == 0 else _rand_sel(rng, SHAPE)
                want = np.ascontiguousarray(full[sel])
                got = arr[sel]
                assert got.tobytes() == want.tobytes(), (r, i, sel)
                if kind == "device":
                    d = arr.get(sel)
                    assert d.cpu().numpy().tobytes() == want.tobytes(), (r, i, sel)
                    torch.cuda.current_stream(device).synchronize()
        return go

    written: dict = {}

    def writer(w):
        def go():
            st2, a2, m2 = _setup(kind, sharded, device)
            h2: dict = {}
            rng = np.random.default_rng(200 + w)
            for i in range(4):
                sel = (Ellipsis,) if i == 0 else _rand_sel(rng, SHAPE)
                shp = O.read(h2, m2, sel).shape
                val = _data(shp, "float32", seed=300 + 10 * w + i) if shp else np.float32(w + i)
                a2[sel] = val
                O.write(h2, m2, sel, val)
            written[w] = (st2, h2)
        return go

    _run([reader(r) for r in range(4)] + [writer(w) for w in range(2)])
    for w, (st2, h2) in written.items():
        got = {k: bytes(v) for k, v in st2.to_dict().items() if not k.endswith("zarr.json")}
        assert got == h2, w
    # the shared array is unchanged by the readers
    assert {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")} == host

"""A long-lived process reading and writing through one pipeline: the per-call
plan cache (bounded, LRU), the pooled device buffers (at most _BUF_POOL_MAX per
size), the library's pinned staging windows and upload slots are reused, not
accumulated.  After a warm-up, a few thousand random reads and writes on a
device store and a host store must not grow the caching allocator's live
bytes or the process's resident set beyond a small bound."""

import os

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import CRC, LE, SHARD, _data
from test_gpu_fuzz import _rand_sel

pytestmark = pytest.mark.gpu

ITERS = int(os.environ.get("ZARR_HIP_STEADY_ITERS", "1500"))


def _rss() -> int:
    import psutil

    return psutil.Process().memory_info().rss


@pytest.mark.parametrize("kind,sharded", [("device", False), ("device", True), ("memory", False), ("memory", True)])
def test_no_growth_under_repeated_reads_and_writes(kind, sharded, device):
    import torch

    import zarr_hip

    shape, chunks = (96, 64, 64), (16, 32, 32)
    store = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
    if sharded:
        codecs = [SHARD(chunks, [LE, CRC])]
        meta = O.ArrayMeta(shape, (32, 64, 64), np.dtype("float32"), 0.0, codecs=codecs)
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, shards=(32, 64, 64), inner_codecs=[LE, CRC])
    else:
        meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 0.0, codecs=[LE, CRC])
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=[LE, CRC])
    host: dict = {}
    data = _data(shape, "float32", seed=11)
    arr[...] = data
    O.write(host, meta, (Ellipsis,), data)
    full = O.read(host, meta)
    rng = np.random.default_rng(5)
    sels = [_rand_sel(rng, shape) for _ in range(64)]  # a working set: the plan cache sees repeats

    def step(i):
        sel = sels[i % len(sels)]
        if i % 50 == 49:  # a write now and then (plans of the old bytes go stale)
            v = np.float32(i % 7)
            arr[sel] = v
            full[sel] = v
        got = arr[sel]
        assert got.tobytes() == np.ascontiguousarray(full[sel]).tobytes(), (i, sel)

    for i in range(200):  # warm: plans, pools, staging windows
        step(i)
    torch.cuda.synchronize(device)
    dev0, rss0 = torch.cuda.memory_allocated(device), _rss()
    for i in range(200, 200 + ITERS):
        step(i)
    torch.cuda.synchronize(device)
    dev1, rss1 = torch.cuda.memory_allocated(device), _rss()
    # a repeat-heavy working set: the bounded cache and pools settle during
    # warm-up; allow some slack for allocator granularity and late plans
    assert dev1 - dev0 < (64 << 20), (dev0, dev1)
    assert rss1 - rss0 < (256 << 20), (rss0, rss1)

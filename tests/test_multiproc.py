"""N>1 path on CPU: world_size-2 `gloo` process group.  Each rank plans its
round-robin share of a sharded batch; the ranks' chunk sets are disjoint and
together cover the batch, and the union of their planned out regions equals
the single-process plan (checked with an all_gather of digests)."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from zarr_hip.parallel import partition


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["round_robin", "contiguous"])
@pytest.mark.parametrize("n,world", [(64, 2), (7, 3), (0, 2), (512, 8)])
def test_partition_disjoint_covering(n, world, mode):
    parts = [partition(n, world, r, mode) for r in range(world)]
    allv = np.concatenate(parts) if parts else np.zeros(0, int)
    assert sorted(allv.tolist()) == list(range(n))
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "zarr-python_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch

    import zarr_hip
    from zarr_hip.parallel import rank_batch
    from zarr_hip.planner import analyze_chain, plan_decode

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = zarr_hip.MemoryStore()
        arr = zarr_hip.Array.create(
            st, (64, 48, 32), (32, 16, 16), "float32", 0.0,
            codecs=[{"name": "sharding_indexed", "configuration": {
                "chunk_shape": [8, 8, 8],
                "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                           {"name": "crc32c"}]}}])
        batch, out_shape = arr.batch_info((slice(3, 61), slice(None), slice(5, 30, 2)))
        mine = rank_batch(batch, world, rank)
        chain = analyze_chain(arr.codec_pipeline.codecs, arr.spec)
        strides = [int(x) for x in np.empty(out_shape, np.float32).strides]  # bytes
        items = [(i * 10000, 9000, False, it[2], it[3]) for i, it in enumerate(mine)]
        offs = set()
        if items:
            t = plan_decode(chain, arr.spec, items, strides, 0)
            offs = set((int(o), int(s)) for o, s in zip(t.chunks["out_off"], t.chunks["sel"]))
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, len(mine), sorted(o for o, _ in offs)))
        q.put(gathered if rank == 0 else None)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_cover_batch():
    import sys

    import zarr_hip
    from zarr_hip.planner import analyze_chain, plan_decode

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    gathered = [r for r in res if r is not None][0]
    # single-process reference plan
    st = zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(
        st, (64, 48, 32), (32, 16, 16), "float32", 0.0,
        codecs=[{"name": "sharding_indexed", "configuration": {
            "chunk_shape": [8, 8, 8],
            "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                       {"name": "crc32c"}]}}])
    batch, out_shape = arr.batch_info((slice(3, 61), slice(None), slice(5, 30, 2)))
    chain = analyze_chain(arr.codec_pipeline.codecs, arr.spec)
    strides = [int(x) for x in np.empty(out_shape, np.float32).strides]  # bytes
    t = plan_decode(chain, arr.spec, [(0, 9000, False, it[2], it[3]) for it in batch], strides, 0)
    full = sorted(int(o) for o in t.chunks["out_off"])
    union = sorted(o for _, _, offs in gathered for o in offs)
    assert union == full
    assert sum(n for _, n, _ in gathered) == len(batch)
    assert len(set(union)) == len(union)  # disjoint out regions

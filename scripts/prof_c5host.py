#!/usr/bin/env python
"""Where a C5 read from a HOST store spends its time (measurement only):
bench.c5_host's setup (2048^3 int16, 256^3 shards of 64^3 inner chunks, a
host MemoryStore), then the seeded 10 % batch read into a device out, with
perf_counter wrappers around the host path's stages and a cProfile top list,
as JSON lines."""

import cProfile
import functools
import io
import json
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402
import workloads as W  # noqa: E402

_T: dict = {}


def _wrap(owner, name, label):
    fn = getattr(owner, name)

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            e = _T.setdefault(label, [0, 0.0])
            e[0] += 1
            e[1] += time.perf_counter() - t0
    setattr(owner, name, w)


def main():
    import torch

    import zarr_hip
    from zarr_hip import pipeline as P
    from zarr_hip import staging as ST
    from zarr_hip import store as S

    dev = torch.device("cuda:0")
    g = W.C5
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    gen = torch.Generator(device=dev).manual_seed(0)
    data = torch.randint(-2 ** 15, 2 ** 15, shape, generator=gen, device=dev, dtype=torch.int16)
    n_shards = int(np.prod([s // c for s, c in zip(shape, shards)]))
    shard_bytes = int(np.prod(shards)) * 2 + 64 * 4 + 64 * 16 + 4
    dstore = zarr_hip.DeviceStore(dev, capacity=n_shards * (shard_bytes + 256) + (1 << 24))
    darr = zarr_hip.Array.create(dstore, shape, inner, "int16", 0, shards=shards, inner_codecs=[bench.LE, bench.CRC])
    sbatch, _ = darr.batch_info((Ellipsis,))
    for i in range(0, len(sbatch), 64):
        darr.codec_pipeline.write_sync(sbatch[i:i + 64], data)
    torch.cuda.synchronize(dev)
    host = zarr_hip.MemoryStore(dstore.to_dict())
    del dstore, darr
    torch.cuda.empty_cache()
    arr = zarr_hip.Array.open(host)
    grid = tuple(s // i for s, i in zip(shape, inner))
    coords = W.partial_selection(grid)
    batch = W.inner_chunk_batch(arr, host, coords, inner)
    out = torch.empty(shape, dtype=torch.int16, device=dev)
    arr.codec_pipeline.read_sync(batch, out)
    torch.cuda.synchronize(dev)
    bench.check_regions(out, data, batch, "c5 host")
    del data
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        arr.codec_pipeline.read_sync(batch, out)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"ms_per_read": round(float(np.median(ts)) * 1e3, 2), "inner_chunks": len(batch)}),
          flush=True)
    stages = [(ST, "gather_sharded_partial", "gather_sharded_partial"), (ST, "stage", "stage"),
              (ST, "staged_host", "staged_host"), (ST, "_touched_slots", "_touched_slots"),
              (S.MemoryStore, "get_ranges_sync", "MemoryStore.get_ranges_sync"),
              (S.MemoryStore, "get_sync", "MemoryStore.get_sync"),
              (P.HipCodecPipeline, "prepare_read", "prepare_read"), (P, "plan_decode", "plan_decode"),
              (P.DecodeProgram, "launch", "DecodeProgram.launch"), (P.DecodeProgram, "results_fast", "results_fast"),
              (ST.Pending, "finish", "Pending.finish")]
    for owner, name, label in stages:
        if hasattr(owner, name):
            _wrap(owner, name, label)
    _T.clear()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    arr.codec_pipeline.read_sync(batch, out)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    print(json.dumps({"wrapped_ms": round(wall * 1e3, 2),
                      "stages_ms": {k: round(v[1] * 1e3, 2) for k, v in sorted(_T.items(), key=lambda kv: -kv[1][1])},
                      "stage_calls": {k: v[0] for k, v in _T.items()}}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    arr.codec_pipeline.read_sync(batch, out)
    torch.cuda.synchronize(dev)
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(json.dumps({"sort": key, "stats": s.getvalue()}), flush=True)


if __name__ == "__main__":
    main()

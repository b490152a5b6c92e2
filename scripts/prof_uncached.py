#!/usr/bin/env python
"""Where an uncached per-call read spends its host time (measurement only):
the headline array in HBM, read_sync with the plan cache off, a DIFFERENT
selection every call (a data loader walking the array), under cProfile.
Prints the per-call wall, then the top functions by cumulative and by own
time as JSON lines."""

import cProfile
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


def main():
    import torch

    from zarr_hip import pipeline as P

    dev = torch.device("cuda:0")
    g = W.HEADLINE
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    src = torch.from_numpy(W.synthetic(shape)).to(dev)
    arr = bench.build_replica(dev, src, shape, inner, [W.LE, W.CRC], shards=shards)
    sels = [(slice(64 * (i % 4), 64 * (i % 4) + 128 + 64 * (i % 2)), slice(None), slice(None)) for i in range(8)]
    batches = [arr.batch_info(s) for s in sels]
    outs = [torch.empty(b[1], dtype=torch.float32, device=dev) for b in batches]
    P.READ_CACHE_SIZE = 0
    pipe = arr.codec_pipeline
    for i in range(16):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    torch.cuda.synchronize(dev)
    n = int(os.environ.get("CALLS", "200"))
    t0 = time.perf_counter()
    for i in range(n):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    wall = (time.perf_counter() - t0) / n
    print(json.dumps({"uncached_ms_per_call": round(wall * 1e3, 4), "calls": n}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(json.dumps({"sort": key, "stats": s.getvalue()}), flush=True)
    for i in range(8):
        pipe.read_sync(batches[i][0], outs[i])
        want = src[sels[i]]
        if not torch.equal(outs[i].view(torch.int32), want.contiguous().view(torch.int32)):
            raise SystemExit("prof_uncached: decoded bytes differ")


if __name__ == "__main__":
    main()

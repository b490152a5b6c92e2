#!/usr/bin/env python
"""Where an uncached per-call read spends its host time (measurement only):
the headline array in HBM, read_sync with the plan cache off, a DIFFERENT
selection every call (a data loader walking the array).  Prints the per-call
wall, then each stage's inclusive mean (perf_counter wrappers around the
read path's functions; a wrapper costs ~0.3 us), then a cProfile top list,
as JSON lines."""

import cProfile
import functools
import io
import json
import os
import pstats
import sys
import time

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
    return fn


def main():
    import torch

    from zarr_hip import pipeline as P
    from zarr_hip import planner as PL
    from zarr_hip import staging as ST

    dev = torch.device("cuda:0")
    g = W.HEADLINE
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    src = torch.from_numpy(W.synthetic(shape)).to(dev)
    arr = bench.build_replica(dev, src, shape, inner, [W.LE, W.CRC], shards=shards)
    if os.environ.get("SEL") == "full":  # bench.device_read_call's read_sync_uncached: the whole array
        sels = [(slice(None), slice(None), slice(None))] * 8
    elif os.environ.get("SEL") == "bench":  # its varying leg: unaligned 128-row windows
        sels = [(slice(16 * i + 8, 16 * i + 136), slice(None), slice(None)) for i in range(8)]
    else:
        sels = [(slice(64 * (i % 4), 64 * (i % 4) + 128 + 64 * (i % 2)), slice(None), slice(None)) for i in range(8)]
    batches = [arr.batch_info(s) for s in sels]
    outs = [torch.empty(b[1], dtype=torch.float32, device=dev) for b in batches]
    P.READ_CACHE_SIZE = 0
    pipe = arr.codec_pipeline
    for i in range(16):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    torch.cuda.synchronize(dev)
    n = int(os.environ.get("CALLS", "400"))
    t0 = time.perf_counter()
    for i in range(n):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    wall = (time.perf_counter() - t0) / n
    print(json.dumps({"uncached_ms_per_call": round(wall * 1e3, 4), "calls": n}), flush=True)
    H = P.HipCodecPipeline
    stages = [
        (P, "normalize_batch", "normalize_batch"), (P, "_resolve_out", "_resolve_out"),
        (H, "prepare_read", "prepare_read"), (H, "_shard_space", "_shard_space"), (H, "_chain", "_chain"),
        (P, "_device_resident", "_device_resident"), (ST, "gather_sources", "gather_sources"),
        (P, "plan_decode", "plan_decode"), (PL, "_plan_native", "_plan_native"),
        (PL, "_native_ctx", "_native_ctx"), (P, "_kernel_flags", "_kernel_flags"),
        (P.DecodeLaunch, "__init__", "DecodeLaunch.__init__"), (P, "_rows_map_host", "_rows_map_host"),
        (P._Upload, "commit", "_Upload.commit"), (P, "_pool_take", "_pool_take"),
        (P, "_generations", "_generations"), (P.DecodeProgram, "launch", "DecodeProgram.launch"),
        (P.DecodeLaunch, "launch", "DecodeLaunch.launch"), (P.DecodeProgram, "results_fast", "results_fast"),
        (P.DecodeProgram, "release", "release"), (P, "_stream_handle", "_stream_handle"),
    ]
    for owner, name, label in stages:
        if hasattr(owner, name):
            _wrap(owner, name, label)
    _T.clear()
    t0 = time.perf_counter()
    for i in range(n):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    wall_w = (time.perf_counter() - t0) / n
    print(json.dumps({"wrapped_ms_per_call": round(wall_w * 1e3, 4),
                      "stages_us_per_call": {k: round(v[1] / n * 1e6, 2) for k, v in
                                             sorted(_T.items(), key=lambda kv: -kv[1][1])},
                      "stage_calls_per_read": {k: round(v[0] / n, 2) for k, v in _T.items()}}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n // 2):
        pipe.read_sync(batches[i % 8][0], outs[i % 8])
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(json.dumps({"sort": "tottime", "stats": s.getvalue()}), flush=True)
    for i in range(8):
        pipe.read_sync(batches[i][0], outs[i])
        want = src[sels[i]]
        if not torch.equal(outs[i].view(torch.int32), want.contiguous().view(torch.int32)):
            raise SystemExit("prof_uncached: decoded bytes differ")


if __name__ == "__main__":
    main()

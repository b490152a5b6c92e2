#!/usr/bin/env python
"""Phase breakdown of a host-resident read (measurement only): C2's 64 encoded
chunks in a host MemoryStore read into a device out by Array.get, with wall
time per phase (fetch + pack + H2D enqueue, planning, table uploads, launch,
sync/results) from wrappers around the product functions, plus the raw pinned
H2D rate on the same box.  One JSON line per phase."""

import json
import os
import sys
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402


def main():
    import torch

    import zarr_hip
    from zarr_hip import pipeline as PL
    from zarr_hip import planner, staging

    dev = torch.device("cuda:0")
    shape, chunks = (256, 256, 256), (64, 64, 64)
    data = bench.synthetic(shape)
    darr = bench.build_replica(dev, torch.from_numpy(data).to(dev), shape, chunks, [bench.LE, bench.CRC])
    kind = os.environ.get("STORE", "memory")
    if kind == "local":
        import tempfile

        if os.environ.get("NOFILE"):  # A/B: LocalStore bytes through Python reads + packing
            del zarr_hip.store.LocalStore.locate_sync
            kind = "local-pyread"
        host = zarr_hip.LocalStore(tempfile.mkdtemp(prefix="zhip_e2e_"))
        for k, v in darr.store_path.store.to_dict().items():
            host.set_sync(k, v)
    else:
        host = (zarr_hip.PinnedMemoryStore if kind == "pinned" else zarr_hip.MemoryStore)(
            darr.store_path.store.to_dict())
    arr = zarr_hip.Array.open(host)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    acc = defaultdict(list)

    def wrap(mod, name, key):
        fn = getattr(mod, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            acc[key].append(time.perf_counter() - t0)
            return r
        setattr(mod, name, w)

    wrap(staging, "gather_sources", "gather_sources(fetch+pack+h2d enqueue)")
    wrap(staging, "stage", "  stage(pack+h2d enqueue)")
    from zarr_hip import buffer as B
    wrap(B, "empty_pinned", "empty_pinned(out)")
    wrap(B, "copy_to_host_from_pinned", "copy_to_host_from_pinned")
    wrap(PL, "_slab_groups", "_slab_groups")
    wrap(PL.HipCodecPipeline, "_read_slabs", "_read_slabs(total)")
    runs = []
    inner_stage = staging.stage

    def count_runs(layout, *a, **k):
        addrs = [(staging._host_view(b).ctypes.data, off, n) for b, off, n in layout.pieces
                 if not isinstance(b, staging.FileRef)]
        r = min(1, len(addrs)) + sum(1 for (h0, d0, _), (h1, d1, _) in zip(addrs, addrs[1:]) if h1 - h0 != d1 - d0)
        runs.append(r)
        return inner_stage(layout, *a, **k)
    staging.stage = count_runs
    wrap(PL, "plan_decode", "plan_decode")
    wrap(PL.DecodeProgram, "launch", "launch")
    wrap(PL.DecodeProgram, "results", "results(sync)")
    orig_init = PL.DecodeLaunch.__init__

    def init(self, *a, **k):
        t0 = time.perf_counter()
        orig_init(self, *a, **k)
        acc["DecodeLaunch.__init__(uploads)"].append(time.perf_counter() - t0)
    PL.DecodeLaunch.__init__ = init
    from zarr_hip import _native as N

    lib = N.lib()
    if os.environ.get("SLAB"):  # measurement: slab group sizing (min MiB, max groups)
        mb, mg = (int(x) for x in os.environ["SLAB"].split(","))
        orig_groups = PL._slab_groups
        PL._slab_groups = lambda b, o, min_bytes=0, max_groups=0: orig_groups(b, o, mb << 20, mg)
    if os.environ.get("STREAMS"):
        lib.zhip_set_tuning(4, int(os.environ["STREAMS"]))
    begin = lib.zhip_stage_begin
    t_get = [0.0]

    def begin_w(*a):
        if t_get[0]:
            acc["get() start -> zhip_stage_begin call"].append(time.perf_counter() - t_get[0])
        return begin(*a)
    lib.zhip_stage_begin = begin_w
    for win in [int(x) for x in os.environ.get("WINDOWS", "1,2,4,8").split(",")]:
        staging.WINDOW = win << 20
        for i in range(12):
            torch.cuda.synchronize(dev)
            if os.environ.get("ONLY_HOST"):
                t0 = time.perf_counter()
                arr[...]
                if i >= 2:
                    acc["TOTAL __getitem__ only"].append(time.perf_counter() - t0)
                continue
            t0 = t_get[0] = time.perf_counter()
            arr.get((Ellipsis,), out=out)
            t_get[0] = 0.0
            torch.cuda.synchronize(dev)
            if i >= 2:
                acc[f"TOTAL get(out=device) {kind} window {win} MiB streams {os.environ.get('STREAMS', '1')}"].append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            arr[...]
            if i >= 2:
                acc[f"TOTAL __getitem__ (host out) {kind} window {win} MiB slab {os.environ.get('SLAB', '8,8')}"].append(time.perf_counter() - t0)
    assert out.view(torch.int32).cpu().numpy().tobytes() == data.view(np.int32).tobytes()
    if os.environ.get("CPROFILE"):
        import cProfile
        import io
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        for _ in range(20):
            arr.get((Ellipsis,), out=out)
        torch.cuda.synchronize(dev)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue(), file=sys.stderr)
    pin = torch.empty(data.nbytes, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(data.nbytes, dtype=torch.uint8, device=dev)
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dbuf.copy_(pin, non_blocking=True)
        torch.cuda.synchronize(dev)
        acc["raw pinned H2D 64 MiB"].append(time.perf_counter() - t0)
    print(json.dumps({"phase": "host-contiguous runs per stage", "runs": runs[-1:], "store": kind}), flush=True)
    for k, v in acc.items():
        print(json.dumps({"phase": k, "ms_med": round(float(np.median(v)) * 1e3, 3), "n": len(v)}), flush=True)


if __name__ == "__main__":
    main()

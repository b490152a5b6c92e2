#!/usr/bin/env python
"""Staging micro-measurements (measurement only): pinned allocation, host
packing rate (zhip_host_copy from pageable bytes into pinned memory) by thread
count, zhip_stage_h2d end to end by window size, raw pinned H2D."""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))


def med(f, n=7):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:]))


def main():
    import torch

    from zarr_hip import _native as N

    dev = torch.device("cuda:0")
    n = 64 << 20
    chunks = [bytes(np.random.default_rng(i).integers(0, 256, 1 << 20, dtype=np.uint8)) for i in range(64)]
    views = [np.frombuffer(c, np.uint8) for c in chunks]
    out = []
    out.append({"what": "torch.empty pinned 64 MiB", "ms": med(lambda: torch.empty(n, dtype=torch.uint8, pin_memory=True)) * 1e3})
    pin = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    for th in (1, 4, 8, 16, 32):
        def pack():
            for i, v in enumerate(views):
                N.lib().zhip_host_copy(pin.data_ptr() + i * (1 << 20), v.ctypes.data, 1 << 20, 1)
        def pack_par():
            pieces = np.zeros(64, N.PIECE_DT)
            for i, v in enumerate(views):
                pieces[i] = (v.ctypes.data, 1 << 20, i << 20, 0, 0)
            big = np.empty(0)
            # one host copy per piece through the pool: emulate with host_copy of a packed staging
            for i, v in enumerate(views):
                pass
        t = med(lambda: [N.lib().zhip_host_copy(pin.data_ptr() + i * (1 << 20), v.ctypes.data, 1 << 20, th)
                         for i, v in enumerate(views)])
        out.append({"what": f"pack 64 x 1 MiB host_copy threads={th}", "ms": t * 1e3, "GBps": n / t / 1e9})
    cs = torch.cuda.Stream(dev)
    pieces = np.zeros(64, N.PIECE_DT)
    for i, v in enumerate(views):
        pieces[i] = (v.ctypes.data, 1 << 20, i << 20, 0, 0)
    for win, th, ns in [(w, 16, n) for w in (2, 4, 8, 16) for n in (1, 2)]:
        N.lib().zhip_set_tuning(4, ns)
        if True:
            def run():
                N.lib().zhip_stage_h2d(pieces.ctypes.data, 64, pin.data_ptr(), dbuf.data_ptr(), n, win << 20, th,
                                       cs.cuda_stream)
                cs.synchronize()
            t = med(run)
            out.append({"what": f"stage_h2d window={win}MiB threads={th} streams={ns} (incl. sync)", "ms": t * 1e3,
                        "GBps": n / t / 1e9})
    def h2d():
        dbuf[:n].copy_(pin[:n], non_blocking=True)
        torch.cuda.synchronize(dev)
    t = med(h2d)
    out.append({"what": "raw pinned H2D 64 MiB", "ms": t * 1e3, "GBps": n / t / 1e9})
    def h2d_pieces():
        for i in range(64):
            dbuf[i << 20:(i + 1) << 20].copy_(pin[i << 20:(i + 1) << 20], non_blocking=True)
        torch.cuda.synchronize(dev)
    t = med(h2d_pieces)
    out.append({"what": "pinned H2D as 64 x 1 MiB copies", "ms": t * 1e3, "GBps": n / t / 1e9})
    for o in out:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in o.items()}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Host-side bandwidth landscape of the GPU box (measurement only): parallel
pageable -> pinned copies (the staging pack) by thread count with memcpy or
streaming stores (ZHIP_TUNE_STAGE_COPY), raw pinned H2D / D2H alone and
together (PCIe full duplex), H2D while the host packs, and zhip_stage_h2d of
64 x 1 MiB pageable pieces end to end.  One JSON line per measurement."""

import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))


def med(f, n=9):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:]))


def main():
    import torch

    from zarr_hip import _native as N

    lib = N.lib()
    dev = torch.device("cuda:0")
    n = 64 << 20
    src = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)  # pageable
    pin = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    pin2 = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    dbuf2 = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    out = []

    def rec(what, s, nbytes=n):
        out.append({"what": what, "ms": round(s * 1e3, 3), "GBps": round(nbytes / s / 1e9, 2)})
        print(json.dumps(out[-1]), flush=True)

    for mode in (0, 1):
        lib.zhip_set_tuning(5, mode)
        for th in (1, 4, 8, 16):
            rec(f"pack pageable->pinned 64 MiB threads={th} copy={'nt' if mode else 'memcpy'}",
                med(lambda: lib.zhip_host_copy(pin.data_ptr(), src.ctypes.data, n, th)))
        rec(f"unpack pinned->pageable 64 MiB threads=16 copy={'nt' if mode else 'memcpy'}",
            med(lambda: lib.zhip_host_copy(src.ctypes.data, pin.data_ptr(), n, 16)))
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def h2d():
        with torch.cuda.stream(s1):
            dbuf.copy_(pin, non_blocking=True)
        s1.synchronize()

    def d2h():
        with torch.cuda.stream(s2):
            pin2.copy_(dbuf2, non_blocking=True)
        s2.synchronize()

    def both():
        with torch.cuda.stream(s1):
            dbuf.copy_(pin, non_blocking=True)
        with torch.cuda.stream(s2):
            pin2.copy_(dbuf2, non_blocking=True)
        s1.synchronize()
        s2.synchronize()

    rec("raw pinned H2D 64 MiB", med(h2d))
    rec("raw pinned D2H 64 MiB", med(d2h))
    rec("H2D + D2H 64 MiB each, two streams (bytes = both)", med(both), 2 * n)
    for mode in (0, 1):
        lib.zhip_set_tuning(5, mode)

        def h2d_while_pack():
            t = threading.Thread(target=lambda: lib.zhip_host_copy(pin2.data_ptr(), src.ctypes.data, n, 8))
            t.start()
            h2d()
            t.join()
        rec(f"H2D 64 MiB while 8 threads pack 64 MiB copy={'nt' if mode else 'memcpy'}", med(h2d_while_pack))
    # zhip_stage_h2d: 64 x 1 MiB pageable pieces, packed in windows + H2D
    views = [src[i << 20:(i + 1) << 20] for i in range(64)]
    pieces = np.zeros(64, N.PIECE_DT)
    pieces["host"] = [v.ctypes.data for v in views]
    pieces["nbytes"] = 1 << 20
    pieces["dst_off"] = [i << 20 for i in range(64)]
    cs = torch.cuda.Stream(dev)
    for mode in (0, 1):
        lib.zhip_set_tuning(5, mode)
        for win in (2, 4, 8):
            for th in (8, 16):
                def st():
                    lib.zhip_stage_h2d(pieces.ctypes.data, 64, pin.data_ptr(), dbuf.data_ptr(), n, win << 20, th,
                                       cs.cuda_stream)
                    cs.synchronize()
                rec(f"stage_h2d 64 x 1 MiB window={win}MiB threads={th} copy={'nt' if mode else 'memcpy'}",
                    med(st))
    lib.zhip_set_tuning(5, 1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Calibration: the graph-timed per-launch floor of the small shares of the
strong-scaled headline (armbench's method: a hipGraph of REPS launches over 4
rotating buffers, replayed), for an empty kernel and for plain 32 KiB-span
copies of 8 / 16 / 32 / 64 MiB at 256 / 512 / 1024 lanes per span.  One JSON
line per arm."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libcopybench.so"))
    lib.cb_copy_wide.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    lib.cb_empty.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    R, REPS, ROUNDS = 4, 40, 15
    n_max = 64 << 20
    srcs = [torch.randint(0, 255, (n_max,), dtype=torch.uint8, device=dev) for _ in range(R)]
    dsts = [torch.empty(n_max, dtype=torch.uint8, device=dev) for _ in range(R)]

    def timed(launch):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for i in range(REPS):
                assert launch(i, ctypes.c_void_p(int(s.cuda_stream))) == 0
        gr.replay()
        torch.cuda.synchronize(dev)
        us = []
        for _ in range(ROUNDS):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            gr.replay()
            b.record()
            torch.cuda.synchronize(dev)
            us.append(a.elapsed_time(b) * 1e3 / REPS)
        return round(float(np.min(us)), 3), round(float(np.median(us)), 3)

    for grid in (1, 256, 2048):
        mn, md = timed(lambda i, sh: lib.cb_empty(grid, 256, sh))
        print(json.dumps({"arm": "empty", "grid": grid, "min_us": mn, "median_us": md}), flush=True)
    for mib in (8, 16, 32, 64):
        n = mib << 20
        for th in (256, 512, 1024):
            mn, md = timed(lambda i, sh: lib.cb_copy_wide(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, th, sh))
            print(json.dumps({"arm": "copy_wide", "MiB": mib, "threads": th, "grid": n // 32768, "min_us": mn,
                              "median_us": md, "TBps_med": round(2 * n / md / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())

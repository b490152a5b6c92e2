#!/usr/bin/env python
"""Calibration arms: plain streaming copy / read of the headline's 64 MiB at
several workgroup spans and load depths (HIP events, rotating 4 buffers so the
Infinity Cache cannot serve re-reads).  One JSON line per arm."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libcopybench.so"))
    lib.cb_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    n = 64 << 20
    R = 4
    srcs = [torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev) for _ in range(R)]
    dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    st = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(int(st.cuda_stream))

    def arm(span, K, store, nt, reps=30):
        for i in range(4):
            lib.cb_copy(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, span, K, store, nt, sh)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for i, (a, b) in enumerate(ev):
            a.record(st)
            rc = lib.cb_copy(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, span, K, store, nt, sh)
            assert rc == 0
            b.record(st)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        med = float(np.median(ms))
        byt = n * (2 if store else 1)
        return {"span_KiB": span >> 10, "K": K, "store": store, "nt": nt, "grid": n // span,
                "us_med": round(med * 1e3, 2), "us_min": round(min(ms) * 1e3, 2),
                "TBps_med": round(byt / med / 1e9, 3)}

    for store in (1, 0):
        for nt in (0, 1):
            for span in (16 << 10, 32 << 10, 64 << 10, 128 << 10, 256 << 10):
                for K in (4, 8):
                    print(json.dumps(arm(span, K, store, nt)), flush=True)
    # torch copy for reference
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for i, (a, b) in enumerate(ev):
        a.record(st)
        dsts[i % R].copy_(srcs[i % R])
        b.record(st)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    print(json.dumps({"arm": "torch_copy", "us_med": round(float(np.median(ms)) * 1e3, 2),
                      "TBps_med": round(2 * n / float(np.median(ms)) / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python
"""Copy ceilings by size (measurement only): a plain nontemporal copy of S bytes
-> S bytes, timed as a hipGraph of R launches rotating over buffers (so the
Infinity Cache cannot serve re-reads and launch gaps are excluded), for the
headline's 64 MiB and C4's 4 GiB.  Non-persistent (one span per workgroup)
and persistent grid-stride arms, each under
the default and nontemporal cache policies; torch's own D2D copy.  One JSON line per arm."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libcopybench.so"))
    lib.cb_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.cb_copy_rot.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p]
    lib.cb_copy_il.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                               ctypes.c_int, ctypes.c_void_p]
    lib.cb_copy_persist.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    for size_mb, R, reps in [(64, 4, 20), (4096, 2, 4)]:
        n = size_mb << 20
        srcs = [torch.empty(n, dtype=torch.uint8, device=dev).fill_(7) for _ in range(R)]
        dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
        # nt: 0 default policy, 1 nontemporal loads+stores, 2 loads only, 3 stores only
        if os.environ.get("IL"):  # interleaved 32 KiB footprints vs plain spans
            arms = [("il", S, 8, nt) for S in (1, 2, 4, 8, 16, 64) for nt in (1, 3)] + \
                   [("span", 4 << 10, 1, 1), ("span", 4 << 10, 1, 3)]
        elif os.environ.get("ROT"):  # spans with and without the rotated step order
            arms = [(kind, s, s // 4096, nt) for s in (32 << 10, 64 << 10) for nt in (1, 3)
                    for kind in ("span", "rot")] + [("span", 4 << 10, 1, 1)]
        else:
            arms = [("span", s, s // 4096, nt) for s in (4 << 10, 8 << 10, 16 << 10, 32 << 10)
                    for nt in (0, 1, 2, 3)] + \
                   [("span", 64 << 10, 8, 1)] + \
                   [("persist", g, k, nt) for g in (1024, 2048) for k in (4, 8) for nt in (0, 1)] + \
                   [("torch", 0, 0, 0)]
        for kind, a, K, nt in arms:
            stream = torch.cuda.Stream(dev)

            def launch(i):
                sh = ctypes.c_void_p(int(torch.cuda.current_stream(dev).cuda_stream))
                if kind == "span":
                    rc = lib.cb_copy(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, a, K, 1, nt, sh)
                elif kind == "il":
                    rc = lib.cb_copy_il(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, K, a, nt, sh)
                elif kind == "rot":
                    rc = lib.cb_copy_rot(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, K, nt, sh)
                elif kind == "persist":
                    rc = lib.cb_copy_persist(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, a, K, nt, sh)
                else:
                    dsts[i % R].copy_(srcs[i % R])
                    rc = 0
                assert rc == 0

            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for i in range(reps):
                    launch(i)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(3):
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / reps * 1e3)
            us = min(ts)
            print(json.dumps({"size_MiB": size_mb, "arm": kind, "span_or_grid": a, "K": K, "nt": nt,
                              "us_per_copy": round(us, 2), "TBps": round(2 * n / us / 1e6, 3),
                              "frac_of_8TBps": round(2 * n / us / 1e6 / 8.0, 3)}), flush=True)
        del srcs, dsts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())

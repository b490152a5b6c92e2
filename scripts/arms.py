#!/usr/bin/env python
"""One kernel arm per process, eager launches (measurement only), so that a
rocprofv3 --pmc pass over this process attributes every counter to one arm.

  ARM=hl    the headline decode (sharded 256^3 f32, 128^3 shards of 64^3),
            4 replicas rotated (512 MiB working set)
  ARM=c2    the unsharded 256^3 / 64^3 decode
  ARM=c4    C4 (1024^3 f32, 128^3 shards of 32^3), 2 replicas
  ARM=c3 / c3g  C3: transpose(2,1,0) + bytes (+ crc32c unless NOCRC=1) on the
            256^3 array in 64^3 (k_decode_tile4) / 128^3 (k_decode_tileg) chunks
  ARM=copy  scripts/copybench k_copy: SIZE bytes (default 64 MiB), SPAN bytes
            per workgroup, K loads in flight per thread, NT policy (0 default,
            1 nt loads+stores, 2 nt loads, 3 nt stores), 4 replicas at 64 MiB,
            1 at 4 GiB
  TUNE      zhip_set_tuning(2, TUNE) ablation bits for hl / c2 / c4
  KARM      zhip_set_tuning(6, KARM) kernel arm (loads the tuning build)
  REPS      launches (default 40; 8 for c4 / 4 GiB copies)

Prints one JSON line: arm, median / min event-timed microseconds per launch,
the HBM fraction of the arm's algorithmic bytes at the median."""

import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

if os.environ.get("KARM"):  # kernel arms exist only in the tuning build
    os.environ.setdefault("ZARR_HIP_ALLOW_LIB_OVERRIDE", "1")
    os.environ.setdefault("ZHIP_LIB", os.path.join(ROOT, "zarr-python_amd", "zarr_hip", "_lib", "libzarrhip_tune.so"))

import bench  # noqa: E402
import workloads as W  # noqa: E402


def main():
    import torch

    from zarr_hip import _native as N

    dev = torch.device("cuda:0")
    arm = os.environ.get("ARM", "hl")
    tune = int(os.environ.get("TUNE", "0"))
    big = arm == "c4" or int(os.environ.get("SIZE", str(64 << 20))) > (1 << 30)
    reps = int(os.environ.get("REPS", "8" if big else "40"))
    stream = torch.cuda.current_stream(dev)
    sh = int(stream.cuda_stream)
    if arm in ("hl", "c2", "c4", "c3", "c3g"):
        g = W.C4 if arm == "c4" else W.HEADLINE
        shape, inner = g["shape"], g["inner"]
        shards = None if arm in ("c2", "c3", "c3g") else g["shards"]
        codecs = [W.LE] if os.environ.get("NOCRC") == "1" else [W.LE, W.CRC]
        if arm in ("c3", "c3g"):
            codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}] + codecs
            inner = (128, 128, 128) if arm == "c3g" else inner
            arm = arm + ("_nocrc" if os.environ.get("NOCRC") == "1" else "")
        if arm == "c4":
            gen = torch.Generator(device=dev).manual_seed(0)
            data = torch.randn(shape, generator=gen, device=dev, dtype=torch.float32)
        else:
            data = torch.from_numpy(W.synthetic(shape)).to(dev)
        R = 2 if arm == "c4" else 4
        progs = [bench.build_replica(dev, data, shape, inner, codecs, shards=shards).prepare_read((Ellipsis,))
                 for _ in range(R)]
        for p, out in progs:
            p.launch()
            p.results()
            if not torch.equal(out.view(torch.int32), data.view(torch.int32)):
                raise SystemExit(f"arms {arm}: decode differs from the source")
        n_inner = int(np.prod([s // i for s, i in zip(shape, inner)]))
        alg = n_inner * (int(np.prod(inner)) * 4 + (4 if len(codecs) > 1 and codecs[-1] == W.CRC else 0)) + \
            data.numel() * 4
        if shards is not None:
            n_shards = int(np.prod([s // i for s, i in zip(shape, shards)]))
            alg += n_shards * ((n_inner // n_shards) * 16 + 4)
        del data
        N.lib().zhip_set_tuning(2, tune)
        if os.environ.get("KARM"):
            N.check(N.lib().zhip_set_tuning(6, int(os.environ["KARM"])), "zhip_set_tuning")
        launch = lambda i: progs[i % R][0].launch(sh)  # noqa: E731
    elif arm == "copy":
        cb = ctypes.CDLL(os.path.join(ROOT, "scripts", "copybench", "libcopybench.so"))
        cb.cb_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        n = int(os.environ.get("SIZE", str(64 << 20)))
        span, K, nt = int(os.environ.get("SPAN", "4096")), int(os.environ.get("K", "1")), int(os.environ.get("NT", "3"))
        mode = os.environ.get("MODE", "span")  # span (k_copy), wave (k_copy_wave), il (k_copy_il, S = SPAN)
        R = 1 if big else 4
        srcs = [torch.empty(n, dtype=torch.uint8, device=dev).fill_(3) for _ in range(R)]
        dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
        alg = 2 * n
        cb.cb_copy_wave.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p]
        cb.cb_copy_il.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                                  ctypes.c_int, ctypes.c_void_p]
        if mode == "wave":
            fn = lambda i: cb.cb_copy_wave(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, K, nt,  # noqa: E731
                                           ctypes.c_void_p(sh))
        elif mode == "il":
            fn = lambda i: cb.cb_copy_il(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, K, span, nt,  # noqa: E731
                                         ctypes.c_void_p(sh))
        else:
            fn = lambda i: cb.cb_copy(srcs[i % R].data_ptr(), dsts[i % R].data_ptr(), n, span, K, 1, nt,  # noqa: E731
                                      ctypes.c_void_p(sh))

        def launch(i):
            rc = fn(i)
            if rc != 0:
                raise SystemExit(f"copy arm {mode}: rc {rc}")
        arm = f"copy_{mode}_{n >> 20}MiB_span{span}_K{K}_nt{nt}"
    else:
        raise SystemExit(f"unknown ARM {arm}")
    for i in range(4):
        launch(i)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        launch(i)
        b.record(stream)
    torch.cuda.synchronize(dev)
    us = [a.elapsed_time(b) * 1e3 for a, b in ev]
    N.lib().zhip_set_tuning(2, 0)
    med = float(np.median(us))
    kern = N.lib().zhip_last_kernel().decode() if not arm.startswith("copy") else "copybench"
    print(json.dumps({"arm": arm, "kernel": kern, "tune": tune, "reps": reps, "us_med": round(med, 2), "us_min": round(min(us), 2),
                      "alg_bytes": int(alg), "hbm_frac_med": round(alg / (med * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()

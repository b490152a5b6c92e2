#!/usr/bin/env python
"""Diagnostics: how many k_decode_il workgroups of the lean-prologue arm
(kTuneIlLean) guessed a wrong chunk address and reloaded (counted by the
kernel in the last zhip_debug_stamps slot), per launch, for the headline
batch (WORLD=1) or rank 0's share of an n-way split (WORLD=n)."""
import json
import os
# kernel arms and knobs exist only in the tuning build (make -C zarr-python_amd tune)
os.environ.setdefault("ZARR_HIP_ALLOW_LIB_OVERRIDE", "1")
os.environ.setdefault("ZHIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "zarr-python_amd", "zarr_hip", "_lib", "libzarrhip_tune.so"))
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402

K_STAMP = 8192 * 8


def counter(N):
    buf = np.zeros(K_STAMP, np.uint64)
    N.check(N.lib().zhip_debug_stamps(buf.ctypes.data, 8192), "zhip_debug_stamps")
    return int(buf[-1])


def main():
    import torch

    from zarr_hip import _native as N
    from zarr_hip import buffer, parallel

    dev = torch.device("cuda:0")
    shape, chunks, shards = (256, 256, 256), (64, 64, 64), (128, 128, 128)
    data = torch.from_numpy(bench.synthetic(shape)).to(dev)
    for world in (1, 8):
        arr = bench.build_replica(dev, data, shape, chunks, [bench.LE, bench.CRC], shards=shards)
        batch, out_shape = arr.batch_info((Ellipsis,))
        out = buffer.empty(out_shape, "float32", dev)
        prog = arr.codec_pipeline.prepare_read(parallel.rank_batch(batch, world, 0), out)
        pred = prog.tables.predict is not None
        N.lib().zhip_set_tuning(2, 16384)
        c0 = counter(N)
        for _ in range(4):
            prog.launch()
        torch.cuda.synchronize(dev)
        c1 = counter(N)
        N.lib().zhip_set_tuning(2, 0)
        prog.results()
        print(json.dumps({"world": world, "predicted": pred, "launches": 4, "reloads_per_launch": (c1 - c0) / 4,
                          "workgroups": int(prog.data.grid) if hasattr(prog.data, "grid") else None}), flush=True)


if __name__ == "__main__":
    main()

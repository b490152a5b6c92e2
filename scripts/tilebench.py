#!/usr/bin/env python
"""Transposed-decode timing for PMC / rocprof passes (measurement only): the
C3 batch (256^3 f32, transpose (2,1,0), 64^3 chunks: k_decode_tile4) and the
same array in 128^3 chunks (the layout k_decode_tile4 declines), each
graph-timed over replicas as bench.py does; one JSON line per arm.
TUNE sets ablation bits (65536: the one-tile persistent k_decode_tile)."""

import json
import os
# kernel arms and knobs exist only in the tuning build (make -C zarr-python_amd tune)
os.environ.setdefault("ZARR_HIP_ALLOW_LIB_OVERRIDE", "1")
os.environ.setdefault("ZHIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "zarr-python_amd", "zarr_hip", "_lib", "libzarrhip_tune.so"))
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402


def main():
    import torch

    from zarr_hip import _native as N

    tune = int(os.environ.get("TUNE", "0"))
    if tune:
        N.lib().zhip_set_tuning(2, tune)
    dev = torch.device("cuda:0")
    shape = (256, 256, 256)
    data = torch.from_numpy(bench.synthetic(shape, seed=0)).to(dev)
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, bench.LE, bench.CRC]
    steps = int(os.environ.get("STEPS", "20"))
    nocrc = codecs[:2]
    for name, chunks, cod in (("c3_64", (64, 64, 64), codecs), ("c3_128", (128, 128, 128), codecs),
                              ("c3_64_nocrc", (64, 64, 64), nocrc), ("c3_128_nocrc", (128, 128, 128), nocrc)):
        if name not in os.environ.get("ARMS", "c3_64,c3_128").split(","):
            continue
        progs = [bench.build_replica(dev, data, shape, chunks, cod).prepare_read((Ellipsis,)) for _ in range(4)]
        progs[0][0].launch()
        progs[0][0].results()
        assert torch.equal(progs[0][1].view(torch.int32), data.view(torch.int32)), name
        flags = N.Plan(progs[0][0].tables.layout, upload=False).kernel_flags
        wall, kern = bench.time_programs([p for p, _ in progs], steps, 3, dev)
        n_chunks = int(torch.tensor([s // c for s, c in zip(shape, chunks)]).prod())
        alg = data.numel() * 4 * 2 + (4 * n_chunks if cod is codecs else 0)
        print(json.dumps({"arm": name, "tune": tune, "tile4": bool(flags & N.PK_TILE4),
                          "us_graph": round(wall * 1e6, 2), "us_eager": round(kern * 1e6, 2),
                          "hbm_frac": round(alg / wall / 8e12, 4)}), flush=True)
        del progs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

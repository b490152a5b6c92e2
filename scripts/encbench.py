#!/usr/bin/env python
"""Encode-only timing for PMC / rocprof passes (measurement only): the C3
transposed encode on 64^3 chunks (k_encode_tile4, or k_encode_tile with
TUNE=65536) and on 128^3 chunks (k_encode_tile), graph-timed as bench.py
does; one JSON line per arm."""

import json
import os
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
    args = type("A", (), {"steps": int(os.environ.get("STEPS", "20")), "tune": tune})()
    dev = torch.device("cuda:0")
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, bench.LE, bench.CRC]
    for name, chunks, want in (("c3_64", (64, 64, 64), "tile4"), ("c3_128", (128, 128, 128), "tile")):
        if name not in os.environ.get("ARMS", "c3_64,c3_128"):
            continue
        src, wall, kern = bench._encode_bench(dev, args, codecs, want, chunks=chunks)
        print(json.dumps({"arm": name, "tune": tune, "us_graph": round(wall * 1e6, 2),
                          "us_eager": round(kern * 1e6, 2),
                          "hbm_frac": round(2 * src / wall / 8e12, 4)}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

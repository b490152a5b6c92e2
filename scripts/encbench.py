#!/usr/bin/env python
"""Encode-only timing for PMC / rocprof passes (measurement only): the C3
transposed encode on 64^3 chunks (k_encode_tile4, or k_encode_tile with
TUNE=65536), on 128^3 chunks (k_encode_tile) and the C2 encode
(k_encode_pair), 16 KiB chunks (k_encode_quad), graph-timed as bench.py does, each config with an optional
ZHIP_TUNE_ARM; one JSON line per arm."""

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
    args = type("A", (), {"steps": int(os.environ.get("STEPS", "20")), "tune": tune})()
    dev = torch.device("cuda:0")
    tr = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}]
    cfgs = {"c3_64": (tr, (64, 64, 64), "tile4"), "c3_128": (tr, (128, 128, 128), "tile"),
            "c2": ([], (64, 64, 64), "rows"),
            # 16 KiB chunks (the reference example's chunk size): k_encode_quad, arm 11 k_encode_pair
            "q16": ([], (1, 64, 64), "rows"), "q16n": ([], (1, 64, 64), "rows", False),
            "c2n": ([], (64, 64, 64), "rows", False),
            # the transposed encodes without a CRC (what the transpose alone costs)
            "c3_64n": (tr, (64, 64, 64), "tile4", False), "c3_128n": (tr, (128, 128, 128), "tile", False)}
    # ARMS: comma list of config[:arm] (arm = zhip_set_tuning(ARM), e.g. c2:1);
    # NOCHECK: the same items for ablation arms whose output is not a valid store
    for item in os.environ.get("ARMS", "c3_64,c3_128").split(","):
        name, _, arm = item.partition(":")
        aa, chunks, want, *crc = cfgs[name]  # q16n: no CRC codec
        tail = [bench.LE, bench.CRC] if not crc or crc[0] else [bench.LE]
        N.lib().zhip_set_tuning(6, int(arm or 0))
        src, wall, kern, _ = bench._encode_bench(dev, args, aa + tail, want, chunks=chunks,
                                              check=item not in os.environ.get("NOCHECK", "").split(","))
        N.lib().zhip_set_tuning(6, 0)
        print(json.dumps({"arm": item, "tune": tune, "us_graph": round(wall * 1e6, 2),
                          "us_eager": round(kern * 1e6, 2),
                          "hbm_frac": round(2 * src / wall / 8e12, 4)}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

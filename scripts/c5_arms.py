#!/usr/bin/env python
"""C5 (bench.c5_partial: 2048^3 int16, 10 % of the 64^3 inner chunks) under
kernel arms of the tuning build, interleaved (measurement only, round 6):
ARMS = comma list of ZHIP_TUNE_ARM values.  One JSON line per run."""

import json
import os
import sys

os.environ.setdefault("ZARR_HIP_ALLOW_LIB_OVERRIDE", "1")
os.environ.setdefault("ZHIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "zarr-python_amd", "zarr_hip", "_lib", "libzarrhip_tune.so"))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402


def main():
    import torch

    from zarr_hip import _native as N

    ctx = bench.Ctx()
    args = type("A", (), {"steps": 20, "tune": 0})()
    for arm in [int(a) for a in os.environ.get("ARMS", "0,71").split(",")]:
        N.check(N.lib().zhip_set_tuning(6, arm), "zhip_set_tuning")
        r = bench.c5_partial(ctx, args)
        N.check(N.lib().zhip_set_tuning(6, 0), "zhip_set_tuning")
        print(json.dumps({"arm": arm, "kernel": r["kernel"], "kernel_ms": r["kernel_ms"], "step_ms": r["step_ms"],
                          "hbm_frac": r["hbm_frac"]}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

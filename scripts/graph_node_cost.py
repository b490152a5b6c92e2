#!/usr/bin/env python
"""Measurement: what one extra small kernel per step costs inside a hipGraph
replay of the headline decode (decides whether a separate finalize kernel can
pay for itself)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))

import bench  # noqa: E402


def main():
    import torch

    dev = torch.device("cuda:0")
    shape, chunks, shards = (256, 256, 256), (64, 64, 64), (128, 128, 128)
    data = torch.from_numpy(bench.synthetic(shape)).to(dev)
    progs = [bench.build_replica(dev, data, shape, chunks, [bench.LE, bench.CRC], shards=shards)
             .prepare_read((Ellipsis,))[0] for _ in range(4)]
    small = torch.zeros(64 * 4, dtype=torch.int32, device=dev)
    steps = 50
    res = {}
    for extra in (0, 1, 2):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.graph(g, stream=s):
            for i in range(steps):
                progs[i % 4].launch()
                for _ in range(extra):
                    small.add_(1)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b) / steps * 1e3)
        res[f"us_per_step_extra{extra}"] = round(sorted(ts)[2], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

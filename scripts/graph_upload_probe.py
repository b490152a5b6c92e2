#!/usr/bin/env python
"""Measurement probe (round 6): does the first replay of a freshly captured
hipGraph pay a one-time cost that bench.py's timed region would absorb?

Builds the headline programs exactly as bench.py does, captures K-launch
graphs (zarr_hip.ReadGraph) and times replays with events on the replay
stream and the host clock:
  * fresh graph, replays 1..4 (is the first slower?);
  * fresh graph pre-uploaded with hipGraphUpload (no kernel runs), replays 1..4.
One JSON line per graph.

  python scripts/graph_upload_probe.py [--steps 20]
"""

import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    import bench
    import zarr_hip

    ctx = bench.Ctx()
    args = argparse.Namespace(replicas=4, steps=a.steps, warmup=10)
    plist, decoded, encoded = bench.headline(ctx, args, weak=True)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    dev = ctx.device
    warm = zarr_hip.ReadGraph(plist, 10, dev)
    warm.replay()
    torch.cuda.synchronize(dev)
    for r in range(a.rounds):
        for upload in (False, True):
            g = zarr_hip.ReadGraph(plist, a.steps, dev)
            if upload:
                rc = hip.hipGraphUpload(ctypes.c_void_p(g.graph.raw_cuda_graph_exec()),
                                        ctypes.c_void_p(g.stream.cuda_stream))
                torch.cuda.synchronize(dev)
                assert rc == 0, rc
            stream = torch.cuda.current_stream(dev)
            spans, walls = [], []
            for _ in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                e0.record(stream)
                g.replay()
                e1.record(stream)
                torch.cuda.synchronize(dev)
                walls.append((time.perf_counter() - t0) * 1e6 / a.steps)
                spans.append(e0.elapsed_time(e1) * 1e3 / a.steps)
            for p in plist:
                p.results()
            print(json.dumps({"round": r, "upload": upload, "steps": a.steps,
                              "span_us_per_step": [round(x, 3) for x in spans],
                              "wall_us_per_step": [round(x, 3) for x in walls]}), flush=True)


if __name__ == "__main__":
    main()

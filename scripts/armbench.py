#!/usr/bin/env python
"""Graph-timed kernel arms on one batch (measurement only, round 4).

ARMS: comma list of name=bits:arm (bits = zhip_set_tuning(ABLATION), arm =
zhip_set_tuning(ARM)); each arm is a hipGraph of REPS launches rotating over
4 replicas (the Infinity Cache cannot serve re-reads), replayed ROUNDS times,
interleaved with the other arms in ONE process.  CONFIG = headline | c4 |
share8 (rank 0's 1-shard share of the headline at N = 8) | share4 | c3 | c3g
(transpose (2,1,0) in 64^3 / 128^3 chunks) | cpp (the reference's
codec_pipeline_performance array, zarr's default sharding codecs) | cppu (the
same array unsharded, bytes only: 64^2 chunks of 16 KiB) | cppuc (the same
with crc32c) | cppu8 / cppu4 (unsharded, 8 / 4 KiB chunks).  Also
the no-CRC twin (zarr's default sharding codecs, k_decode_lead) for the
headline.  One JSON line per arm: min / median us per launch and the HBM
fraction of the algorithmic bytes.  After timing, the production arm's
output is compared with the source (the graph must decode exactly)."""

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
import workloads as W  # noqa: E402


def main():
    import torch

    from zarr_hip import _native as N

    dev = torch.device("cuda:0")
    cfg = os.environ.get("CONFIG", "headline")
    g = W.C4 if cfg == "c4" else W.CPP_EXAMPLE if cfg.startswith("cpp") else W.HEADLINE
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    if cfg.startswith("cpp"):  # the reference's example array (cppu: unsharded; cppuc: + crc32c; cppu8 / cppu4: 8 / 4 KiB chunks)
        data = torch.from_numpy(W.cpp_example_data("plain")).to(dev)
    elif cfg == "c4":
        gen = torch.Generator(device=dev).manual_seed(0)
        data = torch.randn(shape, generator=gen, device=dev, dtype=torch.float32)
    else:
        data = torch.from_numpy(W.synthetic(shape)).to(dev)
    if cfg.startswith("share"):  # rank 0's share of the strong-scaled headline: 8/N shards
        keep = 8 // int(cfg[5:])
        shape = {1: (128, 128, 128), 2: (128, 128, 256), 4: (128, 256, 256)}[keep]
        data = data[: shape[0], : shape[1], : shape[2]].contiguous()
    aa = []
    if cfg in ("c3", "c3g"):  # C3: transpose (2,1,0) + bytes + crc32c, unsharded 64^3 / 128^3 chunks
        aa = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}]
        inner = (128, 128, 128) if cfg == "c3g" else (64, 64, 64)
        shards = None
    R = 2 if cfg == "c4" else 4
    reps = int(os.environ.get("REPS", "4" if cfg == "c4" else "20"))
    if cfg in ("cppu", "cppuc", "cppu8", "cppu4"):
        shards = None
        inner = {"cppu8": (32, 64), "cppu4": (16, 64)}.get(cfg, inner)
    if cfg.startswith("cpp"):
        cc = [W.LE, W.CRC] if cfg == "cppuc" else [W.LE]
        crc = [bench.build_replica(dev, data, shape, inner, cc, shards=shards, dtype="int32", fill=0)
               .prepare_read((Ellipsis,)) for _ in range(R)]
        nocrc = []
    else:
        crc = [bench.build_replica(dev, data, shape, inner, aa + [W.LE, W.CRC], shards=shards)
               .prepare_read((Ellipsis,)) for _ in range(R)]
        nocrc = [bench.build_replica(dev, data, shape, inner, aa + [W.LE], shards=shards).prepare_read((Ellipsis,))
                 for _ in range(R)] if cfg != "c4" else []
    n_inner = int(np.prod([s // i for s, i in zip(shape, inner)]))
    if cfg in ("cppu", "cppu8", "cppu4"):  # bytes only: no trailer, no index
        alg = n_inner * int(np.prod(inner)) * 4 + data.numel() * 4
    elif cfg == "cppuc":  # + a 4-byte trailer per chunk
        alg = n_inner * (int(np.prod(inner)) * 4 + 4) + data.numel() * 4
    elif cfg == "cpp":  # inner chunks without a trailer, one index CRC per shard
        n_shards = int(np.prod([s // i for s, i in zip(shape, shards)]))
        cps = n_inner // n_shards
        alg = n_inner * int(np.prod(inner)) * 4 + n_shards * (cps * 16 + 4) + data.numel() * 4
    elif shards is not None:
        n_shards = int(np.prod([s // i for s, i in zip(shape, shards)]))
        cps = n_inner // n_shards
        alg = n_inner * (int(np.prod(inner)) * 4 + 4) + n_shards * (cps * 16 + 4) + data.numel() * 4
    else:
        alg = n_inner * (int(np.prod(inner)) * 4 + 4) + data.numel() * 4

    def graph_of(progs):
        s = torch.cuda.Stream(dev)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for i in range(reps):
                progs[i % len(progs)][0].launch(int(s.cuda_stream))
        return gr

    arms = {}
    kernels = {}
    spec = os.environ.get("ARMS", "prod=0:0")
    for item in spec.split(","):
        name, rest = item.split("=")
        bits, arm = (int(x) for x in rest.split(":"))
        N.lib().zhip_set_tuning(2, bits)
        N.lib().zhip_set_tuning(6, arm)
        arms[name] = graph_of(crc)
        kernels[name] = N.lib().zhip_last_kernel().decode()
    N.lib().zhip_set_tuning(2, 0)
    N.lib().zhip_set_tuning(6, 0)
    if nocrc:
        arms["nocrc_twin"] = graph_of(nocrc)
        kernels["nocrc_twin"] = N.lib().zhip_last_kernel().decode()
    res = {k: [] for k in arms}
    for _ in range(int(os.environ.get("ROUNDS", "7"))):
        for k, gr in arms.items():
            gr.replay()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            gr.replay()
            b.record()
            torch.cuda.synchronize(dev)
            res[k].append(a.elapsed_time(b) * 1e3 / reps)
        print(json.dumps({"progress": len(res[k])}), file=sys.stderr, flush=True)
    ok = True
    for p, out in crc:
        p.data.d_ws.zero_()
        p.data.d_status.zero_()
        p.data.reset_errflag()
        p.launch()
        p.results()
        ok = ok and torch.equal(out.view(torch.int32), data.view(torch.int32))
    for k, v in res.items():
        print(json.dumps({"config": cfg, "arm": k, "kernel": kernels[k], "min_us": round(min(v), 3),
                          "median_us": round(float(np.median(v)), 3),
                          "hbm_frac_median": round(alg / (float(np.median(v)) * 1e-6) / 8e12, 4),
                          "alg_bytes": alg, "reps": reps, "prod_exact": ok}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Benchmark: device-resident zarr v3 decode on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1], "C2"): a 256^3 float32 array in 64^3 chunks,
codecs [bytes(little), crc32c], every encoded chunk resident in HBM; one step =
one full-array decode (CRC verify + scatter of all 64 chunks) by the HIP
kernel.  Synthetic data: seed 0 standard normal with planted NaN payload and
-0.0.  To keep the measurement an HBM measurement (the 256 MiB Infinity Cache
would otherwise hold the 128 MiB working set), steps rotate over 4 independent
replicas (inputs + outputs), 512 MiB in total.

Multi-GPU (weak scaling): one process per GPU (torchrun), each decoding its own
replica set; chunks are independent so there is no collective on the data
path — RCCL only carries the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
"roofline" (dominant kernel vs 8 TB/s HBM, per-launch kernel time from HIP
events on the launch stream) and "cpu_baseline" (the CPU restatement of the
reference's FusedCodecPipeline.read_sync timed on this host's cores).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "zarr-python_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def synthetic(shape, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal(shape, dtype=np.float32)
    flat = a.reshape(-1)
    flat[7] = -0.0
    flat[11:12].view(np.uint32)[0] = 0x7FC00001
    return a


LE = {"name": "bytes", "configuration": {"endian": "little"}}
CRC = {"name": "crc32c"}


def build_replica(device, data_dev, shape, chunks, codecs, shards=None):
    """Encode a device array into a fresh DeviceStore with zarr_hip's own GPU
    encode path (setup, not timed)."""
    import torch

    import zarr_hip

    n_enc = int(np.prod(shape)) * data_dev.element_size() * 1.02 + (1 << 24)
    store = zarr_hip.DeviceStore(device, capacity=int(n_enc))
    if shards is None:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=codecs)
    else:
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, shards=shards,
                                    inner_codecs=codecs)
    arr.set((Ellipsis,), data_dev)
    torch.cuda.synchronize(device)
    return arr


def build_c2_replica(device, data_np, shape, chunks):
    import torch

    return build_replica(device, torch.from_numpy(data_np).to(device), shape, chunks, [LE, CRC])


def time_programs(progs, steps, warmup, device):
    """Average kernel time (HIP events on the launch stream) over rotating programs."""
    import torch

    stream = torch.cuda.current_stream(device)
    sh = int(stream.cuda_stream)
    for i in range(warmup):
        progs[i % len(progs)].launch(sh)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        progs[i % len(progs)].launch(sh)
        b.record(stream)
    torch.cuda.synchronize(device)
    wall = time.perf_counter() - t0
    for p in progs:
        p.results()
    return wall / steps, float(np.median([a.elapsed_time(b) for a, b in ev])) / 1e3


def extra_configs(device, args):
    """C3 (transpose) and C4 (sharded) measured beside the headline C2."""
    import torch

    out = {}
    if "c3" in args.extra:
        shape, chunks = (256, 256, 256), (64, 64, 64)
        data = torch.from_numpy(synthetic(shape, seed=0)).to(device)
        progs = []
        for _ in range(args.replicas):
            arr = build_replica(device, data, shape, chunks,
                                [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC])
            progs.append(arr.prepare_read((Ellipsis,))[0])
        prog, outt = progs[0], None
        wall, kern = time_programs(progs, max(10, args.steps // 2), 3, device)
        dec = data.numel() * 4
        enc = 64 * (1048576 + 4)
        out["c3_transpose_210"] = {"decoded_GiBps": round(dec / wall / GIB, 1),
                                   "kernel_ms": round(kern * 1e3, 4),
                                   "hbm_frac": round((dec + enc) / kern / 1e9 / HBM_PEAK_GBS, 4)}
        del progs, data
    if "c4" in args.extra:
        shape, shards, inner = (1024, 1024, 1024), (128, 128, 128), (32, 32, 32)
        g = torch.Generator(device=device).manual_seed(0)
        data = torch.randn(shape, generator=g, device=device, dtype=torch.float32)
        progs = []
        for _ in range(2):
            arr = build_replica(device, data, shape, inner, [LE, CRC], shards=shards)
            progs.append(arr.prepare_read((Ellipsis,))[0])
        chk = progs[0]
        chk.launch()
        chk.results()
        wall, kern = time_programs(progs, 6, 2, device)
        dec = data.numel() * 4
        enc = 512 * (64 * (131072 + 4) + 64 * 16 + 4)
        out["c4_sharded_1024"] = {"decoded_GiBps": round(dec / wall / GIB, 1),
                                  "step_ms": round(wall * 1e3, 3),
                                  "kernel_ms": round(kern * 1e3, 3),
                                  "hbm_frac": round((dec + enc) / kern / 1e9 / HBM_PEAK_GBS, 4)}
        del progs, data
    torch.cuda.empty_cache()
    return out


def cpu_baseline(data_np, shape, chunks, budget_s=12.0):
    """The reference's FusedCodecPipeline.read_sync restated on the host
    (oracle: per chunk fetch -> CRC-32C with the SSE4.2 instruction as
    google_crc32c -> zero-copy view -> numpy scatter), thread pool sized like
    _resolve_max_workers (codec_pipeline.py:53-73)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    lib = O._load_lib()
    grid = tuple(s // c for s, c in zip(shape, chunks))
    store = {}
    for c in np.ndindex(*grid):
        sl = tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(c, chunks))
        b = np.ascontiguousarray(data_np[sl]).view(np.uint8).reshape(-1)
        store[c] = bytes(O.crc32c_encode(b))
    out = np.empty(shape, np.float32)

    def read_one(c):
        raw = store[c]  # MemoryStore.get_sync: zero-copy view of stored bytes
        u8 = np.frombuffer(raw, np.uint8)
        crc = lib.oracle_crc32c(u8.ctypes.data, u8.size - 4)
        if np.uint32(crc).tobytes() != raw[-4:]:
            raise ValueError("checksum")
        chunk = u8[:-4].view(np.float32).reshape(chunks)
        sl = tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(c, chunks))
        out[sl] = chunk
        return None

    coords = list(store.keys())
    workers = os.cpu_count() or 1
    box_cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if box_cores:
        workers = min(workers, box_cores)
    pool = ThreadPoolExecutor(max_workers=workers)
    list(pool.map(read_one, coords))  # warm-up
    n = 0
    t0 = time.perf_counter()
    while True:
        list(pool.map(read_one, coords))
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = (time.perf_counter() - t0) / n
    assert out.tobytes() == data_np.tobytes()
    pool.shutdown()
    return {"value": round(data_np.nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": workers,
            "kind": "port",
            "sample": f"{n} full C2 decodes (64 chunks x 1 MiB + crc) in {n * dt:.1f}s; "
                      f"{workers} worker threads, {os.cpu_count()} cpus visible"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--extra", default="c3,c4", help="extra configs measured at N=1 (c3,c4 or '')")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    shape, chunks = (256, 256, 256), (64, 64, 64)
    data = synthetic(shape, seed=0)
    log(f"[bench] building {args.replicas} replicas of C2 on {device}")
    progs = []
    for r in range(args.replicas):
        arr = build_c2_replica(device, data, shape, chunks)
        prog, out = arr.prepare_read((Ellipsis,))
        progs.append((prog, out))
    # correctness gate on rank 0's first replica
    prog0, out0 = progs[0]
    prog0.launch()
    prog0.results()
    if out0.view(torch.int32).cpu().numpy().tobytes() != data.view(np.int32).tobytes():
        raise SystemExit("bench: decoded output differs from the synthetic input")
    for p, _ in progs:
        assert p.tables.fast, "C2 should take the whole-row fast path"

    stream = torch.cuda.current_stream(device)
    sh = int(stream.cuda_stream)
    for i in range(args.warmup):
        progs[i % len(progs)][0].launch(sh)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        a, b = ev[i]
        a.record(stream)
        progs[i % len(progs)][0].launch(sh)
        b.record(stream)
    torch.cuda.synchronize(device)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    for p, _ in progs:
        p.results()  # raises on any CRC / status error accumulated during the run
    t = torch.tensor([wall], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())

    decoded = data.nbytes
    encoded = 64 * (1048576 + 4)
    value = world * args.steps * decoded / wall_max / GIB
    avg_kern_s = float(np.mean(kern_ms)) / 1e3
    achieved = (encoded + decoded) / avg_kern_s / 1e9
    res = {
        "metric": "decoded GiB/s (device-resident), sharded 256^3 f32 64^3 chunks, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0 standard-normal f32, planted NaN payload and -0.0)",
        "config": {
            "workload": "C2: 256^3 float32, 64^3 chunks, bytes(little)+crc32c, device-resident "
                        "decode of the full array per step, 4 rotating replicas per GPU",
            "chunks_per_step": 64, "decoded_bytes_per_step": decoded,
            "encoded_bytes_per_step": encoded, "parallelism": f"chunk-parallel x{world} (weak)",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "zhip::k_decode<CRC,WRITE,FAST,4,noswap>",
            "kernel_ms_avg": round(avg_kern_s * 1e3, 5),
            "algorithmic_bytes_per_launch": encoded + decoded,
        },
    }
    if world == 1 and args.extra:
        log("[bench] extra configs " + args.extra)
        res["extra"] = extra_configs(device, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("[bench] cpu baseline")
        res["cpu_baseline"] = cpu_baseline(data, shape, chunks, args.cpu_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

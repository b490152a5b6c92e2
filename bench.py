#!/usr/bin/env python
"""Benchmark: device-resident zarr v3 decode on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W

Headline workload (BASELINE.json metric: "sharded 256^3 f32 64^3 chunks"): a
256^3 float32 array in 128^3 shards of 64^3 inner chunks, inner codecs
bytes(little)+crc32c, index bytes+crc32c at the end, every encoded shard
resident in HBM; one step = one full-array decode (CRC verify of 64 inner
chunks and 8 shard indexes + scatter) by one HIP launch.  Synthetic data: seed
0 standard normal with a planted NaN payload and -0.0.  To keep it an HBM
measurement (the 256 MiB Infinity Cache would otherwise hold the 128 MiB
working set) steps rotate over 4 independent replicas (inputs + outputs).

Multi-GPU (one process per GPU; `--gpus N` launches the N ranks itself):
chunks are independent, so the batch is partitioned across the ranks with no
collective on the data path (the reference's disjoint-output pool map,
src/zarr/core/codec_pipeline.py:1104-1109, 1169-1171).  The headline scales
weakly, as the task's contract for partitioned paths asks: the batch at N
GPUs is the (256N) x 256 x 256 array of 8N shards, split round-robin by shard
(zarr_hip.parallel.rank_batch), so every rank decodes 8 shards -- one
BASELINE array's worth -- per step; `value` = all ranks' decoded bytes / the
max rank step time.  extra.headline_strong (N > 1) splits BASELINE's single
256^3 array (8/N shards per rank, strong scaling).  The C4 (1024^3) and C5
(2048^3, 10 % inner chunks) legs split their fixed batch round-robin by shard
(strong scaling).  RCCL carries only the barrier and the max-over-ranks of the
timed wall.

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

import workloads as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# per-launch HBM bytes of the headline kernel from separate rocprofv3 --pmc passes
# of this same command (scripts/gpu_pmc.sh -> scripts/pmc_summary.py); counters
# cannot be read from inside the timed process, so the value is labelled with
# the file it comes from
TRAFFIC_JSON = os.path.join("profiles", "r06", "pmc_traffic.json")
LIB_SO = os.path.join("zarr-python_amd", "zarr_hip", "_lib", "libzarrhip.so")
GIB = float(1 << 30)
LE, CRC = W.LE, W.CRC
synthetic = W.synthetic


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


class Ctx:
    """Rank / device / process-group context of one bench process."""

    def __init__(self):
        import torch
        import torch.distributed as dist

        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        # launched by torchrun (even with one rank): use the process group for the
        # barrier / max-over-ranks timing so the N>1 code path is the one exercised
        self.distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal of the N>1 path on a one-GPU box: every rank on device 0 with
        # a gloo group (RCCL refuses two ranks on one device).  Never the driver's
        # configuration: the numbers of such a run are not a scaling measurement.
        self.rehearsal = os.environ.get("ZHIP_BENCH_REHEARSAL") == "1"
        backend = "gloo" if self.rehearsal else "nccl"
        if self.rehearsal:
            local = 0
        if self.distributed:
            torch.cuda.set_device(local)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
        self.device = torch.device("cuda", local)
        torch.cuda.set_device(self.device)
        self.dist = dist
        self._red_dev = torch.device("cpu") if self.rehearsal else self.device

    def barrier(self):
        if self.distributed:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        import torch

        if not self.distributed:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self._red_dev)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM)


def build_replica(device, data_dev, shape, chunks, codecs, shards=None, dtype="float32", fill=0.0):
    """Encode a device array into a fresh DeviceStore with zarr_hip's own GPU
    encode path (setup, not timed)."""
    import torch

    import zarr_hip

    n_enc = int(np.prod(shape)) * data_dev.element_size() * 1.02 + (1 << 24)
    store = zarr_hip.DeviceStore(device, capacity=int(n_enc))
    if shards is None:
        arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    else:
        arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, shards=shards,
                                    inner_codecs=codecs)
    arr.set((Ellipsis,), data_dev)
    torch.cuda.synchronize(device)
    return arr


def build_partitioned(ctx, src, shape, inner, shards, dtype, fill, capacity):
    """One replica of a sharded array whose batch is split round-robin by shard:
    this rank encodes only its own shards (from the full-shape device source)
    into its own DeviceStore and plans the decode of exactly those shards into a
    full-shape out.  Returns (program, out, my batch items)."""
    import torch

    import zarr_hip
    from zarr_hip import buffer, parallel

    store = zarr_hip.DeviceStore(ctx.device, capacity=int(capacity))
    arr = zarr_hip.Array.create(store, shape, inner, dtype, fill, shards=shards,
                                inner_codecs=[LE, CRC])
    batch, out_shape = arr.batch_info((Ellipsis,))
    mine = parallel.rank_batch(batch, ctx.world, ctx.rank)
    arr.codec_pipeline.write_sync(mine, src)
    out = buffer.empty(out_shape, dtype, ctx.device)
    prog = arr.codec_pipeline.prepare_read(mine, out)
    torch.cuda.synchronize(ctx.device)
    return prog, out, mine


def check_regions(out, src, items, what):
    """Byte-compare every owned out region with the source (int views: NaN
    payloads and -0.0 count)."""
    import torch

    iv = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[out.element_size()]
    for it in items:
        osel = tuple(it[3])
        if not torch.equal(out[osel].view(iv), src[osel].view(iv)):
            raise SystemExit(f"bench {what}: decoded bytes differ from the source in {osel}")


def eager_kernel_times(progs, steps, device):
    """Per-launch kernel durations (HIP events around each eager launch on the
    launch stream), rotating over the programs."""
    import torch

    stream = torch.cuda.current_stream(device)
    sh = int(stream.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize(device)
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        progs[i % len(progs)].launch(sh)
        b.record(stream)
    torch.cuda.synchronize(device)
    return [a.elapsed_time(b) / 1e3 for a, b in ev]


def graph_steps(progs, steps, warmup, device, ctx=None):
    """The timed region: ``steps`` full decodes rotating over the programs,
    captured once as a hipGraph (zarr_hip.ReadGraph) and replayed with one
    launch, bracketed by barrier + synchronize.  Returns (this rank's wall
    seconds, max over ranks, event span on the launch stream in seconds)."""
    import torch

    import zarr_hip

    g_warm = zarr_hip.ReadGraph(progs, max(1, warmup), device)
    g_main = zarr_hip.ReadGraph(progs, steps, device)
    g_warm.replay()
    stream = torch.cuda.current_stream(device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if ctx is not None:
        ctx.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    a.record(stream)
    g_main.replay()
    b.record(stream)
    torch.cuda.synchronize(device)
    wall = time.perf_counter() - t0
    if ctx is not None:
        ctx.barrier()
    for p in progs:
        p.results()  # raises on any CRC / status error accumulated during the run
    wall_max = ctx.max(wall) if ctx is not None else wall
    return wall, wall_max, a.elapsed_time(b) / 1e3


def time_programs(progs, steps, warmup, device, ctx=None):
    """(max-over-ranks wall seconds per step of the graph-replayed loop, this
    rank's kernel seconds per launch: the smaller of two upper bounds, the
    median eager event-timed launch and the graph replay's event span / steps;
    the eager median alone is noisy for ~16 us kernels)."""
    _, wall_max, span = graph_steps(progs, steps, warmup, device, ctx)
    kern = eager_kernel_times(progs, steps, device)
    for p in progs:
        p.results()
    return wall_max / steps, min(float(np.median(kern)), span / steps)


def _short_steps(args) -> int:
    """Timed launches for the device-only lines whose launch is tens of
    microseconds (C1, C2, C3, the encodes, the example array): at least 50, so
    the graph span per launch is not swayed by one slow first replay (the
    rocprof traces show single launches up to 1.3x the median)."""
    return max(50, args.steps)


SHORT_WARMUP = 10


def _last_kernel() -> str:
    from zarr_hip import _native as N

    return N.lib().zhip_last_kernel().decode()


def _entry(dec, alg, wall, kern, **kw):
    """One extra's line; decode legs are labelled with the kernel the library
    launched last (zhip_last_kernel: the timed program's data launch)."""
    d = {"decoded_GiBps": round(dec / wall / GIB, 1), "step_ms": round(wall * 1e3, 4),
         "kernel_ms": round(kern * 1e3, 4), "algorithmic_bytes": int(alg),
         "hbm_frac": round(alg / kern / 1e9 / HBM_PEAK_GBS, 4)}
    d.update(kw)
    if "kernel" not in d:
        d["kernel"] = _last_kernel()
    return d


# --------------------------------------------------------------------- configs

def extra_configs(ctx, args):
    """Configs measured beside the headline: BASELINE.json configs[0..4] plus the
    host-memory end-to-end rate.  C4 and C5 run at every N (partitioned); the
    single-GPU configs only at N=1."""
    import torch

    device = ctx.device
    out = {}
    steps = _short_steps(args)
    single = ctx.world == 1
    # the host-memory legs first: after the 4-16 GiB legs below the same reads
    # measured up to 2x slower in one process (caching-allocator and host
    # memory state), so they run while the process is fresh
    if single and "e2e" in args.extra:
        out["e2e_c2_host"] = e2e_host(ctx.device, args)
        torch.cuda.empty_cache()
    if single and "cpp" in args.extra:
        out["cpp_example_4096"] = cpp_example(device, args)
        torch.cuda.empty_cache()
    if single and "c1" in args.extra:
        out["c1_1d_bytes"] = c1_plumbing(device, args)
        torch.cuda.empty_cache()
    shape, chunks = (256, 256, 256), (64, 64, 64)
    if single and "c2" in args.extra:
        # BASELINE configs[1]: the same array unsharded (64 chunks of 64^3)
        data = torch.from_numpy(synthetic(shape, seed=0)).to(device)
        progs = []
        for _ in range(args.replicas):
            p, o = build_replica(device, data, shape, chunks, [LE, CRC]).prepare_read((Ellipsis,))
            progs.append((p, o))
        progs[0][0].launch()
        progs[0][0].results()
        if not torch.equal(progs[0][1].view(torch.int32), data.view(torch.int32)):
            raise SystemExit("bench c2: decoded bytes differ from the source")
        wall, kern = time_programs([p for p, _ in progs], steps, SHORT_WARMUP, device)
        dec = data.numel() * 4
        out["c2_unsharded_256"] = _entry(dec, dec + 64 * (1048576 + 4), wall, kern, checked="bytes")
        del progs
        # the headline array with zarr's DEFAULT sharding codecs (inner chunks
        # bytes only, index bytes + crc32c: sharding.py:423-427): the index
        # checks ride in leading workgroups of the data launch (k_decode_lead)
        progs = []
        for _ in range(args.replicas):
            p, o = build_replica(device, data, shape, chunks, [LE], shards=(128, 128, 128)).prepare_read(
                (Ellipsis,))
            progs.append((p, o))
        progs[0][0].launch()
        progs[0][0].results()
        if not torch.equal(progs[0][1].view(torch.int32), data.view(torch.int32)):
            raise SystemExit("bench sharded default chain: decoded bytes differ from the source")
        fused = progs[0][0].index is None and progs[0][0].data.n_idx == 8
        wall, kern = time_programs([p for p, _ in progs], steps, SHORT_WARMUP, device)
        out["sharded_default_chain_256"] = _entry(
            dec, dec + 64 * 1048576 + 8 * (8 * 16 + 4), wall, kern, checked="bytes",
            kernel=_last_kernel() + (" (index checks in 8 leading workgroups)" if fused
                                     else " (after a separate index launch)"),
            note="headline array and shards, zarr's default sharding codecs: inner bytes only, index bytes+crc32c")
        del progs, data
    if single and "c3" in args.extra:
        data = torch.from_numpy(synthetic(shape, seed=0)).to(device)
        progs = []
        for _ in range(args.replicas):
            arr = build_replica(device, data, shape, chunks,
                                [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC])
            progs.append(arr.prepare_read((Ellipsis,)))
        assert progs[0][0].tables.tile, "C3 should take the LDS-tiled transpose kernel"
        progs[0][0].launch()
        progs[0][0].results()
        if not torch.equal(progs[0][1].view(torch.int32), data.view(torch.int32)):
            raise SystemExit("bench c3: decoded bytes differ from the source")
        from zarr_hip import _native as N
        tile4 = bool(N.Plan(progs[0][0].tables.layout, upload=False).kernel_flags & N.PK_TILE4) and \
            not (args.tune & 65536)
        wall, kern = time_programs([p for p, _ in progs], steps, SHORT_WARMUP, device)
        dec = data.numel() * 4
        out["c3_transpose_210"] = _entry(dec, dec + 64 * (1048576 + 4), wall, kern, checked="bytes",
                                         tile4_eligible=tile4)
        del progs
        # the same array in 128^3 chunks: k_decode_tile4 declines (512 tiles per
        # chunk, two different steps between consecutive tiles) -> k_decode_tileg
        progs = []
        for _ in range(args.replicas):
            arr = build_replica(device, data, shape, (128, 128, 128),
                                [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC])
            progs.append(arr.prepare_read((Ellipsis,)))
        progs[0][0].launch()
        progs[0][0].results()
        if not torch.equal(progs[0][1].view(torch.int32), data.view(torch.int32)):
            raise SystemExit("bench c3 (128^3 chunks): decoded bytes differ from the source")
        kf = N.Plan(progs[0][0].tables.layout, upload=False).kernel_flags
        wall, kern = time_programs([p for p, _ in progs], steps, SHORT_WARMUP, device)
        out["c3_transpose_210_chunks128"] = _entry(
            dec, dec + 8 * (128 ** 3 * 4 + 4), wall, kern, checked="bytes",
            tileg_eligible=bool(kf & N.PK_TILEG),
            note="8 chunks of 128^3: no k_decode_tile4 (round 1: persistent k_decode_tile)")
        del progs, data
    if "c4" in args.extra:
        out["c4_sharded_1024"] = c4_partitioned(ctx, args)
        torch.cuda.empty_cache()
    if "c5" in args.extra:
        out["c5_partial_2048"] = c5_partial(ctx, args)
        torch.cuda.empty_cache()
        if single and not getattr(args, "no_host_legs", False):
            out["c5_host_coalesced"] = c5_host(ctx, args)
            torch.cuda.empty_cache()
    if single and "enc" in args.extra:
        out["encode_c2"] = encode_c2(device, args)
        torch.cuda.empty_cache()
        out["encode_c3"] = encode_c3(device, args)
        torch.cuda.empty_cache()
        out["encode_c3_chunks128"] = encode_c3_general(device, args)
        torch.cuda.empty_cache()
    if single and "call" in args.extra:
        out["device_read_call"] = device_read_call(device, args)
        torch.cuda.empty_cache()
    return out


def device_read_call(device, args):
    """The headline read as a zarr caller issues it: one
    HipCodecPipeline.read_sync per call (eager, no graph, synchronised: the
    call returns with statuses checked), device-resident store and out,
    rotating over the replicas.  Three ways: read_sync on a built batch
    through the per-call plan cache (a repeated read re-launches the cached
    program: no planning, no table upload, one 4-byte error word back);
    Array.get, which also rebuilds the batch (BasicIndexer) every call; and
    read_sync with the cache off (plans and uploads every call, round 2's
    path).  ms_per_call is host wall per call; host_overhead_ms subtracts the
    kernel's own time."""
    import torch

    from zarr_hip import pipeline as P

    g = W.HEADLINE
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    src = torch.from_numpy(synthetic(shape, seed=0)).to(device)
    R = args.replicas
    arrs = [build_replica(device, src, shape, inner, [LE, CRC], shards=shards) for _ in range(R)]
    batches = [a.batch_info((Ellipsis,))[0] for a in arrs]
    outs = [torch.empty(shape, dtype=torch.float32, device=device) for _ in range(R)]
    t0 = time.perf_counter()
    arrs[0].codec_pipeline.read_sync(batches[0], outs[0])
    first_ms = (time.perf_counter() - t0) * 1e3
    for i in range(R):
        arrs[i].codec_pipeline.read_sync(batches[i], outs[i])
        if not torch.equal(outs[i].view(torch.int32), src.view(torch.int32)):
            raise SystemExit("bench device_read_call: decoded bytes differ from the source")
    progs = [a.prepare_read((Ellipsis,))[0] for a in arrs]
    kern = float(np.median(eager_kernel_times(progs, max(20, args.steps), device)))
    del progs
    n = max(50, 2 * args.steps)

    def timed(fn):
        for i in range(R):
            fn(i)
        torch.cuda.synchronize(device)
        t = time.perf_counter()
        for i in range(n):
            fn(i % R)
        return (time.perf_counter() - t) / n

    cached = timed(lambda i: arrs[i].codec_pipeline.read_sync(batches[i], outs[i]))
    get = timed(lambda i: arrs[i].get((Ellipsis,), out=outs[i]))
    keep, P.READ_CACHE_SIZE = P.READ_CACHE_SIZE, 0
    try:
        uncached = timed(lambda i: arrs[i].codec_pipeline.read_sync(batches[i], outs[i]))
    finally:
        P.READ_CACHE_SIZE = keep
    for i in range(R):
        if not torch.equal(outs[i].view(torch.int32), src.view(torch.int32)):
            raise SystemExit("bench device_read_call: decoded bytes differ from the source")
    # a data loader walking the array: a DIFFERENT selection every call (128-row
    # windows at 8 offsets, crossing shard boundaries), plan cache off
    sels = [(slice(16 * i + 8, 16 * i + 136), slice(None), slice(None)) for i in range(8)]
    wouts = [torch.empty((128,) + tuple(shape[1:]), dtype=torch.float32, device=device) for _ in sels]
    wb = [arrs[0].batch_info(sl)[0] for sl in sels]
    wprogs = [arrs[0].codec_pipeline.prepare_read(b, o) for b, o in zip(wb, wouts)]
    wkern = float(np.median(eager_kernel_times(wprogs, max(16, args.steps), device)))
    del wprogs
    keep, P.READ_CACHE_SIZE = P.READ_CACHE_SIZE, 0
    try:
        ctr = [0]

        def walk(_i):
            j = ctr[0] = (ctr[0] + 1) % 8
            arrs[0].codec_pipeline.read_sync(wb[j], wouts[j])

        varying = timed(walk)
    finally:
        P.READ_CACHE_SIZE = keep
    for i in range(8):
        if not torch.equal(wouts[i].view(torch.int32), src[sels[i]].contiguous().view(torch.int32)):
            raise SystemExit("bench device_read_call: a window read differs from the source")
    dec = src.numel() * 4

    def line(w):
        return {"ms_per_call": round(w * 1e3, 4), "decoded_GiBps": round(dec / w / GIB, 1),
                "host_overhead_ms": round((w - kern) * 1e3, 4)}

    return {"kernel_ms": round(kern * 1e3, 4), "calls": n, "first_call_ms": round(first_ms, 3),
            "read_sync_cached": line(cached), "array_get_cached": line(get),
            "read_sync_uncached": line(uncached), "checked": "bytes",
            "read_sync_uncached_varying": {
                "ms_per_call": round(varying * 1e3, 4), "kernel_ms": round(wkern * 1e3, 4),
                "host_overhead_ms": round((varying - wkern) * 1e3, 4),
                "decoded_GiBps": round(128 * 256 * 256 * 4 / varying / GIB, 1),
                "note": "a different 128-row window (16 MiB) every call, plan cache off"},
            "note": "headline config; eager per-call reads, each synchronised; kernel_ms = median "
                    "event-timed eager launch of the same program"}


def c4_partitioned(ctx, args):
    """BASELINE configs[3]: 1024^3 f32, 128^3 shards of 32^3 inner chunks
    (bytes+crc32c; 512 shards, 32 768 inner chunks), the shards split
    round-robin over the ranks (strong scaling: the batch is fixed).  Each rank
    encodes and decodes only its shards; every decoded byte is compared with the
    source; aggregate = all ranks' decoded bytes / max rank time."""
    import torch

    g = W.C4
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    gen = torch.Generator(device=ctx.device).manual_seed(0)
    data = torch.randn(shape, generator=gen, device=ctx.device, dtype=torch.float32)
    n_shards = int(np.prod([s // c for s, c in zip(shape, shards)]))
    mine_n = len(range(ctx.rank, n_shards, ctx.world))
    blob = 64 * (131072 + 4) + 64 * 16 + 4
    cap = mine_n * (blob + 256) + (1 << 20)
    progs = []
    for r in range(2):
        prog, out, mine = build_partitioned(ctx, data, shape, inner, shards, "float32", 0.0, cap)
        if r == 0:
            prog.launch()
            prog.results()
            check_regions(out, data, mine, "c4")
        progs.append(prog)
    del data
    wall, kern = time_programs(progs, 10, 3, ctx.device, ctx)
    my_dec = mine_n * 128 ** 3 * 4
    dec = ctx.sum(my_dec)
    my_alg = my_dec + mine_n * blob
    del progs
    return _entry(dec, my_alg, wall, kern, checked="bytes", shards_per_rank=mine_n,
                  partition=f"round-robin by shard over {ctx.world} rank(s)",
                  note="decoded_GiBps = all ranks' decoded bytes / max rank step time; "
                       "kernel_ms / hbm_frac are this rank's")


def c5_partial(ctx, args):
    """BASELINE configs[4]: 2048^3 int16 in 256^3 shards of 64^3 inner chunks
    (512 shards x 64 inner, 512 KiB each), bytes+crc32c; a random 10 % of the
    inner chunks (seed 1, workloads.partial_selection) decoded per step, one
    batch item per inner chunk, each into its region of a full-shape device
    output.  The shards are split round-robin over the ranks; a rank stages and
    decodes the selected inner chunks of its own shards.  Kernels locate every
    inner chunk through its shard index in HBM; each touched shard's index CRC
    is verified once per step; every selected region is compared with the source."""
    import torch

    import zarr_hip
    from zarr_hip import parallel

    g = W.C5
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    gen = torch.Generator(device=ctx.device).manual_seed(0)
    data = torch.randint(-2 ** 15, 2 ** 15, shape, generator=gen, device=ctx.device, dtype=torch.int16)
    n_shards = int(np.prod([s // c for s, c in zip(shape, shards)]))
    mine_n = len(range(ctx.rank, n_shards, ctx.world))
    shard_bytes = int(np.prod(shards)) * 2 + 64 * 4 + 64 * 16 + 4
    store = zarr_hip.DeviceStore(ctx.device, capacity=mine_n * (shard_bytes + 256) + (1 << 24))
    arr = zarr_hip.Array.create(store, shape, inner, "int16", 0, shards=shards, inner_codecs=[LE, CRC])
    sbatch, _ = arr.batch_info((Ellipsis,))
    my_shards = parallel.rank_batch(sbatch, ctx.world, ctx.rank)
    for i in range(0, len(my_shards), 64):  # encode in groups to bound temporaries
        arr.codec_pipeline.write_sync(my_shards[i:i + 64], data)
    torch.cuda.synchronize(ctx.device)
    mine_keys = {it[0].path for it in my_shards}
    grid = tuple(s // i for s, i in zip(shape, inner))
    coords = W.partial_selection(grid)
    batch = [it for it in W.inner_chunk_batch(arr, store, coords, inner) if it[0].path in mine_keys]
    out = torch.empty(shape, dtype=torch.int16, device=ctx.device)
    prog = arr.codec_pipeline.prepare_read(batch, out)
    prog.launch()
    prog.results()
    check_regions(out, data, batch, "c5")
    del data
    wall, kern = time_programs([prog], max(20, args.steps // 2), 5, ctx.device, ctx)
    n_sel = len(batch)
    touched = len({it[0].path for it in batch})
    my_dec = n_sel * 64 ** 3 * 2
    dec = ctx.sum(my_dec)
    alg = my_dec + n_sel * (64 ** 3 * 2 + 4) + touched * (64 * 16 + 4)
    del prog, out, store, arr
    return _entry(dec, alg, wall, kern, inner_chunks=n_sel, inner_chunks_total=len(coords),
                  shards_touched=touched, checked="bytes",
                  layout="256^3 shards of 64^3 int16 inner chunks",
                  partition=f"round-robin by shard over {ctx.world} rank(s)",
                  note="one output replica; selection 10% random inner chunks, seed 1; "
                       "decoded_GiBps = all ranks' decoded bytes / max rank step time")


def c5_host(ctx, args):
    """C5 from a HOST store (examples/sharding_coalescing): the same 2048^3
    int16 array, 256^3 shards of 64^3 inner chunks, in a host MemoryStore; the
    random 10 % of inner chunks read into a device out through the pipeline's
    host path -- one index suffix request per touched shard, the touched inner
    chunks fetched by coalesced range requests (store.get_ranges_sync with the
    reference's 1 MiB gap / 16 MiB span rules, src/zarr/core/_coalesce.py:61-135),
    packed into pinned windows and decoded on the GPU.  Reports the requests
    issued per read next to what an uncoalesced reader would issue, and the
    host -> HBM decoded rate (PCIe-inclusive: never the headline)."""
    import torch

    import zarr_hip

    g = W.C5
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    gen = torch.Generator(device=ctx.device).manual_seed(0)
    data = torch.randint(-2 ** 15, 2 ** 15, shape, generator=gen, device=ctx.device, dtype=torch.int16)
    n_shards = int(np.prod([s // c for s, c in zip(shape, shards)]))
    shard_bytes = int(np.prod(shards)) * 2 + 64 * 4 + 64 * 16 + 4
    dstore = zarr_hip.DeviceStore(ctx.device, capacity=n_shards * (shard_bytes + 256) + (1 << 24))
    darr = zarr_hip.Array.create(dstore, shape, inner, "int16", 0, shards=shards, inner_codecs=[LE, CRC])
    sbatch, _ = darr.batch_info((Ellipsis,))
    for i in range(0, len(sbatch), 64):
        darr.codec_pipeline.write_sync(sbatch[i:i + 64], data)
    torch.cuda.synchronize(ctx.device)

    class CountingStore(zarr_hip.MemoryStore):
        calls = 0
        fetched = 0

        def get_sync(self, key, byte_range=None, prototype=None):
            v = super().get_sync(key, byte_range, prototype)
            if not key.endswith("zarr.json"):
                CountingStore.calls += 1
                CountingStore.fetched += 0 if v is None else len(v)
            return v

    host = CountingStore(dstore.to_dict())
    del dstore, darr
    torch.cuda.empty_cache()
    arr = zarr_hip.Array.open(host)
    grid = tuple(s // i for s, i in zip(shape, inner))
    coords = W.partial_selection(grid)
    batch = W.inner_chunk_batch(arr, host, coords, inner)
    out = torch.empty(shape, dtype=torch.int16, device=ctx.device)
    arr.codec_pipeline.read_sync(batch, out)
    torch.cuda.synchronize(ctx.device)
    check_regions(out, data, batch, "c5 host")
    del data
    ts, calls, fetched = [], [], []
    for _ in range(5):
        CountingStore.calls = CountingStore.fetched = 0
        torch.cuda.synchronize(ctx.device)
        t0 = time.perf_counter()
        arr.codec_pipeline.read_sync(batch, out)
        torch.cuda.synchronize(ctx.device)
        ts.append(time.perf_counter() - t0)
        calls.append(CountingStore.calls)
        fetched.append(CountingStore.fetched)
    touched = len({it[0].path for it in batch})
    dec = len(batch) * 64 ** 3 * 2
    med = float(np.median(ts))
    return {"host_to_hbm_decoded_GiBps": round(dec / med / GIB, 2), "ms_per_read": round(med * 1e3, 2),
            "requests": int(calls[-1]), "requests_uncoalesced": touched + len(batch),
            "fetched_MiB": round(fetched[-1] / 2 ** 20, 1), "inner_chunks": len(batch),
            "shards_touched": touched, "checked": "bytes",
            "note": "host MemoryStore; index suffix request per touched shard + coalesced inner-chunk "
                    "range requests (1 MiB gap, 16 MiB span); requests_uncoalesced = index + one per "
                    "inner chunk; PCIe-inclusive"}


class _EncodeProg:
    """One prepared k_encode launch (what ChunkWriter._encode_chunks issues for
    complete chunks) in the program interface ReadGraph replays."""

    def __init__(self, launch):
        self.l = launch

    def launch(self, stream=None):
        self.l.launch(stream)

    def check_fresh(self):
        return None

    def results(self):
        return None


def _encode_bench(device, args, codecs, want, chunks=(64, 64, 64), check=True):
    """want: "rows" (k_encode_il / k_encode_pair), "tile4" (k_encode_tile4) or "tile"
    (k_encode_tile, the general transposed encode)."""
    import torch

    import zarr_hip
    from zarr_hip import _native as N
    from zarr_hip.planner import analyze_chain, plan_encode
    from zarr_hip.writer import EncodeLaunch

    shape = (256, 256, 256)
    data = torch.from_numpy(synthetic(shape, seed=0)).to(device)
    progs, checks = [], []
    elen = int(np.prod(chunks)) * 4 + (4 if any(c.get("name") == "crc32c" for c in codecs) else 0)
    n_chunks = int(np.prod([s // c for s, c in zip(shape, chunks)]))
    # 4 replicas, each with its own source copy and store (512 MiB in all, past
    # the 256 MiB Infinity Cache: no step reads a source another step left there)
    for _ in range(4):
        src_r = data.clone()
        store = zarr_hip.DeviceStore(device, capacity=n_chunks * (elen + 256) + (1 << 20))
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 0.0, codecs=codecs)
        batch, _ = arr.batch_info((Ellipsis,))
        spec = batch[0][1]
        chain = analyze_chain(arr.codec_pipeline.codecs, spec)
        offs = [store.arena.reserve(elen) for _ in batch]
        items = [(offs[i], it[2], [sl.start or 0 for sl in it[3]]) for i, it in enumerate(batch)]
        t = plan_encode(chain, spec, items, [int(x) * 4 for x in src_r.stride()], src_r.data_ptr())
        el = EncodeLaunch(t.layout, t.chunks, t.sels, src_r, store.arena.buf, t.fast, device, t.rows,
                          t.tile, t.tile_prefix)
        if want == "rows":
            assert t.rows, "C2 encode should take the row-mapped encode"
        else:
            assert t.tile and el.flags & N.DF_TILE, "C3 encode should take a tiled encode"
            t4 = bool(el.plan.kernel_flags & N.PK_TILE4_ENCODE)
            assert t4 == (want == "tile4"), f"expected the {want} encode"
        progs.append(_EncodeProg(el))
        checks.append((store, arr, batch, offs, elen))
    wall, kern = time_programs(progs, _short_steps(args), SHORT_WARMUP, device)
    kname = N.lib().zhip_last_kernel().decode()  # (mapped encodes; before the check's decodes)
    for store, arr, batch, offs, elen in (checks if check else []):  # (check=False: ablation arms)
        for (bg, *_), off in zip(batch, offs):
            store.register(bg.path, off, elen)
        if not torch.equal(arr.get((Ellipsis,)).view(torch.int32), data.view(torch.int32)):
            raise SystemExit("bench encode: decoded store differs from the source")
    src = data.numel() * 4
    return src, wall, kern, kname


def encode_c3(device, args):
    """Encode side of C3: the 256^3 f32 array written through transpose(2,1,0) +
    bytes + crc32c into 64 chunks of 64^3 by k_encode_tile4 (two LDS tiles per
    workgroup since round 5, "k_encode_tile2"), timed like the decode and
    decoded back for the check."""
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC]
    src, wall, kern, kname = _encode_bench(device, args, codecs, "tile4")
    return _entry(src, src + 64 * (1048576 + 4), wall, kern,
                  kernel="k_encode" if args.tune & 65536 else kname, checked="bytes",
                  note="decoded_GiBps = source bytes encoded per second")


def encode_c3_general(device, args):
    """A transposed encode k_encode_tile4 does not take: the C3 array through
    transpose(2,1,0) into 8 chunks of 128^3 (512 tiles of 64 x 256 B per
    chunk, more than the four-tile kernel's 64, and groups of four
    consecutive tiles at two different steps): k_encode_tileg, tiles grouped
    by four along the stored dim 1 (round 1 sent these to the per-element
    k_encode at 0.05; --tune 65536 runs the one-group-per-workgroup general
    k_encode_tile instead)."""
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC]
    src, wall, kern, _ = _encode_bench(device, args, codecs, "tile", chunks=(128, 128, 128))
    return _entry(src, src + 8 * (128 ** 3 * 4 + 4), wall, kern,
                  kernel="k_encode_tile" if args.tune & 65536 else "k_encode_tileg", checked="bytes",
                  note="decoded_GiBps = source bytes encoded per second; 128^3 chunks")


def encode_c2(device, args):
    """Encode side of C2 (a2/a4/a15): the 256^3 f32 device array written as 64
    chunks of 64^3 with bytes+crc32c into a DeviceStore arena -- gather 16-byte
    rows, empty-chunk check, CRC, trailer -- by k_encode_il (one 32 KiB unit
    per workgroup, steps interleaved in groups of eight; k_encode_pair before
    round 5), the launch HipCodecPipeline.write_sync issues for complete
    chunks.  Timed like the decode (graph replay of K launches); the stored
    bytes are then decoded back and compared with the source."""
    src, wall, kern, kname = _encode_bench(device, args, [LE, CRC], "rows")
    return _entry(src, src + 64 * (1048576 + 4), wall, kern,
                  kernel="k_encode" if args.tune & 64 else kname, checked="bytes",
                  note="decoded_GiBps = source bytes encoded per second")


def c1_plumbing(device, args):
    """BASELINE configs[0] (bench/compress_normal.py-style): 1e7 float32 1-D in
    (2**20,) chunks, bytes codec only (10 chunks, the last a boundary chunk
    stored at full size).  The reference runs it on the CPU pipeline; here:
    the device-resident decode (row decode on 1-D chunks viewed as whole rows) and the MemoryStore
    round trip (host bytes -> HBM -> host), both checked bit-exact."""
    import torch

    import zarr_hip

    n, ck = 10 ** 7, 2 ** 20
    rng = np.random.default_rng(0)
    a = rng.standard_normal(n, dtype=np.float32)
    host = zarr_hip.MemoryStore({})
    harr = zarr_hip.Array.create(host, (n,), (ck,), "float32", 0.0, codecs=[LE])
    harr.set((Ellipsis,), torch.from_numpy(a).to(device))
    torch.cuda.synchronize(device)
    if harr[...].tobytes() != a.tobytes():
        raise SystemExit("bench c1: host round trip differs from the source")
    # 4 replicas (own source store and out each: 320 MB, past the 256 MiB
    # Infinity Cache, so no step re-reads another's bytes from it)
    progs = [zarr_hip.Array.open(zarr_hip.DeviceStore.from_host(host.to_dict(), device)).prepare_read((Ellipsis,))
             for _ in range(4)]
    progs[0][0].launch()
    progs[0][0].results()
    if progs[0][1].cpu().numpy().tobytes() != a.tobytes():
        raise SystemExit("bench c1: device decode differs from the source")
    wall, kern = time_programs([p for p, _ in progs], _short_steps(args), SHORT_WARMUP, device)
    dec = n * 4
    t_rt = []
    for _ in range(0 if getattr(args, "no_host_legs", False) else 5):
        t0 = time.perf_counter()
        harr[...]
        t_rt.append(time.perf_counter() - t0)
    return _entry(dec, dec + 10 * ck * 4, wall, kern, checked="bytes",
                  host_roundtrip_GiBps=round(dec / float(np.median(t_rt)) / GIB, 2) if t_rt else None,
                  note="device decode of 1-D chunks viewed as whole 512-byte rows (planner._split_1d; 128 units per chunk); host_roundtrip = MemoryStore -> HBM -> numpy")


def e2e_host(device, args):
    """Host memory -> host memory (the path's full IO):
    C2's encoded chunks in a host MemoryStore; arr[...] stages them into
    pinned memory, H2D on a copy stream, decodes per window, and copies the
    result back through pinned memory into a numpy array."""
    import torch

    import zarr_hip

    shape, chunks = (256, 256, 256), (64, 64, 64)
    data_np = synthetic(shape, seed=0)
    dev_arr = build_replica(device, torch.from_numpy(data_np).to(device), shape, chunks, [LE, CRC])
    host = zarr_hip.MemoryStore(dev_arr.store_path.store.to_dict())
    arr = zarr_hip.Array.open(host)
    got = arr[...]
    if got.tobytes() != data_np.tobytes():
        raise SystemExit("bench e2e: host read differs from the source")
    out = torch.empty(shape, dtype=torch.float32, device=device)
    t_h2h, t_h2d = [], []
    for _ in range(10):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        arr[...]
        t_h2h.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        arr.get((Ellipsis,), out=out)
        torch.cuda.synchronize(device)
        t_h2d.append(time.perf_counter() - t0)
    if not torch.equal(out.view(torch.int32).cpu(), torch.from_numpy(data_np).view(torch.int32)):
        raise SystemExit("bench e2e: device read differs from the source")
    # the same chunks in a PinnedMemoryStore: DMA straight from the store
    parr = zarr_hip.Array.open(zarr_hip.PinnedMemoryStore(dev_arr.store_path.store.to_dict()))
    if parr[...].tobytes() != data_np.tobytes():
        raise SystemExit("bench e2e: pinned-store read differs from the source")
    p_h2h, p_h2d = [], []
    for _ in range(10):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        parr[...]
        p_h2h.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        parr.get((Ellipsis,), out=out)
        torch.cuda.synchronize(device)
        p_h2d.append(time.perf_counter() - t0)
    if not torch.equal(out.view(torch.int32).cpu(), torch.from_numpy(data_np).view(torch.int32)):
        raise SystemExit("bench e2e: pinned-store device read differs from the source")
    # the same chunks as files of a LocalStore (page cache warm): the staging
    # pool preads them straight into the pinned windows
    import shutil
    import tempfile

    tmp = tempfile.mkdtemp(prefix="zhip_e2e_")
    try:
        lst = zarr_hip.LocalStore(tmp)
        for k, v in dev_arr.store_path.store.to_dict().items():
            lst.set_sync(k, v)
        larr = zarr_hip.Array.open(lst)
        if larr[...].tobytes() != data_np.tobytes():
            raise SystemExit("bench e2e: local-store read differs from the source")
        l_h2h, l_h2d = [], []
        for _ in range(10):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            larr[...]
            l_h2h.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            larr.get((Ellipsis,), out=out)
            torch.cuda.synchronize(device)
            l_h2d.append(time.perf_counter() - t0)
        if not torch.equal(out.view(torch.int32).cpu(), torch.from_numpy(data_np).view(torch.int32)):
            raise SystemExit("bench e2e: local-store device read differs from the source")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    pin = torch.empty(data_np.nbytes, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(data_np.nbytes, dtype=torch.uint8, device=device)
    dbuf.copy_(pin, non_blocking=True)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(10):
        dbuf.copy_(pin, non_blocking=True)
    torch.cuda.synchronize(device)
    h2d_raw = data_np.nbytes * 10 / (time.perf_counter() - t0) / GIB
    dec = data_np.nbytes
    return {"host_to_host_GiBps": round(dec / float(np.median(t_h2h)) / GIB, 2),
            "host_to_hbm_decoded_GiBps": round(dec / float(np.median(t_h2d)) / GIB, 2),
            "pinned_h2d_copy_GiBps": round(h2d_raw, 2),
            "host_to_host_ms": round(float(np.median(t_h2h)) * 1e3, 3),
            "host_to_hbm_ms": round(float(np.median(t_h2d)) * 1e3, 3),
            "pinned_store_to_hbm_decoded_GiBps": round(dec / float(np.median(p_h2d)) / GIB, 2),
            "pinned_store_to_host_GiBps": round(dec / float(np.median(p_h2h)) / GIB, 2),
            "local_store_to_hbm_decoded_GiBps": round(dec / float(np.median(l_h2d)) / GIB, 2),
            "local_store_to_host_GiBps": round(dec / float(np.median(l_h2h)) / GIB, 2),
            "checked": "bytes",
            "note": "MemoryStore values are pageable bytes (packed into pinned windows by the library pool); "
                    "PinnedMemoryStore keeps them page-locked and the read DMAs straight from it; "
                    "LocalStore files (page cache warm) are pread into the pinned windows by the pool"}


# ------------------------------------------------------------------ CPU baseline

def box_cores() -> int:
    """The host cores this process may use: the affinity mask, capped by the
    box's share (OMP_NUM_THREADS is set to the share on the GPU boxes)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap else n)


def _median_s(fn, repeat=3):
    ts = []
    for _ in range(repeat):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def cpp_example(device, args):
    """extra.cpp_example_4096: the reference's own timing harness for this
    boundary (examples/codec_pipeline_performance/codec_pipeline_performance.py:
    67-80, 95-130) -- 4096^2 int32 (64 MiB), 16 shards of 1024^2, 256 inner
    chunks of 64^2 (16 KiB, 256-byte rows) per shard, zarr's default sharding
    codecs, compressors None (arange data) or gzip-6 (noisy data).

    * device: the uncompressed array resident in HBM, one full decode per step
      (one launch: 4096 inner chunks, 16 index CRCs), graph-timed;
    * host: as the example does, the median of 3 full writes and of 3 full
      reads through zarr_hip.Array on a MemoryStore and a LocalStore (host ->
      HBM -> host; compression on the host stage);
    * cpu_port: the oracle's restatement of FusedCodecPipeline's per-shard
      pool map (codec_pipeline.py:1095-1172, 1174-1255) over the same bytes in
      host memory, at 1 worker and at the box's worker share, write and read."""
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    import torch

    import zarr_hip
    from oracle import oracle as O

    g = W.CPP_EXAMPLE
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    res = {"workload": "4096^2 int32, 16 shards of 1024^2, 64^2 inner chunks (codec_pipeline_performance.py)"}
    plain = W.cpp_example_data("plain")
    noisy = W.cpp_example_data("noisy")
    dec = plain.nbytes
    n_inner = (shape[0] // inner[0]) * (shape[1] // inner[1])
    # 1. device-resident decode of the uncompressed chain
    data = torch.from_numpy(plain).to(device)
    progs = []
    for _ in range(args.replicas):
        arr = build_replica(device, data, shape, inner, [LE], shards=shards, dtype="int32", fill=0)
        progs.append(arr.prepare_read((Ellipsis,)))
    progs[0][0].launch()
    progs[0][0].results()
    if not torch.equal(progs[0][1], data):
        raise SystemExit("bench cpp_example: decoded bytes differ from the source")
    wall, kern = time_programs([p for p, _ in progs], _short_steps(args), SHORT_WARMUP, device)
    alg = 2 * dec + 16 * (256 * 16 + 4)
    res["device_uncompressed"] = _entry(dec, alg, wall, kern, checked="bytes",
                                        note=f"{n_inner} inner chunks of 16 KiB + 16 index CRCs per launch")
    del progs, data, arr
    torch.cuda.empty_cache()
    # 2. host stores, full write + full read (the example's measure())
    host = {}
    if getattr(args, "no_host_legs", False):
        return res
    with tempfile.TemporaryDirectory() as tmp:
        for kind in ("memory", "local"):
            for label, codecs, src in (("uncompressed", [LE], plain), ("gzip6", [LE, W.GZIP6], noisy)):
                def mk(kind=kind, label=label):
                    return zarr_hip.MemoryStore() if kind == "memory" else \
                        zarr_hip.LocalStore(os.path.join(tmp, f"{kind}_{label}_{time.perf_counter_ns()}"))

                holder = {}

                def write_once(codecs=codecs, src=src, mk=mk, holder=holder):
                    st = mk()
                    a = zarr_hip.Array.create(st, shape, inner, "int32", 0, shards=shards, inner_codecs=codecs)
                    a[...] = src
                    holder["a"] = a

                w = _median_s(write_once)
                r = _median_s(lambda holder=holder: holder["a"][...])
                if not np.array_equal(holder["a"][...], src):
                    raise SystemExit(f"bench cpp_example: {kind}/{label} round trip mismatch")
                host[f"{kind}_{label}"] = {"write_s": round(w, 4), "read_s": round(r, 4),
                                           "write_GiBps": round(dec / w / GIB, 2),
                                           "read_GiBps": round(dec / r / GIB, 2)}
    res["host"] = host
    # 3. the CPU port: per-shard pool map over the same bytes
    workers = min(16, os.cpu_count() or 1)
    port = {"workers": workers}
    for label, codecs, src in (("uncompressed", [LE], plain), ("gzip6", [LE, W.GZIP6], noisy)):
        meta = O.ArrayMeta(shape, shards, np.dtype("int32"), 0, codecs=[
            {"name": "sharding_indexed", "configuration": {"chunk_shape": list(inner), "codecs": codecs,
                                                           "index_location": "end"}}])
        chain, spec = meta.chain, meta.spec()
        grid = [(i, j) for i in range(shape[0] // shards[0]) for j in range(shape[1] // shards[1])]
        store = {}

        def enc(c, src=src, chain=chain, spec=spec, store=store):
            sl = tuple(slice(x * s, (x + 1) * s) for x, s in zip(c, shards))
            b = O.chain_encode(np.ascontiguousarray(src[sl]), chain, spec)
            if b is not None:
                store["c/%d/%d" % c] = bytes(b)

        out = np.empty(shape, np.int32)

        def decs(c, chain=chain, spec=spec, store=store, out=out):
            sl = tuple(slice(x * s, (x + 1) * s) for x, s in zip(c, shards))
            out[sl] = O.chain_decode(np.frombuffer(store["c/%d/%d" % c], np.uint8), chain, spec)

        for nw in (1, workers):
            with ThreadPoolExecutor(max_workers=nw) as pool:
                t0 = time.perf_counter()
                list(pool.map(enc, grid))
                tw = time.perf_counter() - t0
                t0 = time.perf_counter()
                list(pool.map(decs, grid))
                tr = time.perf_counter() - t0
            if not np.array_equal(out, src):
                raise SystemExit("bench cpp_example: cpu port round trip mismatch")
            port[f"{label}_w{nw}"] = {"write_s": round(tw, 4), "read_s": round(tr, 4),
                                      "read_GiBps": round(dec / tr / GIB, 2)}
    res["cpu_port"] = port
    return res


def cpu_baseline(data_np, shape, chunks, shards, budget_s=12.0):
    """The reference's FusedCodecPipeline.read_sync restated on the host for the
    headline config (oracle port): one pool task per shard
    (codec_pipeline.py:1095-1172) running ShardingCodec._decode_partial_sync
    (sharding.py:1222-1309): index by suffix read -> index CRC -> per inner chunk
    CRC-32C (SSE4.2 instruction, as google_crc32c) -> zero-copy view -> scatter
    into the shard array -> scatter of the shard into out.  Timed at the pool
    size _resolve_max_workers (codec_pipeline.py:53-73) would give on this
    box's share of cores, and at 1 worker."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    lib = O._load_lib()
    cps = tuple(s // c for s, c in zip(shards, chunks))
    n_inner = int(np.prod(cps))
    grid = tuple(s // c for s, c in zip(shape, shards))
    store = {}
    for sc in np.ndindex(*grid):
        ssl = tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(sc, shards))
        shard = data_np[ssl]
        parts, index, top = [], [], 0
        for ic in np.ndindex(*cps):  # packing order is free: the index locates each chunk
            isl = tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(ic, chunks))
            enc = bytes(O.crc32c_encode(np.ascontiguousarray(shard[isl]).view(np.uint8).reshape(-1)))
            index.append((top, len(enc)))
            parts.append(enc)
            top += len(enc)
        idx = np.array(index, "<u8").reshape(-1).view(np.uint8)
        store[sc] = b"".join(parts) + bytes(O.crc32c_encode(idx))
    isz = n_inner * 16 + 4
    out = np.empty(shape, np.float32)

    def crc_ok(u8):
        return np.uint32(lib.oracle_crc32c(u8.ctypes.data, u8.size - 4)).tobytes() == u8[-4:].tobytes()

    def read_shard(sc):
        blob = np.frombuffer(store[sc], np.uint8)
        ib = blob[-isz:]
        if not crc_ok(ib):
            raise ValueError("index checksum")
        idx = ib[:-4].view("<u8").reshape(n_inner, 2)
        sarr = np.empty(shards, np.float32)
        for slot, ic in enumerate(np.ndindex(*cps)):
            o, n = int(idx[slot, 0]), int(idx[slot, 1])
            raw = blob[o:o + n]
            if not crc_ok(raw):
                raise ValueError("checksum")
            isl = tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(ic, chunks))
            sarr[isl] = raw[:-4].view(np.float32).reshape(chunks)
        out[tuple(slice(ci * k, (ci + 1) * k) for ci, k in zip(sc, shards))] = sarr
        return None

    keys = list(store.keys())

    def run(workers, budget):
        pool = ThreadPoolExecutor(max_workers=workers)
        list(pool.map(read_shard, keys))  # warm-up
        n = 0
        t0 = time.perf_counter()
        while True:
            list(pool.map(read_shard, keys))
            n += 1
            if time.perf_counter() - t0 > budget:
                break
        dt = (time.perf_counter() - t0) / n
        pool.shutdown()
        assert out.tobytes() == data_np.tobytes()
        return dt, n

    cores = box_cores()
    workers = min(cores, len(keys))
    dt, n = run(workers, budget_s * 0.6)
    dt1, n1 = run(1, budget_s * 0.4)
    return {"value": round(data_np.nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": workers,
            "kind": "port",
            "sample": f"{n} full decodes of the headline array ({len(keys)} shards x {n_inner} "
                      f"inner chunks of 1 MiB + crc) in {n * dt:.1f}s; {workers} worker threads "
                      f"(one task per shard; {cores} cores in this box's share, "
                      f"{os.cpu_count()} cpus visible)",
            "single_worker": {"value": round(data_np.nbytes / dt1 / GIB, 3), "unit": "GiB/s",
                              "cores": 1, "sample": f"{n1} full decodes in {n1 * dt1:.1f}s"}}


def _pool_rate(fn, tasks, nbytes, budget_s, cores):
    """Time full passes of fn over tasks on a thread pool of min(cores, tasks)
    workers and of 1 worker (FusedCodecPipeline.read_sync's per-item pool map,
    codec_pipeline.py:1095-1172, at the pool size _resolve_max_workers gives on
    this box's share and single-threaded); returns the port's line."""
    from concurrent.futures import ThreadPoolExecutor

    res = {}
    for label, workers, share in (("w", min(cores, len(tasks)), 0.6), ("w1", 1, 0.4)):
        with ThreadPoolExecutor(max_workers=workers) as pool:
            list(pool.map(fn, tasks))  # warm-up
            n, t0 = 0, time.perf_counter()
            while True:
                list(pool.map(fn, tasks))
                n += 1
                if time.perf_counter() - t0 > budget_s * share:
                    break
            dt = (time.perf_counter() - t0) / n
        res[label] = (workers, dt, n)
    (w, dt, n), (_, dt1, n1) = res["w"], res["w1"]
    return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": w, "kind": "port",
            "passes": n, "single_worker": {"value": round(nbytes / dt1 / GIB, 3), "unit": "GiB/s", "cores": 1,
                                           "passes": n1}}


def cpu_config_ports(budget_s=4.0) -> dict:
    """The CPU restatement (oracle port, test infrastructure) of the reference's
    read path for every BASELINE config line beside the headline, timed on this
    host at 1 worker and at the box's share of cores -- reported baselines, not
    targets.  Each reads a bounded sample of its config's workload and says
    which:

    * c2_unsharded_256 / c3_transpose_210: the whole 256^3 f32 array, one pool
      task per 1 MiB chunk: CRC-32C verify (SSE4.2, as google_crc32c;
      crc32c_.py:34-50) -> bytes view (bytes.py:97-120) -> [TransposeCodec
      decode: the (2,1,0) permutation, transpose.py:113-118] -> scatter
      (chunk_utils.py:88-214);
    * c4_sharded_1024: 32 of its 512 shards (a 512 x 512 x 256 region, 128^3
      shards of 32^3 inner chunks), one task per shard: index CRC, then every
      inner chunk's CRC and scatter (sharding.py:1222-1309);
    * c5_partial_2048: 16 of its 512 shards (512 x 512 x 1024 int16, 256^3
      shards of 64^3 inner chunks) with ceil(10 %) of their inner chunks drawn
      as bench c5 draws them (workloads.partial_selection, seed 1), one task per
      selected inner chunk as the GPU batch has it: the shard index by suffix
      read + its CRC, the inner chunk's byte range + CRC, scatter."""
    from oracle import oracle as O

    lib = O._load_lib()
    cores = box_cores()

    def crc_ok(u8):
        return np.uint32(lib.oracle_crc32c(u8.ctypes.data, u8.size - 4)).tobytes() == u8[-4:].tobytes()

    def crc_blob(a):
        return np.frombuffer(bytes(O.crc32c_encode(np.ascontiguousarray(a).view(np.uint8).reshape(-1))), np.uint8)

    out = {}
    # c2 / c3: unsharded 64^3 chunks of the 256^3 array
    shape, chunks = (256, 256, 256), (64, 64, 64)
    data = W.synthetic(shape, seed=0)
    grid = list(np.ndindex(*[s // c for s, c in zip(shape, chunks)]))
    sls = {c: tuple(slice(i * k, (i + 1) * k) for i, k in zip(c, chunks)) for c in grid}
    for name, perm in (("c2_unsharded_256", None), ("c3_transpose_210", (2, 1, 0))):
        store = {c: crc_blob(data[sls[c]] if perm is None else data[sls[c]].transpose(perm)) for c in grid}
        res = np.empty(shape, np.float32)

        def read_chunk(c, store=store, res=res, perm=perm):
            raw = store[c]
            if not crc_ok(raw):
                raise ValueError("checksum")
            a = raw[:-4].view(np.float32)
            res[sls[c]] = a.reshape(chunks) if perm is None else a.reshape(tuple(chunks[p] for p in perm)).transpose(perm)

        line = _pool_rate(read_chunk, grid, data.nbytes, budget_s, cores)
        assert res.tobytes() == data.tobytes()
        line["sample"] = f"the whole 256^3 f32 array: 64 chunks of 64^3 (+crc){'' if perm is None else ', transpose (2,1,0)'}"
        out[name] = line
    del data
    # c4: 32 shards of 128^3 (32^3 inner chunks, bytes + crc32c, index at end)
    out["c4_sharded_1024"] = _sharded_port(lib, crc_ok, crc_blob, (512, 512, 256), (128, 128, 128),
                                           (32, 32, 32), np.float32, None, budget_s, cores)
    out["c4_sharded_1024"]["sample"] = ("32 of the 512 shards (512 x 512 x 256 f32, 128^3 shards of 32^3 "
                                        "inner chunks + crc), one task per shard")
    # c5: 16 shards of 256^3 int16, the 10 % inner-chunk selection
    out["c5_partial_2048"] = _sharded_port(lib, crc_ok, crc_blob, (512, 512, 1024), (256, 256, 256),
                                           (64, 64, 64), np.int16, 0.1, budget_s, cores)
    out["c5_partial_2048"]["sample"] = ("16 of the 512 shards (512 x 512 x 1024 int16, 256^3 shards of 64^3 "
                                        "inner chunks + crc), 10 % of their inner chunks (seed 1), one task "
                                        "per selected inner chunk: index suffix + CRC, chunk range + CRC")
    return out


def _sharded_port(lib, crc_ok, crc_blob, shape, shards, inner, dtype, frac, budget_s, cores):
    """_decode_partial_sync restated (sharding.py:1222-1309) over a sample
    region: frac None = every inner chunk of each shard per task (one task per
    shard), else one task per selected inner chunk."""
    rng = np.random.default_rng(0)
    if np.dtype(dtype).kind == "f":
        data = rng.standard_normal(shape, dtype=np.float32)
    else:
        data = rng.integers(-2 ** 15, 2 ** 15, shape, dtype=np.int16)
    cps = tuple(s // c for s, c in zip(shards, inner))
    n_inner = int(np.prod(cps))
    isz = n_inner * 16 + 4
    sgrid = list(np.ndindex(*[s // c for s, c in zip(shape, shards)]))
    store = {}
    for sc in sgrid:
        shard = data[tuple(slice(i * k, (i + 1) * k) for i, k in zip(sc, shards))]
        parts, index, top = [], [], 0
        for ic in np.ndindex(*cps):
            enc = crc_blob(shard[tuple(slice(i * k, (i + 1) * k) for i, k in zip(ic, inner))])
            index.append((top, enc.size))
            parts.append(enc.tobytes())
            top += enc.size
        idx = np.array(index, "<u8").reshape(-1).view(np.uint8)
        store[sc] = np.frombuffer(b"".join(parts) + crc_blob(idx).tobytes(), np.uint8)
    res = np.zeros(shape, dtype)

    def index_of(blob):
        ib = blob[-isz:]
        if not crc_ok(ib):
            raise ValueError("index checksum")
        return ib[:-4].view("<u8").reshape(n_inner, 2)

    def put(blob, idx, sc, ic):
        slot = int(np.ravel_multi_index(ic, cps))
        o, n = int(idx[slot, 0]), int(idx[slot, 1])
        raw = blob[o:o + n]
        if not crc_ok(raw):
            raise ValueError("checksum")
        reg = tuple(slice(s * k + i * c, s * k + (i + 1) * c) for s, k, i, c in zip(sc, shards, ic, inner))
        res[reg] = raw[:-4].view(dtype).reshape(inner)

    if frac is None:
        def task(sc):
            blob = store[sc]
            idx = index_of(blob)
            for ic in np.ndindex(*cps):
                put(blob, idx, sc, ic)
        tasks, nbytes = sgrid, data.nbytes
    else:
        igrid = tuple(s // c for s, c in zip(shape, inner))
        coords = W.partial_selection(igrid, frac, 1)

        def task(co):
            sc = tuple(int(c) // k for c, k in zip(co, cps))
            ic = tuple(int(c) % k for c, k in zip(co, cps))
            blob = store[sc]
            put(blob, index_of(blob), sc, ic)
        tasks = [tuple(c) for c in coords]
        nbytes = len(tasks) * int(np.prod(inner)) * np.dtype(dtype).itemsize
    line = _pool_rate(task, tasks, nbytes, budget_s, cores)
    if frac is None:
        assert res.tobytes() == data.tobytes()
    else:
        for co in tasks[:8]:
            reg = tuple(slice(c * k, (c + 1) * k) for c, k in zip(co, inner))
            assert res[reg].tobytes() == data[reg].tobytes()
    return line


def lib_sha16() -> str | None:
    """sha256[:16] of the kernel library this process loads."""
    import hashlib

    try:
        with open(os.path.join(ROOT, LIB_SO), "rb") as fh:
            return hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_traffic():
    """(HBM bytes per launch measured by the PMC passes, the library hash they
    were measured on).  The bytes are reported only when that hash is the
    library this run loads: a kernel change leaves them null, not stale."""
    try:
        with open(os.path.join(ROOT, TRAFFIC_JSON)) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    sha = d.get("lib_sha16")
    return (d.get("traffic_bytes_per_launch") if sha is not None and sha == lib_sha16() else None), sha


# ------------------------------------------------------------------------ main

HEADLINE_KERNEL = ["?"]  # the decode kernel the library launched for the headline (zhip_last_kernel)


def headline(ctx, args, weak: bool = False):
    """The headline batch -- BASELINE's 256^3 f32 array in 128^3 shards of 64^3
    inner chunks -- partitioned round-robin by shard over the ranks (strong
    scaling: the array is fixed, each of N ranks owns 8/N of its 8 shards).
    With ``weak`` the global array is (256N) x 256 x 256 and every rank owns 8
    shards (one 256^3 array's worth; reported under extra at N > 1).  Returns
    (programs, decoded bytes per step on this rank, algorithmic bytes per
    launch on this rank)."""
    import torch

    g = W.HEADLINE
    shape1, shards, inner = g["shape"], g["shards"], g["inner"]
    data = synthetic(shape1, seed=0)
    src = torch.from_numpy(data).to(ctx.device)
    rep = ctx.world if weak else 1
    if rep > 1:
        src = src.repeat(rep, 1, 1)
    shape = (shape1[0] * rep,) + shape1[1:]
    blob = 8 * (1048576 + 4) + 8 * 16 + 4
    n_shards = 8 * rep
    mine_n = len(range(ctx.rank, n_shards, ctx.world))
    progs = []
    for r in range(args.replicas):
        prog, out, mine = build_partitioned(ctx, src, shape, inner, shards, "float32", 0.0,
                                            max(mine_n, 1) * (blob + 256) + (1 << 20))
        if r == 0:  # correctness gate: every decoded byte of this rank's shards
            prog.launch()
            prog.results()
            check_regions(out, src, mine, "headline")
            from zarr_hip import _native as N
            HEADLINE_KERNEL[0] = N.lib().zhip_last_kernel().decode()
        assert len(mine) == mine_n, "round-robin by shard"
        assert prog.tables.fast and prog.tables.rows, "the headline should take the whole-row kernel"
        assert prog.index is None and prog.data.n_idx == mine_n, "index CRC checks should be fused"
        progs.append(prog)
    del src
    decoded = mine_n * int(np.prod(shards)) * 4
    encoded = mine_n * blob  # this rank's inner chunks + shard indexes
    return progs, decoded, encoded


def headline_strong(ctx, args):
    """extra.headline_strong (N > 1): BASELINE's single 256^3 array, its 8 shards
    split round-robin over the ranks (8/N per rank; strong scaling)."""
    plist, decoded, encoded = headline(ctx, args, weak=False)
    wall, kern = time_programs(plist, args.steps, args.warmup, ctx.device, ctx)
    dec = ctx.sum(decoded)
    del plist
    return _entry(dec, decoded + encoded, wall, kern, checked="bytes", scaling="strong",
                  workload="256x256x256 f32, 8/N shards of 128^3 per rank",
                  note="decoded_GiBps = the array's decoded bytes / max rank step time; "
                       "kernel_ms / hbm_frac are this rank's")


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return int(so.getsockname()[1])


def launcher_cmd(argv: list, n: int, port: int) -> list:
    """The torchrun command that runs this bench as n ranks on one node (the
    driver's own form: --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n: int, argv: list, env=None) -> int:
    """`python bench.py --gpus N` with no WORLD_SIZE in the environment: start
    the N ranks as ONE child torchrun (nothing here has touched the GPU -- a
    process that has must never exec another program on this pool) and
    return its exit code; rank 0 of the child prints the JSON line."""
    import subprocess

    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[bench] launching {n} ranks: " + " ".join(launcher_cmd(argv, n, 0)[:6]))
    return subprocess.call(launcher_cmd(argv, n, free_port()), env=e)


def rank_plan(gpus: int, env) -> str:
    """'launch' (start N ranks), 'run' (this process is a rank or the only
    one) -- or ValueError when the launcher's world size disagrees with
    --gpus."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws}: launch with matching sizes")
    return "run"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tune", type=int, default=0,
                    help="kernel ablation bits (zhip_set_tuning; measurement experiments only)")
    ap.add_argument("--eager", action="store_true",
                    help="time one host launch per step instead of a hipGraph replay")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--extra-only", action="store_true",
                    help="profiling runs (rocprofv3 per config line): the extra configs only, no headline")
    ap.add_argument("--no-host-legs", action="store_true",
                    help="profiling runs: skip the host-store legs (c5_host, the example's host reads, C1's host "
                         "round trip), whose launches share kernels with the device-resident lines")
    ap.add_argument("--extra-cpu", default="cpu",
                    help="'cpu': time the CPU port of every config line too (N=1, rank 0); '' to skip")
    ap.add_argument("--extra", default="c1,c2,c3,c4,c5,enc,e2e,call,cpp",
                    help="extra configs (subset of c1,c2,c3,c4,c5,enc,e2e,call,cpp, or ''); c4/c5 run "
                         "partitioned at every N, the others at N=1")
    args = ap.parse_args()
    if rank_plan(args.gpus, os.environ) == "launch":
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if os.environ.get("ZHIP_BENCH_DRY") == "1":  # launcher test hook (tests/test_bench_launcher.py)
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"n_gpus": int(os.environ.get("WORLD_SIZE", "1")), "gpus_arg": args.gpus}))
        return

    import torch

    ctx = Ctx()
    device = ctx.device
    if args.tune:
        from zarr_hip import _native as N

        if not N.tuning_build():
            raise SystemExit("--tune needs the tuning build (make -C zarr-python_amd tune; "
                             "ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB=zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so)")
        N.check(N.lib().zhip_set_tuning(2, args.tune), "zhip_set_tuning")
    if args.extra_only:  # rocprofv3 runs of the config lines (profiles/r06/final/)
        res = {"extra": extra_configs(ctx, args), "lib_sha16": lib_sha16(), "steps": args.steps}
        if ctx.rank == 0:
            print(json.dumps(res), flush=True)
        return
    log(f"[bench] building {args.replicas} replicas of the headline batch on {device} "
        f"(rank {ctx.rank} of {ctx.world})")
    plist, decoded, encoded = headline(ctx, args, weak=True)

    if args.eager:
        stream = torch.cuda.current_stream(device)
        sh = int(stream.cuda_stream)
        for i in range(args.warmup):
            plist[i % len(plist)].launch(sh)
        ctx.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        kern_s = eager_kernel_times(plist, args.steps, device)
        wall = time.perf_counter() - t0
        ctx.barrier()
        for p in plist:
            p.results()
        span_s = float(np.sum(kern_s))
        wall_max = ctx.max(wall)
    else:
        wall, wall_max, span_s = graph_steps(plist, args.steps, args.warmup, device, ctx)
        # per-launch durations of the same kernel, eager (for the rocprof cross-check)
        kern_s = eager_kernel_times(plist, args.steps, device)
        for p in plist:
            p.results()

    total_decoded = ctx.sum(args.steps * decoded)  # every rank's own shards of the one array
    value = total_decoded / wall_max / GIB
    # kernel time per launch over the timed region: event span on the launch
    # stream / steps (includes the graph's inter-launch gaps, so it is an upper
    # bound on the kernel duration and `achieved` a lower bound)
    avg_kern_s = span_s / args.steps
    traffic, traffic_sha = pmc_traffic()
    achieved = (encoded + decoded) / avg_kern_s / 1e9
    res = {
        "metric": "decoded GiB/s (device-resident), sharded 256^3 f32 64^3 chunks, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": ctx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0 standard-normal f32, planted NaN payload and -0.0)",
        "config": {
            "workload": "sharded 256^3 float32, 64^3 chunks (128^3 shards of 8 inner chunks; inner "
                        "codecs bytes(little)+crc32c, index bytes+crc32c at end), device-resident "
                        "decode of the full array per step (64 inner chunks + 8 index checks; one "
                        "launch per GPU), 4 rotating replicas per GPU; at N GPUs the batch is the "
                        "(256N)x256x256 array of 8N shards split round-robin by shard (8 shards "
                        "per rank: weak scaling; the strong split is extra.headline_strong)",
            "chunks_per_step": 64 * ctx.world, "shards_per_step": 8 * ctx.world,
            "headline_scaling": "weak since round 4: each of the N ranks decodes its own 8 shards "
                                "(extra.headline_strong splits BASELINE's one 256^3 array 8/N shards "
                                "per rank, the round-3 definition)",
            "decoded_bytes_per_step": int(ctx.sum(decoded)),
            "encoded_bytes_per_step": int(ctx.sum(encoded)),
            "parallelism": f"shard-partitioned x{ctx.world} (weak, no collective on the data path)",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_lib_sha16": traffic_sha, "lib_sha16": lib_sha16(),
            "traffic_source": TRAFFIC_JSON + " (FETCH_SIZE x2 + WRITE_SIZE per launch from "
                              "separate rocprofv3 --pmc passes of this command)",
            "kernel": f"zhip::{HEADLINE_KERNEL[0]}<CRC,4,noswap> (zhip_decode_mapped)",
            "kernel_ms_avg": round(avg_kern_s * 1e3, 5),
            "kernel_ms_eager_mean": round(float(np.mean(kern_s)) * 1e3, 5),
            "timing": "eager launches" if args.eager else
                      "hipGraph replay of the K launches; kernel_ms_avg = event span / K",
            "algorithmic_bytes_per_launch": encoded + decoded,
        },
    }
    del plist
    torch.cuda.empty_cache()
    if args.extra:
        log("[bench] extra configs " + args.extra)
        res["extra"] = extra_configs(ctx, args)
        if ctx.world > 1:
            res["extra"]["headline_strong"] = headline_strong(ctx, args)
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        log("[bench] cpu baseline")
        g = W.HEADLINE
        res["cpu_baseline"] = cpu_baseline(synthetic(g["shape"], seed=0), g["shape"], g["inner"],
                                           g["shards"], args.cpu_budget)
        if args.extra and "cpu" in args.extra_cpu:
            log("[bench] cpu ports of the config lines")
            for name, port in cpu_config_ports(args.cpu_budget / 3).items():
                if name in res.get("extra", {}):
                    res["extra"][name]["cpu_port"] = port
    if ctx.rank == 0:
        print(json.dumps(res), flush=True)
    if ctx.distributed:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()

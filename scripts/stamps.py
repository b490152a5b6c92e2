#!/usr/bin/env python
"""Per-workgroup phase timeline of k_decode_pair on the headline batch
(diagnostics: ablation bit 1024 makes every workgroup record s_memrealtime
stamps; see zhip_debug_stamps).  Prints one JSON line per phase with quantiles
(microseconds, relative to the earliest workgroup start), plus the number of
workgroups resident per CU over time.

Slots: 0 start, 1 loads issued, 2 tables + barrier, 3 unit A stored,
4 unit B stored, 5 CRC lookups done, 6 run end (atomic returned), 7 exit.
k_decode_il (the default since round 3): 0 start, 1 loads issued, 2 tables
+ barrier, 3 stores and Horner steps done, 4 reduced contribution ready
(publication issued right after), 7 exit.
"""
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


def main():
    import torch

    from zarr_hip import _native as N

    dev = torch.device("cuda:0")
    shape, chunks, shards = (256, 256, 256), (64, 64, 64), (128, 128, 128)
    data = torch.from_numpy(bench.synthetic(shape)).to(dev)
    tune = int(os.environ.get("TUNE", "0"))
    progs = []
    # WORLD=n: only rank 0's shards of an n-way round-robin split (the bench's
    # strong-scaled headline at n GPUs), decoded into a full-shape out
    world = int(os.environ.get("WORLD", "1"))
    from zarr_hip import buffer, parallel

    for _ in range(4):
        codecs = [bench.LE] if os.environ.get("NOCRC") else [bench.LE, bench.CRC]
        arr = bench.build_replica(dev, data, shape, chunks, codecs, shards=shards)
        if world == 1:
            progs.append(arr.prepare_read((Ellipsis,))[0])
        else:
            batch, out_shape = arr.batch_info((Ellipsis,))
            out = buffer.empty(out_shape, "float32", dev)
            progs.append(arr.codec_pipeline.prepare_read(parallel.rank_batch(batch, world, 0), out))
    sh = int(torch.cuda.current_stream(dev).cuda_stream)
    N.lib().zhip_set_tuning(2, 1024 | tune)
    N.lib().zhip_set_tuning(6, int(os.environ.get("ARM", "0")))  # a kernel arm (k_decode_ilw: 26 / 27)
    for i in range(8):
        progs[i % 4].launch(sh)
    torch.cuda.synchronize(dev)
    N.lib().zhip_set_tuning(2, 0)
    N.lib().zhip_set_tuning(6, 0)
    for p in progs:
        p.results()
    il = N.lib().zhip_last_kernel().decode().startswith("k_decode_il")
    n_wg = (2048 if (tune & 128 or il) else 1024) // world
    buf = np.zeros(n_wg * 8, np.uint64)
    N.check(N.lib().zhip_debug_stamps(buf.ctypes.data, n_wg), "zhip_debug_stamps")
    st = buf.reshape(n_wg, 8)
    hw = (st[:, 0] >> np.uint64(32)).astype(np.int64)
    t = (st & np.uint64(0xFFFFFFFF)).astype(np.int64)
    t0 = t[:, 0].min()
    rel = (t - t0) * 0.01  # 100 MHz -> us
    if os.environ.get("STAMPS_OUT"):  # every workgroup's stamps and hardware ids, for offline analysis
        np.savez(os.environ["STAMPS_OUT"], rel=rel, hw=(st[:, 0] >> np.uint64(32)).astype(np.int64))
    names = ["start", "loads_issued", "tables_barrier", "A_stored", "B_stored", "runend_barrier", "V_ready", "exit"]
    if il:  # k_decode_il's slots (TUNE variant)
        names = ["start", "loads_issued", "tables_barrier", "stored_hornered", "V_ready", "-", "-", "exit"]
    for i, nm in enumerate(names):
        if rel[:, i].min() < -1e3:
            continue  # slot not recorded by this variant
        q = np.percentile(rel[:, i], [0, 10, 50, 90, 100])
        print(json.dumps({"phase": nm, "us_q0_10_50_90_100": [round(float(x), 2) for x in q]}))
    for a, b in [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7)]:
        d = rel[:, b] - rel[:, a]
        if np.abs(d).max() > 1e4:
            continue
        q = np.percentile(d, [10, 50, 90])
        print(json.dumps({"delta": f"{names[a]}->{names[b]}", "us_q10_50_90": [round(float(x), 2) for x in q]}))
    # the slowest 5 % of workgroups (the kernel's tail): their phase medians
    tail = rel[:, 7] >= np.percentile(rel[:, 7], 95)
    print(json.dumps({"tail_wgs": int(tail.sum()), "phase_medians_us": {
        nm: round(float(np.median(rel[tail, i])), 2) for i, nm in enumerate(names)
        if rel[:, i].min() > -1e3}}))
    xcc = (hw >> 24) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    per_cu = np.bincount(np.unique(cu_key, return_inverse=True)[1])
    print(json.dumps({"wg_per_xcc": np.bincount(xcc, minlength=8).tolist(),
                      "distinct_cus": int(len(per_cu)),
                      "wg_per_cu_histogram": {int(k): int(v) for k, v in zip(*np.unique(per_cu, return_counts=True))},
                      "kernel_span_us": round(float(rel[:, 7].max()), 2)}))
    # end time vs number of workgroups sharing the CU
    n_on_cu = per_cu[np.unique(cu_key, return_inverse=True)[1]]
    for k in sorted(set(n_on_cu.tolist())):
        print(json.dumps({"wgs_on_cu": int(k), "exit_us_median": round(float(np.median(rel[n_on_cu == k, 7])), 2),
                          "exit_us_max": round(float(np.max(rel[n_on_cu == k, 7])), 2)}))


if __name__ == "__main__":
    main()

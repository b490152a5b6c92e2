#!/usr/bin/env python
"""Kernel ablation / tuning matrix for the C2 decode (interleaved rounds in ONE
process, cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per arm:
median / min kernel ms over rounds, algorithmic GB/s, plus a torch D2D copy of
the same bytes as the practical ceiling."""

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
    shape, chunks = (256, 256, 256), (64, 64, 64)
    data = bench.synthetic(shape)
    progs = []
    R = int(os.environ.get("REPLICAS", "4"))
    for _ in range(R):
        arr = bench.build_c2_replica(dev, data, shape, chunks)
        progs.append(arr.prepare_read((Ellipsis,)))
    stream = torch.cuda.current_stream(dev)
    sh = int(stream.cuda_stream)
    alg = 64 * (1048576 + 4) + data.nbytes

    def time_arm(launch, n=20):
        for i in range(5):
            launch(i)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(n)]
        for i, (a, b) in enumerate(evs):
            a.record(stream)
            launch(i)
            b.record(stream)
        torch.cuda.synchronize(dev)
        return [a.elapsed_time(b) for a, b in evs]

    arms = []
    grids = [int(g) for g in os.environ.get("GRIDS", "0").split(",")]
    ablations = [int(a) for a in os.environ.get("ABLATIONS", "0,1").split(",")]
    for g in grids:
        for ab in ablations:
            arms.append(("decode", g, ab))
    # K (blocks per thread per unit) variants: separate plans of the same tables
    from zarr_hip import pipeline as PL
    kvar = {}
    for kb in [int(k) for k in os.environ.get("BLOCKS", "").split(",") if k]:
        N.lib().zhip_set_tuning(3, kb)
        PL._PLAN_CACHE.clear()
        kvar[kb] = []
        for prog, out in progs:
            t = prog.tables
            kvar[kb].append(PL.DecodeLaunch(t.layout, t.chunks, t.sels, prog.data.src,
                                            prog.data.src_size, out, True, dev, rows=t.rows))
        arms.append(("decodeK%d" % kb, 0, 0))
    N.lib().zhip_set_tuning(3, 0)
    PL._PLAN_CACHE.clear()
    srcs = [torch.empty(data.nbytes, dtype=torch.uint8, device=dev) for _ in range(R)]
    dsts = [torch.empty(data.nbytes, dtype=torch.uint8, device=dev) for _ in range(R)]
    # no-CRC twin of the same batch: same kernel structure, no tables / atomics
    from zarr_hip.pipeline import DecodeLaunch
    nocrc, nocrc_rows, fastpath, nocrc_pred, crc_nopred = [], [], [], [], []
    for prog, out in progs:
        t = prog.tables
        L2 = type(t.layout).from_buffer_copy(bytes(t.layout))
        L2.flags = L2.flags & ~N.LF_CRC
        ch = t.chunks.copy()
        ch["src_len"] -= 4
        nocrc.append(DecodeLaunch(L2, ch, t.sels, prog.data.src, prog.data.src_size, out, True, dev))
        nocrc_rows.append(DecodeLaunch(L2, ch, t.sels, prog.data.src, prog.data.src_size, out, True, dev,
                                       rows=True))
        fastpath.append(DecodeLaunch(t.layout, t.chunks, t.sels, prog.data.src, prog.data.src_size, out,
                                     True, dev, rows=False))
        # prediction on / off for both twins (the decode arm uses the program's own setting)
        nocrc_pred.append(DecodeLaunch(L2, ch, t.sels, prog.data.src, prog.data.src_size, out, True, dev,
                                       rows=True, predict=t.predict))
        crc_nopred.append(DecodeLaunch(t.layout, t.chunks, t.sels, prog.data.src, prog.data.src_size, out,
                                       True, dev, rows=True))
    # write-locality probe: the same bytes in chunks of whole output planes
    # (every unit writes contiguous 32 KiB instead of 256-byte rows at 1 KiB stride)
    alt = {}
    for name in [a for a in os.environ.get("ALT_CHUNKS", "").split(",") if a]:
        ck = tuple(int(x) for x in name.split("x"))
        alt[name] = [bench.build_c2_replica(dev, data, shape, ck).prepare_read((Ellipsis,))[0]
                     for _ in range(R)]
        arms.append(("alt_" + name, 0, 0))
    arms.append(("fastpath", 0, 8))
    for g in grids:
        arms.append(("nocrc_rows", g, 0))
    if progs[0][0].tables.predict is not None:
        arms.append(("nocrc_pred", 0, 0))
        arms.append(("crc_nopred", 0, 0))
    arms.append(("torch_copy", 0, 0))
    arms.append(("torch_read_sum", 0, 0))
    results = {a: [] for a in arms}
    rounds = int(os.environ.get("ROUNDS", "5"))
    for _ in range(rounds):
        for arm in arms:
            kind, g, ab = arm
            if kind == "decode":
                N.lib().zhip_set_tuning(1, g)
                N.lib().zhip_set_tuning(2, ab)
                ms = time_arm(lambda i: progs[i % R][0].launch(sh))
            elif kind.startswith("decodeK"):
                N.lib().zhip_set_tuning(1, g)
                N.lib().zhip_set_tuning(2, 0)
                kl = kvar[int(kind[7:])]
                ms = time_arm(lambda i: kl[i % R].launch(sh))
            elif kind in ("nocrc", "nocrc_rows", "fastpath", "nocrc_pred", "crc_nopred"):
                N.lib().zhip_set_tuning(1, g)
                N.lib().zhip_set_tuning(2, ab)
                L = {"nocrc": nocrc, "nocrc_rows": nocrc_rows, "fastpath": fastpath, "nocrc_pred": nocrc_pred,
                     "crc_nopred": crc_nopred}[kind]
                ms = time_arm(lambda i: L[i % R].launch(sh))
            elif kind.startswith("alt_"):
                N.lib().zhip_set_tuning(1, 0)
                N.lib().zhip_set_tuning(2, 0)
                L = alt[kind[4:]]
                ms = time_arm(lambda i: L[i % R].launch(sh))
            elif kind == "torch_copy":
                ms = time_arm(lambda i: dsts[i % R].copy_(srcs[i % R]))
            else:
                ms = time_arm(lambda i: srcs[i % R].view(torch.int32).sum())
            results[arm].extend(ms)
    N.lib().zhip_set_tuning(1, 0)
    N.lib().zhip_set_tuning(2, 0)
    for p, out in progs:
        p.data.d_ws.zero_()
        p.launch(sh)
        p.results()
        assert p.tables.rows, "C2 should take k_decode_rows"
        assert out.view(torch.int32).cpu().numpy().tobytes() == data.view(np.int32).tobytes()
    for kb, kl in kvar.items():
        for i, l in enumerate(kl):
            l.launch(sh)
            st = l.statuses()
            assert (st["code"] == 0).all(), f"K={kb}: bad statuses"
            assert progs[i][1].view(torch.int32).cpu().numpy().tobytes() == data.view(np.int32).tobytes()
    for arm, ms in results.items():
        kind, g, ab = arm
        med = float(np.median(ms))
        byts = alg if kind != "torch_read_sum" else data.nbytes
        if kind == "torch_copy":
            byts = 2 * data.nbytes
        print(json.dumps({"arm": kind, "grid": g, "ablation": ab, "ms_med": round(med, 4),
                          "ms_min": round(float(np.min(ms)), 4),
                          "GBps_med": round(byts / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Graph-timed kernel arms on the headline batch (measurement only).

Every arm is captured as a hipGraph of REPS launches rotating over 4 replicas
(so the Infinity Cache cannot serve re-reads and host launch gaps are out of
the number) and replayed; arms are interleaved over ROUNDS rounds in ONE
process.  Arms: the production decode, decode with tuning bits (TUNES, comma
list; ablations that skip work give invalid results and are timing-only), the
no-CRC twin of the same batch, and the 32 KiB-span nontemporal copy of the
same bytes (scripts/copybench) as the practical ceiling.  One JSON line per
arm: min / median microseconds per launch and the HBM fraction of the
algorithmic bytes."""

import ctypes
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
    g = W.HEADLINE if cfg == "headline" else W.C4
    shape, shards, inner = g["shape"], g["shards"], g["inner"]
    if cfg == "headline":
        data = torch.from_numpy(W.synthetic(shape)).to(dev)
    else:
        gen = torch.Generator(device=dev).manual_seed(0)
        data = torch.randn(shape, generator=gen, device=dev, dtype=torch.float32)
    R = 4 if cfg == "headline" else 2
    reps = int(os.environ.get("REPS", "20" if cfg == "headline" else "4"))
    crc = [bench.build_replica(dev, data, shape, inner, [W.LE, W.CRC], shards=shards).prepare_read((Ellipsis,))
           for _ in range(R)]
    nocrc = [bench.build_replica(dev, data, shape, inner, [W.LE], shards=shards).prepare_read((Ellipsis,))
             for _ in range(R)] if cfg == "headline" else []
    n_inner = int(np.prod([s // i for s, i in zip(shape, inner)]))
    n_shards = int(np.prod([s // i for s, i in zip(shape, shards)]))
    cps = n_inner // n_shards
    alg = n_inner * (int(np.prod(inner)) * 4 + 4) + n_shards * (cps * 16 + 4) + data.numel() * 4
    cb = ctypes.CDLL(os.path.join(ROOT, "scripts", "copybench", "libcopybench.so"))
    cb.cb_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n = data.numel() * 4
    Rc = R if cfg == "headline" else 1
    srcs = [torch.empty(n, dtype=torch.uint8, device=dev).fill_(3) for _ in range(Rc)]
    dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(Rc)]

    def graph_of(launch):
        s = torch.cuda.Stream(dev)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for i in range(reps):
                launch(i, int(s.cuda_stream))
        return gr

    arms = {}
    tunes = [int(x) for x in os.environ.get("TUNES", "0").split(",") if x != ""]
    for tb in tunes:
        N.lib().zhip_set_tuning(2, tb)  # read at launch time: captured into the graph's params
        arms[f"decode_tune{tb}"] = graph_of(lambda i, sh: crc[i % R][0].launch(sh))
    N.lib().zhip_set_tuning(2, 0)
    if nocrc:
        arms["nocrc_twin"] = graph_of(lambda i, sh: nocrc[i % R][0].launch(sh))
    arms["copy_32k"] = graph_of(lambda i, sh: cb.cb_copy(srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(), n,
                                                         32 << 10, 8, 1, 1, ctypes.c_void_p(sh)))
    # default-policy loads, nontemporal stores (the better copy policy at 64 MiB)
    arms["copy_8k_ldef"] = graph_of(lambda i, sh: cb.cb_copy(srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(), n,
                                                             8 << 10, 2, 1, 3, ctypes.c_void_p(sh)))
    # interleaved spans (k_copy_il: workgroup j of a group of S takes steps j,
    # j + S, ...) and wave-contiguous spans (k_copy_wave), default loads + nt stores
    cb.cb_copy_il.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                              ctypes.c_int, ctypes.c_void_p]
    cb.cb_copy_wave.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p]
    for S, K in ((8, 8), (4, 8), (8, 16), (16, 16)):
        arms[f"copy_il_S{S}_K{K}"] = graph_of(lambda i, sh, S=S, K=K: cb.cb_copy_il(
            srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(), n, K, S, 3, ctypes.c_void_p(sh)))
    arms["copy_4k_ldef"] = graph_of(lambda i, sh: cb.cb_copy(srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(), n,
                                                             4 << 10, 1, 1, 3, ctypes.c_void_p(sh)))
    arms["copy_32k_k8_ldef"] = graph_of(lambda i, sh: cb.cb_copy(srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(),
                                                                 n, 32 << 10, 8, 1, 3, ctypes.c_void_p(sh)))
    arms["copy_wave_k8"] = graph_of(lambda i, sh: cb.cb_copy_wave(srcs[i % Rc].data_ptr(), dsts[i % Rc].data_ptr(),
                                                                  n, 8, 3, ctypes.c_void_p(sh)))
    # the headline's access pattern without codec work (scripts/copybench k_scatter)
    cb.cb_scatter.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    ssrc = [torch.empty(64 * 1048580 + 64, dtype=torch.uint8, device=dev).fill_(5) for _ in range(R)] \
        if cfg == "headline" else []
    for cs, nm in (((1048576, "al"), (1048580, "mis")) if cfg == "headline" else ()):
        for u in (1, 2, 11, 12, 22):
            arms[f"scatter_{nm}_u{u}"] = graph_of(
                lambda i, sh, cs=cs, u=u: cb.cb_scatter(ssrc[i % R].data_ptr(), dsts[i % R].data_ptr(), cs, u,
                                                        ctypes.c_void_p(sh)))
    # the sharded decode's access pattern without codec work (scripts/copybench
    # k_scatter_g): source chunks at the shard packing's stride, 4 ce-byte rows
    cb.cb_scatter_geo.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    ce = inner[0]
    cstride = ce ** 3 * 4 + 4
    Rg = R if cfg == "headline" else 1
    srcg = [torch.empty(n_inner * cstride + 64, dtype=torch.uint8, device=dev).fill_(5) for _ in range(Rg)]
    for nm, mode, K, S in (("nat_K1", 0, 1, 1), ("nat_K2", 0, 2, 1), ("nat_K4", 0, 4, 1), ("nat_K8", 0, 8, 1),
                           ("nat_K16", 0, 16, 1), ("il_S4_K8", 1, 8, 4), ("il_S8_K8", 1, 8, 8),
                           ("xq_K4", 2, 4, 1), ("xq_K8", 2, 8, 1), ("xq_K16", 2, 16, 1), ("xw_K8", 3, 8, 1)):
        arms[f"scatterg_{nm}"] = graph_of(lambda i, sh, mode=mode, K=K, S=S: cb.cb_scatter_geo(
            srcg[i % Rg].data_ptr(), dsts[i % Rg].data_ptr(), cstride, ce, mode, K, S, ctypes.c_void_p(sh)))
    if os.environ.get("COPIES", "1") == "0":
        arms = {k: v for k, v in arms.items() if not (k.startswith("copy") or k.startswith("scatter_"))
                or k in ("copy_4k_ldef", "copy_32k_k8_ldef")}
    res = {k: [] for k in arms}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for k, gr in arms.items():
            gr.replay()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            gr.replay()
            b.record()
            torch.cuda.synchronize(dev)
            res[k].append(a.elapsed_time(b) * 1e3 / reps)
    for p, _ in crc:
        p.data.d_ws.zero_()
        p.data.d_status.zero_()
        p.launch()
        p.results()
    if not torch.equal(crc[0][1].view(torch.int32), data.view(torch.int32)):
        raise SystemExit("graphbench: production decode output differs")
    for k, v in res.items():
        byt = 2 * n if (k.startswith("copy") or k.startswith("scatter")) else alg
        print(json.dumps({"arm": k, "us_min": round(min(v), 2), "us_med": round(float(np.median(v)), 2),
                          "hbm_frac_min": round(byt / (min(v) * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()

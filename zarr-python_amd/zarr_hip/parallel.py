"""Multi-GPU partitioning: one process per GPU, chunks split across ranks.

Chunks (or shards) are independent — the reference's read_sync already maps
them over a pool with disjoint out selections (src/zarr/core/codec_pipeline.py:
1104-1109, 1169-1171) — so a batch is partitioned into per-rank sub-batches
with no collective on the data path.  RCCL (torch.distributed "nccl") is only
used by callers for barriers / timing reductions, and by `gather_to` for an
optional post-step gather of results onto one rank.
"""

from __future__ import annotations

import numpy as np


def partition(n_items: int, world: int, rank: int, mode: str = "round_robin") -> np.ndarray:
    """Indices of the batch items owned by `rank` (disjoint, covering)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    idx = np.arange(int(n_items))
    if mode == "round_robin":
        return idx[rank::world]
    if mode == "contiguous":
        per, rem = divmod(int(n_items), world)
        start = rank * per + min(rank, rem)
        return idx[start: start + per + (1 if rank < rem else 0)]
    raise ValueError(f"unknown partition mode {mode!r}")


def rank_batch(batch: list, world: int, rank: int, mode: str = "round_robin") -> list:
    """The rank's sub-batch of a CodecPipeline batch_info list."""
    return [batch[i] for i in partition(len(batch), world, rank, mode)]


def read_partitioned(array, selection, world: int, rank: int, out=None, mode: str = "round_robin"):
    """Each rank decodes only its chunks of `selection` into its own device
    `out` (full selection shape; the other ranks' regions are left untouched).
    Returns (out, results)."""
    import torch

    from . import buffer

    batch, out_shape = array.batch_info(selection)
    mine = rank_batch(batch, world, rank, mode)
    if out is None:
        dev = torch.device("cuda", torch.cuda.current_device())
        out = buffer.empty(out_shape, array.metadata.dtype, dev, array.config.order)
    if not mine:
        return out, ()
    return out, array.codec_pipeline.read_sync(mine, out)


def owned_regions(array, selection, world: int, rank: int, mode: str = "round_robin"):
    """Out selections owned by `rank` (for assembling / checking partitioned reads)."""
    batch, _ = array.batch_info(selection)
    return [batch[i][3] for i in partition(len(batch), world, rank, mode)]


# ------------------------------------------------------------ one process, N GPUs
class DeviceGroup:
    """Several GPUs driven from ONE process (a zarr caller's ``arr[...]`` has no
    process group): a batch is split round-robin by item (chunk or shard, as
    BASELINE's C4 wording) over ``devices``; each device stages, plans and
    decodes its own sub-batch on its own stream from its own host thread into
    its own ``out`` (full selection shape; only its items' regions are
    written), so the devices never exchange data.  This is the reference's
    disjoint-output pool map (src/zarr/core/codec_pipeline.py:1104-1109,
    1169-1171) with a GPU per worker.  ``gather`` assembles the regions onto
    one device afterwards (peer copies over xGMI), outside any timed decode.

    Items whose bytes sit in host memory are staged to the device that decodes
    them (every device's H2D on its own copy stream: the node's PCIe links in
    parallel); items in a DeviceStore on another device are copied device to
    device.  A device may be listed twice (devices=[0, 0] runs two workers on
    one GPU: the test of this path on a one-GPU box)."""

    def __init__(self, devices, mode: str = "round_robin"):
        import torch

        if not devices:
            raise ValueError("DeviceGroup needs at least one device")
        self.devices = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in devices]
        self.mode = mode
        self.streams = []
        for d in self.devices:
            with torch.cuda.device(d):
                self.streams.append(torch.cuda.Stream(d))
        from concurrent.futures import ThreadPoolExecutor

        self._pool = ThreadPoolExecutor(max_workers=len(self.devices), thread_name_prefix="zarr_hip_dev")

    def _map(self, fn):
        futs = [self._pool.submit(fn, i) for i in range(len(self.devices))]
        return [f.result() for f in futs]

    def prepare_read(self, pipeline, batch_info, out_shape, dtype, order: str = "C", outs=None) -> "GroupProgram":
        """Plan every device's sub-batch (tables uploaded, staging begun).
        ``outs``: one tensor per device (full selection shape) or None (each
        allocated on its device)."""
        import torch

        from . import buffer
        from .pipeline import normalize_batch

        batch = normalize_batch(batch_info)
        W = len(self.devices)
        parts = [partition(len(batch), W, r, self.mode) for r in range(W)]

        def plan(i):
            dev = self.devices[i]
            with torch.cuda.device(dev), torch.cuda.stream(self.streams[i]):
                out = outs[i] if outs is not None else buffer.empty(out_shape, dtype, dev, order)
                idx = parts[i]
                prog = pipeline.prepare_read([batch[j] for j in idx], out) if len(idx) else None
                return prog, out, idx

        return GroupProgram(self, self._map(plan), len(batch))

    def read_sync(self, pipeline, batch_info, out_shape, dtype, order: str = "C", outs=None):
        """(per-device outs, per-item GetResults in batch order)."""
        prog = self.prepare_read(pipeline, batch_info, out_shape, dtype, order, outs)
        prog.launch()
        return prog.outs, prog.results()


class GroupProgram:
    """Planned per-device reads of a DeviceGroup: launch() starts every
    device's decode from its own thread on its own stream; results()
    synchronises all of them and returns statuses in batch order."""

    def __init__(self, group: DeviceGroup, parts: list, n_items: int):
        self.group = group
        self.parts = parts  # [(DecodeProgram | None, out, item indices)]
        self.n_items = n_items

    @property
    def outs(self) -> list:
        return [p[1] for p in self.parts]

    def launch(self) -> None:
        import torch

        g = self.group

        def go(i):
            prog = self.parts[i][0]
            if prog is None:
                return
            with torch.cuda.device(g.devices[i]):
                prog.launch(int(g.streams[i].cuda_stream))

        g._map(go)

    def synchronize(self) -> None:
        for s in self.group.streams:
            s.synchronize()

    def results(self) -> tuple:
        import torch

        g = self.group
        out: list = [None] * self.n_items

        def res(i):
            prog, _, idx = self.parts[i]
            if prog is None:
                return
            g.streams[i].synchronize()
            with torch.cuda.device(g.devices[i]), torch.cuda.stream(g.streams[i]):
                for j, r in zip(idx, prog.results()):
                    out[j] = r

        g._map(res)
        return tuple(out)

    def gather(self, batch_info, into) -> None:
        """Copy every device's item regions into ``into`` (any device): the
        optional post-step gather, outside the decode.  A device whose items
        form bands of the out along its outermost dim that no other device's
        items touch, and tile those bands completely, sends each band in ONE
        copy (a contiguous range of a C or F out: one peer copy over xGMI);
        otherwise its items go one region each, so regions of `into` that no
        item selects are left alone.
        The copies run asynchronously on the receiving device's stream and
        are waited for once."""
        import torch

        from .pipeline import normalize_batch

        batch = normalize_batch(batch_info)
        self.synchronize()
        dim = outer_dim(into.stride(), tuple(into.shape))
        owner = item_bands(batch, [idx for _, _, idx in self.parts], dim)
        stream = torch.cuda.current_stream(into.device)
        with torch.cuda.stream(stream):
            for (prog, out, idx), spans in zip(self.parts, owner):
                if out.device == into.device and out.data_ptr() == into.data_ptr():
                    continue
                if spans is not None:  # one copy per band only where the part's items tile it
                    band = sum(into.narrow(dim, lo, hi - lo).numel() for lo, hi in spans)
                    if sum(_cells(tuple(batch[j][3])) for j in idx) != band:
                        spans = None  # (regions no item writes hold garbage in the part's out)
                if spans is not None:
                    for lo, hi in spans:
                        into.narrow(dim, lo, hi - lo).copy_(out.narrow(dim, lo, hi - lo), non_blocking=True)
                else:
                    for j in idx:
                        osel = tuple(batch[j][3])
                        into[osel].copy_(out[osel], non_blocking=True)
        stream.synchronize()


# ------------------------------------------- a pipeline over several devices
def outer_dim(strides, shape) -> int:
    """The out dim with the largest stride among dims longer than 1 (dim 0 of
    a C-order array, the last of an F-order one): bands along it are
    contiguous byte ranges of the out.  0 for a 0-d out (a scalar selection):
    device_bands / item_bands find no slice there, so nothing is banded."""
    if not shape:
        return 0
    dims = [d for d in range(len(shape)) if shape[d] > 1] or [0]
    return max(dims, key=lambda d: abs(int(strides[d])))


def device_bands(batch: list, n_dev: int, dim: int):
    """Split a batch into at most ``n_dev`` groups of consecutive bands of the
    out along ``dim`` (every item's out selection on ``dim`` is one band
    [start, stop); items of a band stay together), balanced by item count.
    Returns [(lo, hi, item indices)] or None when the selections do not form
    bands (an int or stepped out selection on ``dim``)."""
    bands: dict = {}
    for j, it in enumerate(batch):
        osel = tuple(it[3])
        if dim >= len(osel) or not isinstance(osel[dim], slice) or (osel[dim].step or 1) != 1:
            return None
        s = osel[dim]
        bands.setdefault((int(s.start or 0), int(s.stop)), []).append(j)
    keys = sorted(bands)
    for (a0, b0), (a1, b1) in zip(keys, keys[1:]):
        if a1 < b0:
            return None  # overlapping bands: not a chunk grid projection
    total = len(batch)
    groups, cur, acc = [], [], 0
    for k in keys:
        cur.append(k)
        acc += len(bands[k])
        if len(groups) < n_dev - 1 and acc * n_dev >= total * (len(groups) + 1):
            groups.append(cur)
            cur = []
    if cur:
        groups.append(cur)
    return [(g[0][0], g[-1][1], [j for k in g for j in bands[k]]) for g in groups]


def item_bands(batch: list, parts: list, dim: int) -> list:
    """Per part (a list of item indices): its items' maximal runs of touching
    bands [lo, hi) along ``dim`` -- or None for a part whose items are not
    unit-step slices there or whose runs overlap another part's items (then
    its regions move one item at a time)."""
    spans_of = []
    for idx in parts:
        iv = []
        for j in idx:
            osel = tuple(batch[j][3])
            s = osel[dim] if dim < len(osel) else None
            if not isinstance(s, slice) or (s.step or 1) != 1:
                iv = None
                break
            iv.append((int(s.start or 0), int(s.stop)))
        if iv is None:
            spans_of.append(None)
            continue
        iv.sort()
        runs: list = []
        for a, b in iv:
            if runs and a <= runs[-1][1]:
                runs[-1][1] = max(runs[-1][1], b)
            else:
                runs.append([a, b])
        spans_of.append([tuple(r) for r in runs])
    out = []
    for i, sp in enumerate(spans_of):
        if sp is None:
            out.append(None)
            continue
        clash = False
        for k, other in enumerate(spans_of):
            if k == i:
                continue
            if other is None:
                clash = True  # unknown extents elsewhere: stay per item
                break
            for a, b in sp:
                if any(a < d and c < b for c, d in other):
                    clash = True
                    break
            if clash:
                break
        out.append(None if clash else sp)
    return out


def item_device(it) -> int | None:
    """The GPU whose HBM already holds an item's encoded bytes (a path into a
    DeviceStore, a getter over a DeviceRef), None for host-resident bytes."""
    from .store import DeviceRef, DeviceStore

    bg = it[0]
    st = getattr(bg, "store", None)
    if isinstance(st, DeviceStore):
        return int(st.device.index or 0)
    v = getattr(bg, "value", None)
    if isinstance(v, DeviceRef):
        return int(v.arena.device.index or 0)
    return None


def placement(batch: list, out_device: int | None) -> dict | None:
    """Where each item decodes when some of the batch's bytes are already in
    HBM: every device-resident item on the GPU that holds it (decoding there
    moves no encoded bytes between GPUs), host-resident items with the out's
    device (or the device holding most items).  {device: [item indices]}, or
    None when every item's bytes are in host memory (then the batch splits
    into bands over all the pipeline's devices)."""
    locs = [item_device(it) for it in batch]
    held = [d for d in locs if d is not None]
    if not held:
        return None
    if out_device is not None and out_device in held:
        home = out_device
    else:
        home = max(set(held), key=held.count)
    by_dev: dict = {}
    for j, d in enumerate(locs):
        by_dev.setdefault(home if d is None else d, []).append(j)
    return by_dev


def _read_placed(sub, batch: list, by_dev: dict, t, h, dim: int) -> tuple:
    """read_multi for device-resident items: each device decodes the items
    whose bytes it holds -- into the out itself when the out lives there,
    else into a slab over its items' band of the out (one copy back when no
    other device's items touch the band, else one copy per item region)."""
    import numpy as np
    import torch

    results: list = [None] * len(batch)
    devs = list(by_dev)
    spans = dict(zip(devs, item_bands(batch, [by_dev[d] for d in devs], dim)))
    shape = tuple(t.shape) if t is not None else h.shape

    def job(d):
        idx = by_dev[d]
        items = [batch[j] for j in idx]
        if t is not None and t.device.index == d:
            res = sub.read_sync(items, t)
        else:
            sp = spans[d]
            lo, hi = (sp[0][0], sp[-1][1]) if sp else (0, shape[dim])
            if t is not None:
                target = t.narrow(dim, lo, hi - lo)
                slab = _dense_like(target, torch.device("cuda", d))
            else:
                target = torch.from_numpy(np.moveaxis(np.moveaxis(h, dim, 0)[lo:hi], 0, dim))
                slab = torch.empty(tuple(target.shape), dtype=target.dtype, device=torch.device("cuda", d))
            shifted = [_shift(it, dim, lo) for it in items] if sp else items
            whole = sp is not None and len(sp) == 1
            if whole and sum(_cells(it[3]) for it in items) < slab.numel():
                slab.copy_(target)  # regions no item writes keep their values
            res = sub.read_sync(shifted, slab)
            if whole:
                target.copy_(slab)  # one peer copy (device out) / D2H (host out) of the band
            else:
                for it in shifted:
                    osel = tuple(it[3])
                    target[osel].copy_(slab[osel])
            torch.cuda.current_stream(torch.device("cuda", d)).synchronize()
        for j, r in zip(idx, res):
            results[j] = r

    _run_on_devices(sub, [(d, (lambda d=d: job(d))) for d in devs])
    return tuple(results)


def _cells(osel) -> int:
    n = 1
    for s in osel:
        if isinstance(s, slice):
            n *= max(0, -((int(s.start or 0) - int(s.stop)) // (s.step or 1)))
    return n


def _dense_like(band, device):
    """An empty dense tensor of band's shape on `device` whose dims are laid out
    in band's stride order (a C band gets a C slab, an F band an F slab), so
    the slab -> band copy is one contiguous range."""
    import torch

    order = sorted(range(band.dim()), key=lambda d: -abs(band.stride(d)))
    strides = [0] * band.dim()
    acc = 1
    for d in reversed(order):
        strides[d] = acc
        acc *= band.shape[d]
    return torch.empty_strided(tuple(band.shape), tuple(strides), dtype=band.dtype, device=device)


def _shift(it, dim: int, lo: int):
    osel = list(it[3])
    s = osel[dim]
    osel[dim] = slice(int(s.start or 0) - lo, int(s.stop) - lo, 1)
    return tuple(it[:3]) + (tuple(osel),) + tuple(it[4:])


def _device_pipes(pipe):
    """One single-device twin of a multi-device pipeline (plan cache of its own)."""
    from dataclasses import replace

    sub = pipe._aux.get("single")
    if sub is None:
        sub = pipe._aux["single"] = replace(pipe, devices=(), _read_cache={}, _aux={})
    return sub


def _run_on_devices(pipe, jobs):
    """jobs: [(device index, fn)] run concurrently, one host thread per job
    (each with that device current); exceptions propagate."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    pool = pipe._aux.get("dev_pool")
    if pool is None or pool._max_workers < len(jobs):
        pool = pipe._aux["dev_pool"] = ThreadPoolExecutor(max_workers=max(8, len(jobs)),
                                                          thread_name_prefix="zarr_hip_devs")

    def run(job):
        d, fn = job
        with torch.cuda.device(d):
            return fn()

    futs = [pool.submit(run, j) for j in jobs]
    return [f.result() for f in futs]


def read_multi(pipe, batch: list, out, drop_axes: tuple):
    """HipCodecPipeline.read_sync with ``devices``.  Items whose bytes already
    sit in a GPU's HBM (a DeviceStore) decode on that GPU (``placement``):
    only decoded bands move, never encoded bytes -- a store on one GPU with
    the out on the same GPU is the single-device read.  Host-resident items
    are split into bands of the out along its outermost dim (the reference's
    disjoint-output pool map, codec_pipeline.py:1104-1109, 1169-1171, with a
    GPU per worker); every device decodes its band into a compact slab of its
    own -- the out's own band when the out lives on that device, else a slab
    tensor there -- and the slab reaches the out in ONE contiguous copy (a
    peer copy over xGMI for a device out, a D2H over the device's own PCIe
    link for a host out).  None when the batch does not split (one band,
    drop_axes): the caller reads on one device."""
    import numpy as np
    import torch

    from .interop import device_tensor, host_array

    if drop_axes:
        return None
    t = device_tensor(out)
    h = host_array(out) if t is None else None
    if t is None and h is None:
        return None
    shape = tuple(t.shape) if t is not None else h.shape
    if not shape:  # a 0-d out (every index an integer): one element, one device
        return None
    strides = tuple(t.stride()) if t is not None else tuple(x // h.itemsize for x in h.strides)
    dim = outer_dim(strides, shape)
    # bytes already in HBM decode where they are (no encoded bytes between GPUs)
    by_dev = placement(batch, t.device.index if t is not None else None)
    if by_dev is not None:
        if len(by_dev) == 1 and t is not None and t.device.index in by_dev:
            return None  # one device holds the bytes and the out: the single-device read
        return _read_placed(_device_pipes(pipe), batch, by_dev, t, h, dim)
    groups = device_bands(batch, len(pipe.devices), dim)
    if groups is None or len(groups) < 2:
        return None
    sub = _device_pipes(pipe)
    results: list = [None] * len(batch)

    def job(gi, dev):
        lo, hi, idx = groups[gi]
        items = [_shift(batch[j], dim, lo) for j in idx]
        if t is not None:
            band = t.narrow(dim, lo, hi - lo)
            if band.device.index == dev:
                res = sub.read_sync(items, band)
            else:
                slab = _dense_like(band, torch.device("cuda", dev))
                res = sub.read_sync(items, slab)
                band.copy_(slab)  # one peer copy of the band
                torch.cuda.current_stream(band.device).synchronize()
        else:
            band = np.moveaxis(h, dim, 0)[lo:hi]
            band = np.moveaxis(band, 0, dim)
            res = sub.read_sync(items, band)  # host out: staged, decoded and copied back on `dev`
        for j, r in zip(idx, res):
            results[j] = r

    devs = pipe.devices
    _run_on_devices(pipe, [(devs[gi], (lambda gi=gi: job(gi, devs[gi]))) for gi in range(len(groups))])
    return tuple(results)


def write_multi(pipe, batch: list, value, drop_axes: tuple, partial_encode: bool) -> bool:
    """HipCodecPipeline.write_sync with ``devices``: items split into bands of
    the value as for reads, every device encodes its band's chunks (its value
    band copied to it) and writes them to the store.  Host stores only: a
    DeviceStore's arena lives on one device, which then encodes everything.
    False when the batch does not split (the caller writes on one device)."""
    import numpy as np
    import torch

    from .store import DeviceStore

    if drop_axes or any(isinstance(getattr(it[0], "store", None), DeviceStore) for it in batch):
        return False
    is_t = isinstance(value, torch.Tensor)
    vshape = tuple(value.shape) if hasattr(value, "shape") else ()
    if len(vshape) == 0:
        dim = 0
        ndim = len(batch[0][3])
        groups = device_bands(batch, len(pipe.devices), 0) if ndim else None
    else:
        strides = tuple(value.stride()) if is_t else tuple(x // value.itemsize for x in value.strides)
        dim = outer_dim(strides, vshape)
        groups = device_bands(batch, len(pipe.devices), dim)
    if groups is None or len(groups) < 2:
        return False
    sub = _device_pipes(pipe)

    def job(gi, dev):
        lo, hi, idx = groups[gi]
        items = [_shift(batch[j], dim, lo) for j in idx]
        if len(vshape) == 0:
            v = value
            items = [batch[j] for j in idx]
        elif is_t:
            v = value.narrow(dim, lo, hi - lo)
            if v.is_cuda and v.device.index != dev:
                v = v.to(torch.device("cuda", dev))
        else:
            v = np.moveaxis(np.moveaxis(value, dim, 0)[lo:hi], 0, dim)
        sub._write_sync(items, v, (), partial_encode)

    devs = pipe.devices
    _run_on_devices(pipe, [(devs[gi], (lambda gi=gi: job(gi, devs[gi]))) for gi in range(len(groups))])
    return True

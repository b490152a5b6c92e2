"""Host -> HBM staging for batches whose bytes live in host memory.

The reference reads chunk bytes into host buffers (``ByteGetter.get_sync``,
``Store.get_ranges_sync`` with ``coalesce_ranges`` for partial shards:
src/zarr/abc/store.py:474-539, src/zarr/core/_coalesce.py:61-135,
src/zarr/codecs/sharding.py:1695-1752).  Here those bytes are packed into one
pinned buffer (256-byte aligned placements) by the library's host thread pool
(zhip_stage_h2d, csrc/staging.cpp), in windows of ``WINDOW`` bytes; each
window's ``hipMemcpyAsync`` is issued on a dedicated copy stream by the thread
that packs it, so host packing overlaps PCIe transfer with no per-window
Python.  The packing job runs on a stager thread while the caller plans the
decode (tables, uploads); the consuming launch waits for the copy stream once
(``Pending.finish``).

Partial shard reads follow the reference's IO shape: the index is fetched
by a suffix (or prefix) range request, the touched inner chunks' byte ranges
are fetched with coalescing, and only those bytes cross PCIe.  The host reads
the u64 (offset, length) pairs to know what to fetch; the index CRC itself is
verified on the GPU (the staged index bytes go through the NO_WRITE decode
launch), so errors surface with the reference's message.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from .interop import byte_payload, is_missing_key_error, request_classes, staged_bytes
from .store import ALIGN, TAIL_SLACK, DeviceRef, FileRef, MemoryStore, StorePath, pinned_spans

# 4 MiB windows: smaller ones pay ~10 us per hipMemcpyAsync, larger ones start
# the DMA late (scripts/stage_micro.py)
WINDOW = int(os.environ.get("ZARR_HIP_STAGE_WINDOW", str(4 << 20)))
# partial shard reads: shards are staged in runs of this many bytes, each run
# one packing job begun as soon as its bytes are fetched
GROUP = int(os.environ.get("ZARR_HIP_STAGE_GROUP", str(64 << 20)))
MAX_U64 = np.uint64(0xFFFFFFFFFFFFFFFF)

_COPY_STREAMS: dict = {}
_COPY_MODE_SET = [False]


def _copy_mode() -> None:
    """ZARR_HIP_STAGE_COPY=memcpy selects plain memcpy packing (measurement
    arm; the library default is streaming stores, ZHIP_TUNE_STAGE_COPY)."""
    if _COPY_MODE_SET[0]:
        return
    _COPY_MODE_SET[0] = True
    mode = os.environ.get("ZARR_HIP_STAGE_COPY", "")
    if mode:
        from . import _native as N

        N.lib().zhip_set_tuning(5, 0 if mode == "memcpy" else 1)


def _workers() -> int:
    n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap or 8, 16))


def _copy_stream(device):
    import torch

    key = torch.device(device).index
    s = _COPY_STREAMS.get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _COPY_STREAMS[key] = s
    return s


def quiesce() -> None:
    """Wait for every staging copy already enqueued (before host bytes they
    read are reused)."""
    for s in list(_COPY_STREAMS.values()):
        s.synchronize()


class StagingLayout:
    """Aligned placements of host byte pieces inside one staging buffer."""

    def __init__(self):
        self.pieces: list = []  # (buffer-like, dst_off, nbytes)
        self.top = 0

    def add(self, buf) -> tuple[int, int]:
        n = len(buf) if buf is not None else 0
        off = self.top
        if n:
            self.pieces.append((buf, off, n))
        self.top = (off + n + ALIGN - 1) // ALIGN * ALIGN
        return off, n

    def reserve(self, n: int) -> int:
        """Space filled later by a device-to-device copy."""
        off = self.top
        self.top = (off + n + ALIGN - 1) // ALIGN * ALIGN
        return off


def _host_view(buf) -> np.ndarray:
    return buf if isinstance(buf, np.ndarray) else np.frombuffer(buf, dtype=np.uint8)


class Pending:
    """Staged bytes on their way to HBM: the device buffer (allocated now,
    filled on the copy stream by a library packing job that runs without the
    Python GIL) and what the consuming launch must wait for.  ``finish()``
    (idempotent) joins the job, makes the launch stream wait for the copy
    stream, then runs the device-to-device copies of pieces that were already
    on the device.

    The job owns what it reads and writes (``keepalive``: the device buffer,
    the pinned packing block, the host views and encoded file paths): a
    begun job keeps running in a library thread until it is ended, so every
    path that drops a Pending without consuming it -- an exception between
    begin and launch, a slab loop that stops early -- must ``abort()`` it.
    ``abort()`` joins the job and waits for its copies before the buffers can
    go back to torch's caching allocators; ``__del__`` is the safety net."""

    def __init__(self, dev, job, cs, post, keepalive=()):
        self.dev = dev
        self._job = job
        self._cs = cs
        self._post = post
        self.keepalive = list(keepalive)

    @property
    def active(self) -> bool:
        return self._job is not None

    def finish(self, stream: int | None = None) -> None:
        if self._job is None:
            return
        import torch

        from . import _native as N

        st = torch.cuda.current_stream(self.dev.device) if stream is None else \
            torch.cuda.ExternalStream(stream, device=self.dev.device)
        # the launch stream waits for this job's copies (an event the library
        # recorded after its last one), not for later jobs already queued on
        # cs; handle 0 is the default stream and waits like any other
        rc = N.lib().zhip_stage_end(self._job, int(st.cuda_stream))
        self._job = None
        if rc != 0:
            # a failed job may have enqueued some copies: they must be done
            # before the caller's exception frees the buffers they touch
            self._cs.synchronize()
            self._post = []
            N.check(rc, "zhip_stage_h2d")
        if self._post:
            with torch.cuda.stream(st):
                for fn in self._post:
                    fn(self.dev)
        self._post = []

    def abort(self) -> None:
        """End a job that will not be consumed: join the packing thread, wait
        for every copy it enqueued; errors are swallowed (the caller is already
        unwinding, or nobody will read the bytes)."""
        job, self._job = self._job, None
        self._post = []
        if job is None:
            return
        try:
            from . import _native as N

            N.lib().zhip_stage_end(job, self._cs.cuda_stream)
            self._cs.synchronize()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass

    def __del__(self):
        if getattr(self, "_job", None) is not None:
            self.abort()


def _piece_table(pieces: list):
    """zhip_piece records of (buffer-like, dst_off, nbytes) pieces; returns
    (table, views to keep alive, all pieces page-locked)."""
    from . import _native as N

    # file pieces carry an encoded path (kept alive with the job) and an offset;
    # bytes objects are addressed in place (ctypes.cast: a third of the cost
    # of a numpy view's .ctypes per piece, which adds up over a batch)
    views = [np.frombuffer(buf.path.encode() + b"\0", np.uint8) if isinstance(buf, FileRef)
             else buf if type(buf) is bytes else _host_view(buf) for buf, _, _ in pieces]
    table = np.zeros(len(views), N.PIECE_DT)
    _cast, _vp = ctypes.cast, ctypes.c_void_p
    addrs = [_cast(v, _vp).value if type(v) is bytes else v.ctypes.data for v in views]
    table["host"] = addrs
    table["nbytes"] = [n for _, _, n in pieces]
    table["dst_off"] = [off for _, off, _ in pieces]
    files = [isinstance(buf, FileRef) for buf, _, _ in pieces]
    flags = [N.PIECE_FILE if f else 0 for f in files]
    if any(files):
        table["file_off"] = [buf.offset if f else 0 for f, (buf, _, _) in zip(files, pieces)]
    spans = pinned_spans()
    if spans:
        flags = [fl or (N.PIECE_PINNED if any(lo <= a and a + n <= hi for lo, hi in spans) else 0)
                 for fl, a, (_, _, n) in zip(flags, addrs, pieces)]
    table["flags"] = flags
    return table, views, bool(flags) and all(fl == N.PIECE_PINNED for fl in flags)


def _begin_job(pieces: list, dev, dev_off: int, total: int, cs, post=()):
    """One library packing job: `pieces` (dst offsets relative to dev_off)
    into dev[dev_off: dev_off + total] on copy stream cs.  Returns its Pending."""
    import torch

    from . import _native as N

    table, views, all_pinned = _piece_table(pieces)
    # the packing buffer (pinned, reused through torch's caching host allocator)
    host = torch.empty(16 if all_pinned else total + TAIL_SLACK, dtype=torch.uint8, pin_memory=True)
    job = N.lib().zhip_stage_begin(table.ctypes.data, len(table), host.data_ptr(), dev.data_ptr() + dev_off,
                                   total, WINDOW, _workers(), cs.cuda_stream)
    if not job:
        raise N.NativeError("zhip_stage_begin: out of memory")
    # the pinned block and the host views must outlive the copies: the job
    # holds them until it is finished or aborted, the program afterwards
    # (dropped after its results() synchronised)
    return Pending(dev, job, cs, list(post), [dev, host, views])


def _stage_target(total: int, device):
    """A new device buffer for staged bytes and the copy stream that fills it
    (after the compute stream's earlier work)."""
    import torch

    _copy_mode()
    dev = torch.empty(max(total, 16) + TAIL_SLACK, dtype=torch.uint8, device=device)
    compute = torch.cuda.current_stream(device)
    cs = _copy_stream(device)
    cs.wait_stream(compute)
    dev.record_stream(cs)
    return dev, cs


def stage(layout: StagingLayout, device, post=(), defer: bool = False):
    """Copy every piece to one new device buffer.  Returns (dev, keepalive,
    pending); with defer the packing job keeps running when this returns and
    the caller must ``pending.finish()`` before the first use of dev."""
    total = max(layout.top, 16)
    dev, cs = _stage_target(total, device)
    pending = _begin_job(layout.pieces, dev, 0, total, cs, post)
    if not defer:
        pending.finish()
    return dev, pending.keepalive, pending


class PendingGroup:
    """Several packing jobs filling one device buffer, begun as their bytes
    arrived (Pending's interface: finish / abort / active / keepalive)."""

    def __init__(self, dev, parts: list):
        self.dev = dev
        self.parts = parts
        self.keepalive = [p.keepalive for p in parts]

    @property
    def active(self) -> bool:
        return any(p.active for p in self.parts)

    def finish(self, stream: int | None = None) -> None:
        for p in self.parts:
            p.finish(stream)

    def abort(self) -> None:
        for p in self.parts:
            p.abort()


# encoded bytes copied device to device by gather_sources (another GPU's
# arena): parallel.read_multi decodes device-resident items where they live,
# and the tests check that it then stages nothing
D2D_COPIES = [0]


def gather_sources(batch: list, device, defer: bool = False, start: bool = True):
    """Resolve every ByteGetter to (offset, length, missing) inside ONE device
    buffer: the shared arena for DeviceStore batches, else a staged copy.
    ByteGetters may be this package's or zarr's (whose get_sync returns a
    Buffer, src/zarr/storage/_common.py:247-258).
    Returns (src, size, [(off, len, missing)], keepalive, pending | None).
    With start=False a host-sourced batch is laid out but not staged yet:
    src is None and the last element is a callable that starts the staging
    (deferred) and returns (src, keepalive, pending)."""
    import torch

    raws = _memory_values(batch)
    host_only = raws is not None  # bytes / None only: no device pieces to look for
    if raws is None:
        raws = []
        for item in batch:
            bg = item[0]
            loc = getattr(getattr(bg, "store", None), "locate_sync", None)
            if loc is not None:  # a local file: the staging pool preads it (ZHIP_PIECE_FILE)
                raws.append(loc(bg.path))
            else:
                raws.append(staged_bytes(bg.get_sync(prototype=None) if hasattr(bg, "get_sync") else bg))
    arenas = {} if host_only else {id(r.arena): r.arena for r in raws if isinstance(r, DeviceRef)}
    all_dev = not host_only and all(r is None or isinstance(r, DeviceRef) for r in raws)
    tdev = torch.device(device)
    if arenas and any(a.device.type != tdev.type or (a.device.index or 0) != (tdev.index or 0)
                      for a in arenas.values()):
        all_dev = False  # another GPU's arena: its bytes are copied to `device` below
    if all_dev and len(arenas) <= 1:
        if arenas:
            arena = next(iter(arenas.values()))
            src, size = arena.buf, arena.top
        else:
            src = torch.zeros(TAIL_SLACK + 16, dtype=torch.uint8, device=device)
            size = 0
        srcs = [(0, 0, True) if r is None else (r.offset, r.length, False) for r in raws]
        return src, size, srcs, [src], None
    lay = StagingLayout()
    srcs = []
    dev_refs = []
    pieces, top, A = lay.pieces, 0, ALIGN - 1
    for r in raws:  # StagingLayout.add / reserve inlined (one pass per batch item)
        if r is None:
            srcs.append((0, 0, True))
            continue
        if not host_only and isinstance(r, (DeviceRef, torch.Tensor)):  # device bytes elsewhere: D2D below
            n = r.length if isinstance(r, DeviceRef) else r.numel()
            dev_refs.append((r, top))
        else:
            n = len(r)
            if n:
                pieces.append((r, top, n))
        srcs.append((top, n, False))
        top = (top + n + A) & ~A
    lay.top = top
    def d2d(dev):  # after the H2D windows (which also cover the reserved gaps)
        for r, off in dev_refs:
            v = r.arena.view(r.offset, r.length) if isinstance(r, DeviceRef) else r
            dev[off: off + v.numel()].copy_(v)
            D2D_COPIES[0] += 1

    if not start:
        return None, lay.top, srcs, [], lambda: stage(lay, device, post=[d2d] if dev_refs else [], defer=True)
    dev, keep, pending = stage(lay, device, post=[d2d] if dev_refs else [], defer=defer)
    return dev, lay.top, srcs, keep, pending


def _memory_values(batch: list):
    """Whole values of a batch whose getters are all StorePaths into ONE of this
    package's MemoryStores (the class itself: a subclass may override
    get_sync), read from its dict in one pass: the per-item getter chain
    (StorePath.get_sync -> MemoryStore.get_sync -> memoryview -> staging view)
    is most of a host read's Python cost before the first DMA.  The bytes
    objects go to the packer as they are (addressed in place).  None when the
    batch is anything else."""
    bg0 = batch[0][0]
    if type(bg0) is not StorePath or type(bg0.store) is not MemoryStore:
        return None
    st = bg0.store
    if not all(type(it[0]) is StorePath and it[0].store is st for it in batch):
        return None
    get = st._d.get
    vals = [get(it[0].path) for it in batch]
    return [v if v is None or type(v) is bytes else staged_bytes(memoryview(v)) for v in vals]


def staged_host(buf):
    """A fetched byte range as host bytes for the pinned packer."""
    if isinstance(buf, (bytes, bytearray, memoryview)):
        return buf
    return byte_payload(buf, host=True)


def _shard_key(bg):
    st = getattr(bg, "store", None)
    return (id(st), getattr(bg, "path", id(bg)))


def _touched_slots(csel, shard_shape, inner_shape, strides):
    """Linear inner-chunk slots a chunk selection of ints and unit-step slices
    touches, by interval arithmetic; None for other forms (the caller then
    projects: strided slices may skip inner chunks).  A list of ints."""
    los, his = [], []
    for s, n, c in zip(csel, shard_shape, inner_shape):
        if type(s) is slice:
            a, b, step = s.indices(n)
            if step != 1:
                return None
            if a >= b:
                return []
            los.append(a // c)
            his.append((b - 1) // c + 1)
        elif isinstance(s, (int, np.integer)):
            i = int(s) + (n if int(s) < 0 else 0)
            los.append(i // c)
            his.append(i // c + 1)
        else:
            return None
    slots = [0]
    for lo, hi, st in zip(los, his, strides):
        if hi - lo == 1:
            off = lo * st
            slots = [x + off for x in slots]
        else:
            slots = [x + k * st for x in slots for k in range(lo, hi)]
    return slots


def gather_sharded_partial(batch: list, sh, cps, n_inner: int, inner_shape, spec, device,
                           defer: bool = False, inner_decode=None):
    """Host-sourced sharded batch: index by range request, touched inner chunks
    by coalesced range requests, staged into one device buffer.  With
    ``inner_decode`` (a list of inner-chunk bytes -> their fixed-size bytes:
    the inner chain's host stage, hoststage.py) every fetched inner chunk
    passes through it on the host before it is staged.

    Returns (src, size, item_missing[n_items], resolved, keepalive) where
    resolved[i] = (src_by_slot, len_by_slot, miss_by_slot, index_src_or_-1)."""
    from .indexing import basic_projections

    isz = sh.shard_index_size(n_inner)
    cps_strides = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
    st_list = [int(x) for x in cps_strides]
    sshape = tuple(int(x) for x in spec.shape)
    ishape = tuple(int(x) for x in inner_shape)
    shards: dict = {}
    item_shard = []
    for item in batch:
        k = _shard_key(item[0])
        if k not in shards:
            shards[k] = {"bg": item[0], "slots": set()}
        csel = tuple(item[2])
        sl = _touched_slots(csel, sshape, ishape, st_list) if len(csel) == len(sshape) else None
        if sl is None:
            pr = basic_projections(csel, spec.shape, inner_shape)
            sl = (pr.coords * cps_strides[None, :]).sum(axis=1).tolist()
        shards[k]["slots"].update(sl)
        item_shard.append(k)
    # 1. every touched shard's index (one range request each) and the layout:
    #    [index bytes][touched inner chunks] per shard, each chunk's size known
    #    from its index entry (a host-stage chain: the decoded chunk size)
    out_of_shard = {}
    plans = []
    top, A = 0, ALIGN - 1
    cfg = spec.config  # forwarded like sharding.py:1695-1752
    cap = int(np.prod(ishape)) * spec.dtype.itemsize + 4  # the largest encoded inner chunk of a GPU chain

    def fetch_ranges(bg, st, reqs):
        """(request index, bytes) of every range, or None when the shard
        vanished between the index and data reads."""
        try:
            if st is not None and hasattr(st, "get_ranges_sync"):
                return list(st.get_ranges_sync(bg.path, reqs, prototype=spec.prototype,
                                               max_gap_bytes=cfg.sharding_coalesce_max_gap_bytes,
                                               max_coalesced_bytes=cfg.sharding_coalesce_max_bytes))
            return [(j, bg.get_sync(prototype=None, byte_range=r)) for j, r in enumerate(reqs)]
        except Exception as e:
            if not is_missing_key_error(e):
                raise
            return None

    for k, s in shards.items():
        bg = s["bg"]
        st = getattr(bg, "store", None)
        Range, Suffix = request_classes(st)
        req = Suffix(isz) if sh.index_location == "end" else Range(0, isz)
        raw = bg.get_sync(prototype=None, byte_range=req)
        if raw is None:
            out_of_shard[k] = None  # whole shard missing -> fill (status "missing")
            continue
        raw = byte_payload(raw, host=True)
        if len(raw) < isz:
            raise ValueError("shard blob is shorter than its index")
        idx = np.frombuffer(raw, dtype="<u8", count=2 * n_inner).reshape(n_inner, 2)
        if inner_decode is not None and sh.index_has_crc:
            # the offsets drive host decompression before the GPU sees the
            # index: verify it here first, as _decode_shard_index_sync does
            # (sharding.py:624-631), so a corrupted index raises the checksum
            # message, not the decompressor's error
            from .hoststage import host_crc32c
            from .pipeline import crc_error_message

            body = np.frombuffer(raw, np.uint8, count=isz - 4)
            stored = int(np.frombuffer(raw, "<u4", count=1, offset=isz - 4)[0])
            computed = host_crc32c(body)
            if stored != computed:
                raise ValueError(crc_error_message(stored, computed))
        lo = top
        pieces = []
        idx_off = -1
        if sh.index_has_crc:
            idx_off = top
            pieces.append((raw, top, len(raw)))
            top = (top + len(raw) + A) & ~A
        src_by = np.zeros(n_inner, np.int64)
        len_by = np.zeros(n_inner, np.int64)
        miss_by = np.ones(n_inner, bool)
        reqs, fetch = [], []
        eager = False
        ent = idx.reshape(-1).tolist()  # plain ints: (offset, length) per slot
        whole = None
        if st is not None and hasattr(st, "locate_sync") and inner_decode is None:
            # a local file: each touched inner chunk is one pread of the shard
            # file by the staging pool (no coalescing needed: no request cost)
            whole = st.locate_sync(bg.path)
            if whole is None:
                out_of_shard[k] = None
                continue
        for slot in sorted(s["slots"]):
            o, n = ent[2 * slot], ent[2 * slot + 1]
            if o == MAX_U64 and n == MAX_U64:
                continue  # missing inner chunk -> fill (sharding.py:700-712)
            if whole is not None:
                if o + n > whole.length:
                    raise ValueError("shard index entry points outside the shard blob")
                pieces.append((FileRef(whole.path, o, n), top, n))
                src_by[slot], len_by[slot], miss_by[slot] = top, n, False
                top = (top + n + A) & ~A
                continue
            reqs.append(Range(o, o + n))
            fetch.append((slot, top, n))
            top = (top + n + A) & ~A
            eager = eager or n > cap
        if reqs and (inner_decode is not None or eager):
            # a host stage first (its output size is the GPU chain's), or an
            # index entry longer than any encoded inner chunk (a corrupted
            # index; the GPU's index check reports it): fetched now, laid out
            # at the sizes that arrive
            got = fetch_ranges(bg, st, reqs)
            if got is None:
                out_of_shard[k] = None
                continue
            bufs = [staged_host(buf) for _, buf in got]
            if inner_decode is not None:
                bufs = inner_decode(bufs)
            top = pieces[-1][1] + ((pieces[-1][2] + A) & ~A) if pieces else lo
            for (j, _), buf in zip(got, bufs):
                slot = fetch[j][0]
                pieces.append((buf, top, len(buf)))
                src_by[slot], len_by[slot], miss_by[slot] = top, len(buf), False
                top = (top + len(buf) + A) & ~A
            reqs, fetch = [], []
        out_of_shard[k] = (src_by, len_by, miss_by, idx_off)
        plans.append((k, bg, st, lo, top, pieces, reqs, fetch))
    # 2. the chunk bytes, shard by shard: each run of shards reaching GROUP
    #    bytes becomes its own packing job into its slice of the buffer, begun
    #    as soon as its bytes are fetched, so the copies of early shards overlap
    #    the requests (and the Python) of later ones
    dev, cs = _stage_target(top, device)
    parts: list = []
    run: list = []
    run_lo = run_hi = 0

    def emit():
        if run:
            parts.append(_begin_job([(b, off - run_lo, n) for b, off, n in run], dev, run_lo, run_hi - run_lo, cs))
    try:
        for k, bg, st, lo, hi, pieces, reqs, fetch in plans:
            if reqs:
                got = fetch_ranges(bg, st, reqs)
                if got is None:  # the shard vanished between the index and data reads
                    out_of_shard[k] = None
                    continue
                src_by, len_by, miss_by, _ = out_of_shard[k]
                for j, buf in got:
                    buf = staged_host(buf)
                    slot, off, size = fetch[j]
                    m = len(buf)
                    if m > size:
                        raise ValueError("an inner chunk is larger than its index entry")
                    pieces.append((buf, off, m))
                    src_by[slot], len_by[slot], miss_by[slot] = off, m, False
                pieces.sort(key=lambda x: x[1])  # packing jobs take pieces in destination order
            if not run:
                run_lo = lo
            run.extend(pieces)
            run_hi = hi
            if run_hi - run_lo >= GROUP:
                emit()
                run = []
        emit()
    except BaseException:
        for p in parts:  # begun jobs must not outlive the buffers they fill
            p.abort()
        raise
    pending = PendingGroup(dev, parts)
    if not defer:
        pending.finish()
    missing = np.array([out_of_shard[k] is None for k in item_shard], bool)
    resolved = [out_of_shard[k] for k in item_shard]
    return dev, top, missing, resolved, pending.keepalive, pending

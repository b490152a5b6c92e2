"""Write path of HipCodecPipeline: FusedCodecPipeline.write_sync
(src/zarr/core/codec_pipeline.py:1174-1253) with the codec compute on the GPU.

Per batch:
  * complete chunks are encoded straight from the (device) value array; the
    part of an edge chunk outside the array is written as the fill value
    (_merge_chunk_array, src/zarr/core/chunk_utils.py:115-162); a scalar value
    is read through a stride-0 view (nothing array-sized is materialised);
  * partial chunks: every existing chunk of the batch is decoded by ONE GPU
    launch into a stacked temporary (absent chunks come out as the fill
    value), the value is merged into it with a device copy, and the temporary
    is encoded as whole chunks;
  * empty chunks (all elements == fill under NDBuffer.all_equal rules) are
    deleted instead of stored unless write_empty_chunks (chunk_utils.py:43-85);
  * sharded arrays: inner chunks are encoded densely in subchunk write order
    into the shard blob, then one packing launch elides empty inner chunks and
    writes the index + its CRC (sharding.py:887-950); an all-empty shard is
    deleted.  Without array->array codecs around the sharding codec this is
    the reference's partial encode (ShardingCodec._encode_partial_sync,
    sharding.py:774-885): only the inner chunks the write touches are merged
    and re-evaluated, untouched ones keep their state (a present inner chunk
    stays present even if it holds only fill, an absent one stays absent),
    and a shard the write does not cover whole is read first.  With them, the
    whole merged shard is encoded (ShardingCodec._encode_sync, 716-772).
Encoded bytes land directly in the DeviceStore arena (no copy) or, for host
stores, in a device staging buffer copied back once per batch.
"""

from __future__ import annotations

import numpy as np

from . import _native as N
from .buffer import torch_dtype
from .indexing import basic_projections, subchunk_order
from .interop import is_own_store, wrap_for_setter
from .planner import SEL_DT, ChainInfo, analyze_chain, plan_encode
from .spec import ArraySpec
from .store import ALIGN, DeviceStore, TAIL_SLACK


def _torch():
    import torch

    return torch


def _upload(arr: np.ndarray, device):
    torch = _torch()
    b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    t = torch.empty(max(b.size, 16), dtype=torch.uint8, device=device)
    if b.size:
        t[: b.size].copy_(torch.from_numpy(b.copy()))
    return t


class EncodeLaunch:
    """One zhip_encode launch over flat chunk tables.  Every launch writes every
    chunk's non-empty flag (the library zeroes the flags itself before a kernel
    that ORs them, include/zarrhip.h), so a prepared launch can be replayed."""

    def __init__(self, layout: N.Layout, chunks: np.ndarray, sels: np.ndarray, arr, dst, fast: bool,
                 device, rows: bool = False, tile: bool = False, tile_prefix: bool = False):
        from .pipeline import _rows_map, _whole_sels, get_plan

        torch = _torch()
        self.plan = get_plan(layout)
        self.n = len(chunks)
        self.device = device
        self.d_chunks = _upload(chunks, device)
        self.d_sels = _upload(sels if len(sels) else np.zeros(1, SEL_DT), device)
        self.d_status = torch.zeros(max(self.n, 1) * 4, dtype=torch.int32, device=device)
        self.d_ws = torch.zeros(max(self.n, 1) * max(4, self.plan.workspace_words), dtype=torch.int32,
                                device=device)  # zhip_plan_info
        self.d_nonempty = torch.zeros(max(self.n, 1), dtype=torch.int32, device=device)
        self.arr = arr
        self.dst = dst
        self.flags = N.DF_FAST_ROWS if fast else 0
        # whole-row batches encode in k_encode_pair through the row map
        self.d_rowmap = _rows_map(self.plan, sels, device) if fast and rows else None
        if self.d_rowmap is not None and _whole_sels(layout, sels):
            self.flags |= N.DF_WHOLE  # whole chunks: destinations from the plan (zarrhip.h)
        # transposed layouts: k_encode_tile4 (full selections, full tiles, <= 64
        # tiles per chunk: the library decides) or k_encode_tile (any tiling,
        # prefix-box selections of edge chunks)
        if not fast and self.plan.kernel_flags & N.PK_TILE:
            if tile:
                self.flags |= N.DF_TILE
            elif tile_prefix:
                self.flags |= N.DF_TILE_PREFIX

    def launch(self, stream: int | None = None) -> None:
        from .pipeline import _stream_handle

        if self.n == 0:
            return
        s = _stream_handle(self.device) if stream is None else stream
        N.check(N.lib().zhip_encode_mapped(self.plan.handle, self.arr.data_ptr(), self.dst.data_ptr(),
                                           self.d_chunks.data_ptr(), self.n, self.d_sels.data_ptr(),
                                           self.d_status.data_ptr(), self.d_ws.data_ptr(),
                                           self.d_nonempty.data_ptr(), self.flags,
                                           self.d_rowmap.data_ptr() if self.d_rowmap is not None else None,
                                           s), "zhip_encode_mapped")

    def nonempty(self) -> np.ndarray:
        from . import pipeline as P

        P.SYNCS[0] += 1
        return self.d_nonempty[: self.n].cpu().numpy().astype(bool)


class PendingWrites:
    """Encodes launched but not yet committed (a batch of several chunk specs,
    pipeline._write_sync): every group's merge reads, encodes and flag words
    are queued first, then ONE zhip_wait_ranges brings back all the groups'
    decode error / verdict words and non-empty flags, errors raise before
    anything is stored, and each group's results are committed."""

    def __init__(self):
        self.items = []  # (dest, setters, [(EncodeLaunch, idx)], elen, keep_all, prototype, [DecodeProgram])

    def finish(self, device) -> None:
        from .pipeline import _RangeSet

        rngs, shape = [], []
        for dest, setters, launches, elen, keep, proto, checks in self.items:
            for prog in checks:
                r = prog.wait_ranges()
                rngs += r
                shape.append(("check", sum(x[1] for x in r) // 4))
            for l, _ in launches:
                rngs.append((l.d_nonempty.data_ptr(), 4 * l.n))
                shape.append(("ne", l.n))
        host = _RangeSet(rngs).wait(device).copy() if rngs else np.zeros(0, np.uint32)
        pos, k = 0, 0
        for dest, setters, launches, elen, keep, proto, checks in self.items:
            for prog in checks:
                n = shape[k][1]
                prog.results_from_words(host[pos: pos + n])  # raises like the reference
                pos += n
                k += 1
            ne = np.zeros(len(setters), bool)
            for l, idx in launches:
                ne[idx] = host[pos: pos + l.n] != 0
                pos += l.n
                k += 1
            dest.finish(setters, [elen if (keep or ne[i]) else 0 for i in range(len(setters))], proto)
        self.items = []


def _value_tensor(value, dtype, device):
    torch = _torch()
    td = torch_dtype(dtype)
    if isinstance(value, torch.Tensor):
        v = value.to(device=device, dtype=td)
    else:
        a = np.asarray(value)
        if a.dtype != np.dtype(dtype):
            a = a.astype(dtype)
        # np.array keeps 0-d values 0-d (np.ascontiguousarray would make them 1-d)
        v = torch.from_numpy(np.array(a, dtype=np.dtype(dtype).newbyteorder("="), order="C",
                                      copy=True)).to(device)
    return v


def _is_full_region(csel, osel, chunk_shape) -> bool:
    for s in csel:
        if isinstance(s, (int, np.integer)):
            return False
        if (s.start or 0) != 0 or (s.step or 1) != 1:
            return False
    return True


def _covers_shard(csel, shard_shape) -> bool:
    """The write covers every element of the shard (is_complete_shard,
    sharding.py:1437-1445: all inner chunks touched, each completely)."""
    for s, n in zip(csel, shard_shape):
        if isinstance(s, (int, np.integer)):
            if n != 1:
                return False
            continue
        if (s.start or 0) != 0 or (s.step or 1) != 1 or s.stop < n:
            return False
    return True


class _Dest:
    """Where a batch's encoded blobs go: the DeviceStore arena (held under its
    lock from reservation to launch) or a device staging buffer."""

    def __init__(self, setters, nbytes_each, device):
        torch = _torch()
        self.store = None
        if setters and all(isinstance(getattr(s, "store", None), DeviceStore) for s in setters) and \
                len({id(s.store) for s in setters}) == 1:
            self.store = setters[0].store
        self.reserved = int(nbytes_each)
        self.offs = []
        if self.store is not None:
            self.lock = self.store.arena.lock
            self.lock.acquire()
            for _ in setters:
                self.offs.append(self.store.arena.reserve(nbytes_each))
            self.buf = self.store.arena.buf
        else:
            self.lock = None
            top = 0
            for _ in setters:
                self.offs.append(top)
                top = (top + nbytes_each + ALIGN - 1) // ALIGN * ALIGN
            self.buf = torch.empty(top + TAIL_SLACK, dtype=torch.uint8, device=device)

    def release_lock(self):
        if self.lock is not None:
            self.lock.release()
            self.lock = None

    def finish(self, setters, lengths, prototype):
        """Store / delete each setter's result (length 0 = elided)."""
        self.release_lock()
        host = None
        if self.store is None and any(int(n) for n in lengths):
            host = self.buf.cpu().numpy()
        for i, s in enumerate(setters):
            n = int(lengths[i])
            if self.store is not None:
                if n == 0:
                    s.delete_sync()
                self.store.commit(s.path, self.offs[i], n, self.reserved)
            elif n == 0:
                s.delete_sync()
            else:
                data = host[self.offs[i]: self.offs[i] + n].tobytes()
                st = getattr(s, "store", None)
                s.set_sync(data if is_own_store(st) else wrap_for_setter(data, prototype))


class ChunkWriter:
    """Batch writer for one array (unsharded or sharded chain)."""

    def __init__(self, codecs, spec: ArraySpec, array_shape, device):
        self.chain: ChainInfo = analyze_chain(codecs, spec)
        self.spec = spec
        self.array_shape = tuple(array_shape)
        self.device = device

    def write(self, batch, value, codecs, drop_axes=(), partial_encode: bool = True,
              pending: "PendingWrites | None" = None) -> None:
        """pending (unsharded chains): queue the merge read's check and the
        encode's commit on it instead of synchronising here."""
        from .pipeline import HipCodecPipeline, _Raw

        torch = _torch()
        if drop_axes:
            raise NotImplementedError("drop_axes writes are not on the GPU path")
        spec = self.spec
        v = _value_tensor(value, spec.dtype, self.device)
        scalar = v.dim() == 0
        if scalar:
            # the reference writes the scalar into every selected element: read it
            # through a stride-0 view of the selection's extent (no array-sized copy)
            shp = [0] * len(batch[0][3])
            for it in batch:
                for d, s in enumerate(it[3]):
                    shp[d] = max(shp[d], s.stop)
            v = v.reshape((1,) * len(shp)).expand(tuple(shp)) if shp else v.reshape(())
        chunk_shape = spec.shape
        sharded_partial = self.chain.shard is not None and partial_encode
        complete_items, partial_items = [], []
        for it in batch:
            bs, sp, csel, osel, is_complete = it
            if sharded_partial:
                full = _covers_shard(csel, chunk_shape)
            else:
                full = is_complete and v.dim() and _is_full_region(csel, osel, chunk_shape)
            (complete_items if full else partial_items).append(it)
        # partial chunks: ONE decode of every existing chunk into a stacked
        # temporary (absent -> fill), then the merge on the device
        temp = None
        present = None
        deferred = None  # the merge read, when its check is left to `pending`
        if partial_items:
            pipe = HipCodecPipeline.from_codecs(codecs, warn=False).evolve_from_array_spec(spec)
            temp = torch.empty((len(partial_items),) + tuple(chunk_shape),
                               dtype=torch_dtype(spec.dtype), device=self.device)
            full = tuple(slice(0, s, 1) for s in chunk_shape)
            raws = [bs.get_sync(prototype=None) for bs, *_ in partial_items]
            rb = [(_Raw(raw), spec, full, full, True) for raw in raws]
            stride0 = temp.stride(0) * temp.element_size()
            prog = pipe.prepare_read(rb, temp[0], (), np.arange(len(rb), dtype=np.int64) * stride0)
            prog.launch()
            if sharded_partial:
                st, repairs = self._check_partial_merge(prog, partial_items, chunk_shape)
            elif pending is None or self.chain.shard is not None:
                prog.results()
            else:
                deferred = prog
            if sharded_partial:
                # per (item, inner slot): the inner chunk exists in the stored shard
                n_inner = int(np.prod(self.chain.shard.chunks_per_shard(chunk_shape)))
                present = np.zeros((len(partial_items), n_inner), bool)
                ch = prog.tables.chunks
                present[prog.tables.item_of_chunk, ch["slot"].astype(np.int64)] = \
                    st["code"] != N.ST_MISSING
                missing_item = np.array([r is None for r in raws], bool)
                present[missing_item] = False
            for i, (bs, sp, csel, osel, _) in enumerate(partial_items):
                temp[i][tuple(csel)] = v[tuple(osel)] if v.dim() else v
        if self.chain.shard is not None:
            return self._encode_shards(complete_items, partial_items, v, temp, present,
                                       sharded_partial, repairs if sharded_partial and partial_items else (),
                                       raws if partial_items else None)
        self._encode_chunks(complete_items, partial_items, v, temp, pending,
                            [deferred] if deferred is not None else [])

    def _check_partial_merge(self, prog, partial_items, shard_shape):
        """The merge read of a partial shard write, checked as
        ShardingCodec._encode_partial_sync (sharding.py:774-885) checks it: the
        stored shard index is parsed (its CRC verified), and only the inner
        chunks the write touches but does not cover whole are decoded (their
        CRCs verified, merge_and_encode_chunk).  An inner chunk that fails its
        check raises the reference's message only then; a touched, completely
        overwritten one is replaced by the value; an untouched one is carried
        over as stored -- its bytes copied verbatim into the new shard
        (returned as repairs: (partial item, inner slot)).  Returns (the
        chunk statuses, repairs)."""
        from .pipeline import crc_error_message

        st = prog.data.statuses()  # (consumes the deferred CRC verdicts)
        ist = prog.index.statuses() if prog.index is not None else (
            prog.data.index_statuses() if prog.data.n_idx else None)
        if ist is not None:
            badi = np.nonzero(ist["code"] != N.ST_OK)[0]
            if len(badi):
                r = ist[badi[0]]
                raise ValueError(crc_error_message(int(r["stored"]), int(r["computed"])))
        codes = st["code"]
        bad = np.nonzero((codes != N.ST_OK) & (codes != N.ST_MISSING))[0]
        repairs: list = []
        if not len(bad):
            return st, repairs
        sh = self.chain.shard
        cps = sh.chunks_per_shard(shard_shape)
        cstr = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
        item_of = prog.tables.item_of_chunk
        slot_of = prog.tables.chunks["slot"].astype(np.int64)
        touched: dict = {}
        errors = []
        for j in bad:
            i = int(item_of[j])
            if i not in touched:
                pr = basic_projections(tuple(partial_items[i][2]), tuple(shard_shape), tuple(sh.chunk_shape))
                touched[i] = dict(zip(((pr.coords * cstr[None, :]).sum(axis=1)).tolist(), pr.complete.tolist()))
            s = int(slot_of[j])
            if s not in touched[i]:
                repairs.append((i, s))
            elif not touched[i][s]:
                errors.append((i, s, j))
        if errors:
            _, _, j = min(errors)  # the first shard of the batch, the first inner chunk of its indexer
            r = st[j]
            if r["code"] == N.ST_CRC_MISMATCH:
                raise ValueError(crc_error_message(int(r["stored"]), int(r["computed"])))
            if r["code"] == N.ST_INDEX_OOB:
                raise ValueError("shard index entry points outside the shard blob")
            raise ValueError("encoded chunk length does not match the fixed-size codec chain")
        return st, repairs

    def _encode_chunks(self, complete_items, partial_items, v, temp, pending=None, checks=()):
        spec = self.spec
        chain = self.chain
        itemsize = spec.dtype.itemsize
        chunk_shape = spec.shape
        nbytes = int(np.prod(chunk_shape)) * itemsize
        elen = nbytes + (4 if chain.crc else 0)
        setters = [it[0] for it in complete_items] + [it[0] for it in partial_items]
        dest = _Dest(setters, elen, self.device)
        try:
            launches = []
            if complete_items:
                vstr = [int(s) * itemsize for s in v.stride()]
                items = []
                for i, (bs, sp, csel, osel, _) in enumerate(complete_items):
                    items.append((dest.offs[i], csel, [s.start or 0 for s in osel]))
                t = plan_encode(chain, spec, items, vstr, v.data_ptr())
                launches.append((EncodeLaunch(t.layout, t.chunks, t.sels, v, dest.buf, t.fast, self.device,
                                              t.rows, t.tile, t.tile_prefix), list(range(len(complete_items)))))
            if partial_items:
                tstr = [int(s) * itemsize for s in temp.stride()]
                base = len(complete_items)
                full = tuple(slice(0, s, 1) for s in chunk_shape)
                items = []
                for i in range(len(partial_items)):
                    items.append((dest.offs[base + i], full, [0] * spec.ndim))
                t = plan_encode(chain, spec, items, tstr[1:], temp.data_ptr())
                # the leading temp index goes into out_off
                t.chunks["out_off"] = np.arange(len(partial_items)) * tstr[0]
                launches.append((EncodeLaunch(t.layout, t.chunks, t.sels, temp, dest.buf, t.fast,
                                              self.device, t.rows, t.tile, t.tile_prefix),
                                 [base + i for i in range(len(partial_items))]))
            for l, _ in launches:
                l.launch()
        finally:
            dest.release_lock()
        if pending is not None:  # committed by PendingWrites.finish after one readback
            pending.items.append((dest, setters, launches, elen, spec.config.write_empty_chunks, spec.prototype,
                                  list(checks)))
            return
        nonempty = np.zeros(len(setters), bool)
        for l, idx in launches:
            nonempty[idx] = l.nonempty()
        keep_all = spec.config.write_empty_chunks
        lengths = [elen if (keep_all or nonempty[i]) else 0 for i in range(len(setters))]
        dest.finish(setters, lengths, spec.prototype)

    def _encode_shards(self, complete_items, partial_items, v, temp, present, partial_encode,
                       repairs=(), raws=None):
        torch = _torch()
        spec = self.spec
        chain = self.chain
        sh = chain.shard
        inner = chain.inner
        itemsize = spec.dtype.itemsize
        shard_shape = spec.shape
        cps = sh.chunks_per_shard(shard_shape)
        n_inner = int(np.prod(cps))
        inner_shape = sh.chunk_shape
        nbytes = int(np.prod(inner_shape)) * itemsize
        elen = nbytes + (4 if inner.crc else 0)
        index_size = sh.shard_index_size(n_inner)
        data_start = index_size if sh.index_location == "start" else 0
        blob_max = n_inner * elen + index_size
        # rank -> inner coords in the codec's subchunk_write_order (sharding.py:1090-1107;
        # morton unless the caller chose otherwise -- it is not part of the metadata)
        order = subchunk_order(tuple(cps), sh.subchunk_write_order)
        cstr = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
        slot_of_rank = (order * cstr[None, :]).sum(axis=1)
        rank_of_slot = np.zeros(n_inner, np.uint32)
        rank_of_slot[slot_of_rank] = np.arange(n_inner, dtype=np.uint32)
        setters = [it[0] for it in complete_items] + [it[0] for it in partial_items]
        inner_spec = ArraySpec(inner_shape, spec.dtype, spec.fill_value, spec.config)
        wec = spec.config.write_empty_chunks
        # per (shard, rank): 1 = keep, 0 = elide, -1 = decided by the encode's
        # non-empty flag (and write_empty_chunks).  Partial encode: inner chunks
        # the write does not touch keep their stored state.
        mode = None
        if partial_encode and partial_items:
            mode = np.full((len(setters), n_inner), -1, np.int8)
            base = len(complete_items)
            for j, it in enumerate(partial_items):
                pr = basic_projections(tuple(it[2]), shard_shape, inner_shape)
                touched = np.zeros(n_inner, bool)
                touched[(pr.coords * cstr[None, :]).sum(axis=1)] = True
                keep = present[j] & ~touched
                m = np.where(touched, -1, np.where(keep, 1, 0)).astype(np.int8)
                mode[base + j] = m[slot_of_rank]
        dest = _Dest(setters, blob_max, self.device)
        offs = dest.offs
        try:
            launches = []

            def shard_items(src_items, arr_start_fn, region_fn):
                items = []
                for j, it in enumerate(src_items):
                    blob = offs[it[1]]
                    region = region_fn(j)
                    for r in range(n_inner):
                        ic = order[r]
                        lo = [int(c) * s for c, s in zip(ic, inner_shape)]
                        csel = []
                        for d in range(len(ic)):
                            hi = min(inner_shape[d], max(0, region[d] - lo[d]))
                            csel.append(slice(0, hi, 1))
                        astart = arr_start_fn(j, lo)
                        items.append((blob + data_start + r * elen, tuple(csel), astart))
                return items

            if complete_items:
                vstr = [int(s) * itemsize for s in v.stride()]
                src = [(it, i) for i, it in enumerate(complete_items)]

                def region_c(j):
                    bs, sp, csel, osel, _ = complete_items[j]
                    return [s.stop - (s.start or 0) for s in csel]

                def astart_c(j, lo):
                    osel = complete_items[j][3]
                    return [(s.start or 0) + l for s, l in zip(osel, lo)]

                items = shard_items(src, astart_c, region_c)
                t = plan_encode(inner, inner_spec, items, vstr, v.data_ptr())
                launches.append(EncodeLaunch(t.layout, t.chunks, t.sels, v, dest.buf, t.fast, self.device,
                                             t.rows, t.tile, t.tile_prefix))
            if partial_items:
                tstr = [int(s) * itemsize for s in temp.stride()]
                base = len(complete_items)
                src = [(it, base + i) for i, it in enumerate(partial_items)]
                items = shard_items(src, lambda j, lo: list(lo), lambda j: list(shard_shape))
                t = plan_encode(inner, inner_spec, items, tstr[1:], temp.data_ptr())
                t.chunks["out_off"] += np.repeat(np.arange(len(partial_items)) * tstr[0], n_inner)
                launches.append(EncodeLaunch(t.layout, t.chunks, t.sels, temp, dest.buf, t.fast,
                                             self.device, t.rows, t.tile, t.tile_prefix))
            for l in launches:
                l.launch()
            # untouched inner chunks that failed their check keep their stored
            # bytes (the reference carries them over without decoding them)
            if repairs:
                from .nested import _host_bytes

                base = len(complete_items)
                for i, s in repairs:
                    raw = _host_bytes(raws[i])
                    ib = raw[:index_size] if sh.index_location == "start" else raw[len(raw) - index_size:]
                    off, ln = (int(x) for x in np.frombuffer(ib[: 16 * n_inner].tobytes(), "<u8").reshape(n_inner, 2)[s])
                    if ln != elen:
                        raise ValueError("encoded chunk length does not match the fixed-size codec chain")
                    at = int(offs[base + i]) + data_start + int(rank_of_slot[s]) * elen
                    dest.buf[at: at + elen].copy_(torch.from_numpy(np.array(raw[off: off + ln], np.uint8)).to(dest.buf.device))
            # pack: one workgroup per shard over all launches' inner chunks
            nonempty = torch.cat([l.d_nonempty[: l.n] for l in launches])
            pflags = (N.PF_INDEX_START if sh.index_location == "start" else 0) | \
                (N.PF_INDEX_CRC if sh.index_has_crc else 0)
            if mode is not None:
                d_mode = torch.from_numpy(mode.reshape(-1).astype(np.int32)).to(self.device)
                dec = (nonempty != 0) | wec
                nonempty = torch.where(d_mode < 0, dec.to(torch.int32), d_mode).to(torch.int32).contiguous()
            elif wec:
                pflags |= N.PF_KEEP_EMPTY
            shards = np.zeros(len(setters), dtype=[("blob", "<u8"), ("first", "<u4"), ("_pad", "<u4")])
            shards["blob"] = offs
            shards["first"] = np.arange(len(setters)) * n_inner
            d_shards = _upload(shards, self.device)
            d_rank = _upload(rank_of_slot, self.device)
            d_newrank = torch.empty(max(len(setters) * n_inner, 1), dtype=torch.int32, device=self.device)
            d_blen = torch.zeros(max(len(setters), 1), dtype=torch.int64, device=self.device)
            from .pipeline import _stream_handle

            N.check(N.lib().zhip_shard_pack(launches[0].plan.handle, dest.buf.data_ptr(), d_shards.data_ptr(),
                                            len(setters), n_inner, elen, index_size, pflags,
                                            nonempty.data_ptr(), d_newrank.data_ptr(), d_rank.data_ptr(),
                                            d_blen.data_ptr(), _stream_handle(self.device)),
                    "zhip_shard_pack")
        finally:
            dest.release_lock()
        blen = d_blen[: len(setters)].cpu().numpy()
        dest.finish(setters, blen, spec.prototype)

"""Write path of HipCodecPipeline: FusedCodecPipeline.write_sync
(src/zarr/core/codec_pipeline.py:1174-1253) with the codec compute on the GPU.

Per batch:
  * complete chunks are encoded straight from the (device) value array; the
    part of an edge chunk outside the array is written as the fill value
    (_merge_chunk_array, src/zarr/core/chunk_utils.py:115-162);
  * partial chunks: the existing chunk is decoded on the GPU into a temporary
    (or filled when absent), the value is merged into it with a device copy,
    and the temporary is encoded as a whole chunk;
  * empty chunks (all elements == fill under NDBuffer.all_equal rules) are
    deleted instead of stored unless write_empty_chunks (chunk_utils.py:43-85);
  * sharded arrays: inner chunks are encoded densely in Morton order into the
    shard blob, then one packing launch elides empty inner chunks and writes
    the index + its CRC (sharding.py:716-950); an all-empty shard is deleted.
Encoded bytes land directly in the DeviceStore arena (no copy) or, for host
stores, in a device staging buffer copied back once per batch.
"""

from __future__ import annotations

import numpy as np

from . import _native as N
from .buffer import torch_dtype
from .indexing import subchunk_order
from .planner import SEL_DT, ChainInfo, analyze_chain, plan_encode
from .spec import ArraySpec
from .store import DeviceStore, TAIL_SLACK


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
    """One zhip_encode launch over flat chunk tables."""

    def __init__(self, layout: N.Layout, chunks: np.ndarray, sels: np.ndarray, arr, dst, fast: bool,
                 device, rows: bool = False, tile: bool = False):
        from .pipeline import _rows_map, get_plan

        torch = _torch()
        self.plan = get_plan(layout)
        self.n = len(chunks)
        self.device = device
        self.d_chunks = _upload(chunks, device)
        self.d_sels = _upload(sels if len(sels) else np.zeros(1, SEL_DT), device)
        self.d_status = torch.zeros(max(self.n, 1) * 4, dtype=torch.int32, device=device)
        self.d_ws = torch.zeros(max(self.n, 1) * 4, dtype=torch.int32, device=device)
        self.d_nonempty = torch.zeros(max(self.n, 1), dtype=torch.int32, device=device)
        self.arr = arr
        self.dst = dst
        self.flags = N.DF_FAST_ROWS if fast else 0
        # whole-row batches encode in k_encode_pair through the row map
        self.d_rowmap = _rows_map(self.plan, sels, device) if fast and rows else None
        # k_encode_pair with an even number of units per chunk (<= 32) writes every
        # chunk's non-empty flag itself (last arrival); otherwise flags are OR-ed
        # into a zeroed array
        upc = self.plan.units_per_chunk
        self.flags_by_kernel = self.d_rowmap is not None and upc % 2 == 0 and upc <= 32
        # transposed layouts with full tiles: k_encode_tile4 (also writes every flag)
        if tile and not fast and self.plan.kernel_flags & N.PK_TILE4_ENCODE:
            self.flags |= N.DF_TILE
            self.flags_by_kernel = True

    def launch(self, stream: int | None = None) -> None:
        from .pipeline import _stream_handle

        if self.n == 0:
            return
        if not self.flags_by_kernel:
            self.d_nonempty.zero_()
        s = _stream_handle(self.device) if stream is None else stream
        N.check(N.lib().zhip_encode_mapped(self.plan.handle, self.arr.data_ptr(), self.dst.data_ptr(),
                                           self.d_chunks.data_ptr(), self.n, self.d_sels.data_ptr(),
                                           self.d_status.data_ptr(), self.d_ws.data_ptr(),
                                           self.d_nonempty.data_ptr(), self.flags,
                                           self.d_rowmap.data_ptr() if self.d_rowmap is not None else None,
                                           s), "zhip_encode_mapped")

    def nonempty(self) -> np.ndarray:
        return self.d_nonempty[: self.n].cpu().numpy().astype(bool)


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


def _chunk_region(coords, chunk_shape, array_shape):
    """Data region of a chunk inside the array (edge chunks are clipped)."""
    return tuple(slice(0, min(c, n - i * c)) for i, c, n in zip(coords, chunk_shape, array_shape))


class ChunkWriter:
    """Batch writer for one array (unsharded or sharded chain)."""

    def __init__(self, codecs, spec: ArraySpec, array_shape, device):
        self.chain: ChainInfo = analyze_chain(codecs, spec)
        self.spec = spec
        self.array_shape = tuple(array_shape)
        self.device = device

    def write(self, batch, value, codecs, drop_axes=()) -> None:
        torch = _torch()
        from .pipeline import HipCodecPipeline

        if drop_axes:
            raise NotImplementedError("drop_axes writes are not on the GPU path")
        spec = self.spec
        v = _value_tensor(value, spec.dtype, self.device)
        scalar = v.dim() == 0
        if scalar:
            # the reference writes the scalar into every selected element
            shp = [0] * len(batch[0][3])
            for it in batch:
                for d, s in enumerate(it[3]):
                    shp[d] = max(shp[d], s.stop)
            v = v.expand(tuple(shp)).contiguous() if shp else v.reshape(())
        chunk_shape = spec.shape
        ndim = spec.ndim
        complete_items, partial_items = [], []
        for it in batch:
            bs, sp, csel, osel, is_complete = it
            if is_complete and v.dim() and _is_full_region(csel, osel, chunk_shape):
                complete_items.append(it)
            else:
                partial_items.append(it)
        # partial chunks: decode existing -> merge on device -> encode as complete
        temp = None
        if partial_items:
            pipe = HipCodecPipeline.from_codecs(codecs).evolve_from_array_spec(spec)
            temp = torch.empty((len(partial_items),) + tuple(chunk_shape),
                               dtype=torch_dtype(spec.dtype), device=self.device)
            full = tuple(slice(0, s, 1) for s in chunk_shape)
            for i, (bs, sp, csel, osel, _) in enumerate(partial_items):
                raw = bs.get_sync(prototype=None)
                if raw is None:
                    fv = np.array(spec.fill_value if spec.fill_value is not None else 0,
                                  dtype=spec.dtype.newbyteorder("="))
                    temp[i].copy_(torch.from_numpy(fv.reshape((1,) * len(chunk_shape))).to(
                        self.device).expand(tuple(chunk_shape)))
                else:
                    from .pipeline import _Raw

                    pipe.read_sync([(_Raw(raw), spec, full, full, True)], temp[i])
                temp[i][tuple(csel)] = v[tuple(osel)] if v.dim() else v
        self._encode_chunks(batch, complete_items, partial_items, v, temp)

    def _encode_chunks(self, batch, complete_items, partial_items, v, temp):
        torch = _torch()
        spec = self.spec
        chain = self.chain
        itemsize = spec.dtype.itemsize
        chunk_shape = spec.shape
        if chain.shard is not None:
            return self._encode_shards(complete_items, partial_items, v, temp)
        nbytes = int(np.prod(chunk_shape)) * itemsize
        elen = nbytes + (4 if chain.crc else 0)
        # destination: arena (DeviceStore) or a staging buffer
        store = None
        setters = [it[0] for it in complete_items] + [it[0] for it in partial_items]
        if setters and all(isinstance(getattr(s, "store", None), DeviceStore) for s in setters) and \
                len({id(s.store) for s in setters}) == 1:
            store = setters[0].store
        offs = []
        if store is not None:
            for _ in setters:
                offs.append(store.arena.reserve(elen))
            dst = store.arena.buf
        else:
            top = 0
            for _ in setters:
                offs.append(top)
                top = (top + elen + 255) // 256 * 256
            dst = torch.empty(top + TAIL_SLACK, dtype=torch.uint8, device=self.device)
        launches = []
        if complete_items:
            vstr = [int(s) * itemsize for s in v.stride()]
            items = []
            for i, (bs, sp, csel, osel, _) in enumerate(complete_items):
                items.append((offs[i], csel, [s.start or 0 for s in osel]))
            t = plan_encode(chain, spec, items, vstr, v.data_ptr())
            launches.append((EncodeLaunch(t.layout, t.chunks, t.sels, v, dst, t.fast, self.device, t.rows, t.tile),
                             list(range(len(complete_items)))))
        if partial_items:
            tstr = [int(s) * itemsize for s in temp.stride()]
            base = len(complete_items)
            full = tuple(slice(0, s, 1) for s in chunk_shape)
            items = []
            for i in range(len(partial_items)):
                items.append((offs[base + i], full, [i] + [0] * spec.ndim))
            t = plan_encode(chain, spec, items, tstr[1:], temp.data_ptr())
            # the leading temp index goes into out_off
            t.chunks["out_off"] = np.arange(len(partial_items)) * tstr[0]
            launches.append((EncodeLaunch(t.layout, t.chunks, t.sels, temp, dst, t.fast, self.device, t.rows, t.tile),
                             [base + i for i in range(len(partial_items))]))
        for l, _ in launches:
            l.launch()
        nonempty = np.zeros(len(setters), bool)
        for l, idx in launches:
            nonempty[idx] = l.nonempty()
        keep_all = spec.config.write_empty_chunks
        host = None
        if store is None:
            host = dst.cpu().numpy()
        for i, s in enumerate(setters):
            if not keep_all and not nonempty[i]:
                s.delete_sync()
            elif store is not None:
                store.register(s.path, offs[i], elen)
            else:
                s.set_sync(host[offs[i]: offs[i] + elen].tobytes())

    def _encode_shards(self, complete_items, partial_items, v, temp):
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
        rank_of_slot = np.zeros(n_inner, np.uint32)
        rank_of_slot[(order * cstr[None, :]).sum(axis=1)] = np.arange(n_inner, dtype=np.uint32)
        setters = [it[0] for it in complete_items] + [it[0] for it in partial_items]
        store = None
        if setters and all(isinstance(getattr(s, "store", None), DeviceStore) for s in setters) and \
                len({id(s.store) for s in setters}) == 1:
            store = setters[0].store
        offs = []
        if store is not None:
            for _ in setters:
                offs.append(store.arena.reserve(blob_max))
            dst = store.arena.buf
        else:
            top = 0
            for _ in setters:
                offs.append(top)
                top = (top + blob_max + 255) // 256 * 256
            dst = torch.empty(top + TAIL_SLACK, dtype=torch.uint8, device=self.device)
        inner_spec = ArraySpec(inner_shape, spec.dtype, spec.fill_value, spec.config)
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
            launches.append(EncodeLaunch(t.layout, t.chunks, t.sels, v, dst, t.fast, self.device, t.rows, t.tile))
        if partial_items:
            tstr = [int(s) * itemsize for s in temp.stride()]
            base = len(complete_items)
            src = [(it, base + i) for i, it in enumerate(partial_items)]
            items = shard_items(src, lambda j, lo: list(lo), lambda j: list(shard_shape))
            t = plan_encode(inner, inner_spec, items, tstr[1:], temp.data_ptr())
            t.chunks["out_off"] += np.repeat(np.arange(len(partial_items)) * tstr[0], n_inner)
            launches.append(EncodeLaunch(t.layout, t.chunks, t.sels, temp, dst, t.fast, self.device, t.rows, t.tile))
        for l in launches:
            l.launch()
        # pack: one workgroup per shard over all launches' inner chunks
        nonempty = torch.cat([l.d_nonempty[: l.n] for l in launches])
        shards = np.zeros(len(setters), dtype=[("blob", "<u8"), ("first", "<u4"), ("_pad", "<u4")])
        shards["blob"] = offs
        shards["first"] = np.arange(len(setters)) * n_inner
        d_shards = _upload(shards, self.device)
        d_rank = _upload(rank_of_slot, self.device)
        d_newrank = torch.empty(max(len(setters) * n_inner, 1), dtype=torch.int32, device=self.device)
        d_blen = torch.zeros(max(len(setters), 1), dtype=torch.int64, device=self.device)
        flags = (N.PF_INDEX_START if sh.index_location == "start" else 0) | \
            (N.PF_INDEX_CRC if sh.index_has_crc else 0) | \
            (N.PF_KEEP_EMPTY if spec.config.write_empty_chunks else 0)
        from .pipeline import _stream_handle

        N.check(N.lib().zhip_shard_pack(launches[0].plan.handle, dst.data_ptr(), d_shards.data_ptr(),
                                        len(setters), n_inner, elen, index_size, flags,
                                        nonempty.data_ptr(), d_newrank.data_ptr(), d_rank.data_ptr(),
                                        d_blen.data_ptr(), _stream_handle(self.device)),
                "zhip_shard_pack")
        blen = d_blen[: len(setters)].cpu().numpy()
        host = None if store is not None else dst.cpu().numpy()
        for i, s in enumerate(setters):
            n = int(blen[i])
            if n == 0:
                s.delete_sync()
            elif store is not None:
                store.register(s.path, offs[i], n)
            else:
                s.set_sync(host[offs[i]: offs[i] + n].tobytes())


def _is_full_region(csel, osel, chunk_shape) -> bool:
    for s in csel:
        if isinstance(s, (int, np.integer)):
            return False
        if (s.start or 0) != 0 or (s.step or 1) != 1:
            return False
    return True


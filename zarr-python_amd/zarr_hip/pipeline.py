"""HipCodecPipeline: the drop-in CodecPipeline (src/zarr/abc/codec.py:315-508).

Same surface as the reference's FusedCodecPipeline (codec_pipeline.py:950-1355):
``from_codecs`` / ``evolve_from_array_spec`` / ``validate`` /
``compute_encoded_size`` / ``supports_partial_decode`` / ``read`` / ``read_sync`` /
``write`` / ``write_sync`` / ``decode`` / ``encode``.  The codec compute runs on
the GPU: ``read`` plans the whole batch on the host (planner.py), uploads the
flat tables once and launches one fused decode kernel per batch (plus one
shard-index verification launch for sharded batches).  Errors surface as the
reference's exceptions after the batch completes.

``prepare_read`` exposes the device-resident program so a caller (bench.py,
repeated reads of the same selection) can re-launch without re-planning.
"""

from __future__ import annotations

import asyncio
import os
import threading
import warnings
import weakref
from dataclasses import dataclass, field, replace
from typing import Any, Iterable

import numpy as np

from . import _native as N
from . import staging
from .codecs import (ShardingCodec, TransposeCodec, evolve_codecs, is_v2_codec, parse_codecs, split_codecs,
                     split_host_tail)
from .interop import device_tensor, host_array
from .planner import CHUNK_DT, SEL_DT, STATUS_DT, ChainInfo, Tables, analyze_chain, plan_decode, predict_rows
from .spec import ArraySpec, GetResult, coerce_spec
from .store import DeviceRef, DeviceStore, _resolve_range


def _torch():
    import torch

    return torch


def _stream_handle(device) -> int:
    """The raw HIP stream torch treats as current on `device`."""
    torch = _torch()
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is None:
        return int(torch.cuda.current_stream(device).cuda_stream)
    idx = device if isinstance(device, int) else getattr(device, "index", None)
    return int(raw(torch.cuda.current_device() if idx is None else idx))


def _upload(arr: np.ndarray, device):
    torch = _torch()
    b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    t = torch.empty(max(b.size, 16), dtype=torch.uint8, device=device)
    if b.size:
        t[: b.size].copy_(torch.from_numpy(b.copy()))
    return t


# device buffers of per-call reads, reused (read_sync with the plan cache off
# or missed): table blocks by power-of-two size, zeroed status / workspace
# blocks by exact size -- returned only after a launch whose results came back
# clean, so a reused workspace is zero and its error word clear
_BUF_POOL: dict = {}
_BUF_POOL_MAX = 8


def _dev_key(device) -> int:
    idx = getattr(device, "index", device)
    return _torch().cuda.current_device() if idx is None else int(idx)


def _pool_take(kind: str, n: int, device, dtype):
    torch = _torch()
    key = (kind, n, _dev_key(device))
    try:  # (list.pop is atomic: two threads never take the same buffer)
        return _BUF_POOL.get(key, []).pop()
    except IndexError:
        pass
    if kind.startswith("z"):
        return torch.zeros(n, dtype=dtype, device=device)
    return torch.empty(n, dtype=dtype, device=device)


def _pool_give(kind: str, t) -> None:
    key = (kind, t.numel(), t.device.index)
    lst = _BUF_POOL.setdefault(key, [])
    if len(lst) < _BUF_POOL_MAX:
        lst.append(t)


class _Upload:
    """Several host tables in ONE host -> device copy (256-byte aligned parts
    of one device buffer): zhip_upload packs them into a page-locked buffer
    of the library's, instead of one pageable copy each."""

    def __init__(self, device, pooled: bool = False):
        self.device = device
        self.parts: list = []
        self.top = 0
        self.pooled = pooled
        self.dev = None

    def add(self, arr: np.ndarray) -> int:
        b = arr if arr.flags.c_contiguous else np.ascontiguousarray(arr)
        off = self.top
        self.parts.append((off, b))
        self.top = (off + max(b.nbytes, 16) + 255) // 256 * 256
        return len(self.parts) - 1

    def commit(self, stream: int) -> list:
        """Device addresses of the parts (the device buffer is self.dev)."""
        import ctypes

        torch = _torch()
        total = max(self.top, 16)
        if self.pooled:
            cap = 1 << max(12, (total - 1).bit_length())
            self.dev = _pool_take("t", cap, self.device, torch.uint8)
        else:
            self.dev = torch.empty(total, dtype=torch.uint8, device=self.device)
        n = len(self.parts)
        # one ctypes block: [host pointers][sizes][offsets]
        arg = (ctypes.c_uint64 * (3 * n))(*([b.ctypes.data for _, b in self.parts] +
                                           [b.nbytes for _, b in self.parts] + [o for o, _ in self.parts]))
        a = ctypes.addressof(arg)
        base = self.dev.data_ptr()
        N.check(N.lib().zhip_upload(a, a + 8 * n, a + 16 * n, n, base, total, stream), "zhip_upload")
        return [base + o for o, _ in self.parts]


def crc_error_message(stored: int, computed: int) -> str:
    """The reference's message (src/zarr/codecs/crc32c_.py:46-49)."""
    s = np.uint32(stored).tobytes()
    c = np.uint32(computed).tobytes()
    return f"Stored and computed checksum do not match. Stored: {s!r}. Computed: {c!r}."


_PLAN_CACHE: dict = {}


def get_plan(layout: N.Layout) -> N.Plan:
    """Plans are cached per (layout bytes, device): building them is host math +
    one small upload, kept off the timed path.  A layout object also keeps its
    plans (the per-geometry layouts of the native planner are reused across
    calls: no key bytes to build)."""
    torch = _torch()
    dev = torch.cuda.current_device()
    mine = layout.__dict__.get("_zplans")
    if mine is not None:
        p = mine.get(dev)
        if p is not None:
            return p
    key = (bytes(layout), dev)
    p = _PLAN_CACHE.get(key)
    if p is None:
        p = N.Plan(layout, upload=True)
        _PLAN_CACHE[key] = p
    if mine is None:
        mine = layout.__dict__.setdefault("_zplans", {})
    mine[dev] = p
    return p


def _kernel_flags(layout: N.Layout) -> int:
    """zhip_plan_kernel_flags of the layout's plan, memoised on the plan."""
    p = get_plan(layout)
    f = getattr(p, "_pk", None)
    if f is None:
        f = p._pk = p.kernel_flags
    return f


def _rows_map_host(plan, sels: np.ndarray):
    """zhip_rows_map over the host copy of the selections; None when the
    library declines the layout (then the launch takes the persistent row
    decode)."""
    n_sels = max(len(sels), 1)
    if not len(sels):
        sels = np.zeros(1, SEL_DT)
    sels = np.ascontiguousarray(sels)
    n = int(N.lib().zhip_rows_map_len(plan.handle, n_sels))
    if n == 0:
        return None
    host = np.zeros(n, N.ROWBLK_DT)
    rc = N.lib().zhip_rows_map(plan.handle, sels.ctypes.data, n_sels, host.ctypes.data, n)
    if rc == N.E_UNSUPPORTED:
        return None
    N.check(rc, "zhip_rows_map")
    return host


def _whole_sels(layout: N.Layout, sels: np.ndarray) -> bool:
    """Every selection of the (deduplicated) table is its chunk's whole
    region -- start 0, count = chunk shape, unit steps -- so a row-map launch
    may take ZHIP_DF_WHOLE (destinations computed from the plan's affine form
    of the whole-chunk map instead of loaded from the map)."""
    if len(sels) != 1:
        return False
    nd = layout.ndim
    s = sels[0]
    shape = np.array(layout.shape[:nd])
    return bool((s["start"][:nd] == 0).all() and (s["count"][:nd] == shape).all() and (s["step"][:nd] == 1).all())


def _rows_map(plan, sels: np.ndarray, device):
    """_rows_map_host, uploaded."""
    host = _rows_map_host(plan, sels)
    return None if host is None else _upload(host, device)


class DecodeLaunch:
    """One zhip_decode launch with its device-resident tables."""

    def __init__(self, layout: N.Layout, chunks: np.ndarray, sels: np.ndarray, src, src_size: int,
                 out, fast: bool, device, tile: bool = False, index_chunks: np.ndarray | None = None,
                 rows: bool = False, predict: "N.Predict | None" = None, pooled: bool = False):
        torch = _torch()
        self.plan = get_plan(layout)
        self.pooled = pooled
        self.n = len(chunks)
        self.device = device
        # shard-index CRC checks fused into this launch (zhip_decode_indexed)
        self.n_idx = 0 if index_chunks is None else len(index_chunks)
        self.src = src
        self.src_size = src_size
        self.out = out
        # (DF_DEFER: this path reads the deferred CRC verdict words back with the
        # error word, results_fast / merge_verdicts, and alternates the banks)
        self.flags = (N.DF_FAST_ROWS if fast else 0) | (N.DF_TILE if tile else 0) | \
            (N.DF_ROWS if fast and rows else 0) | N.DF_DEFER
        self.predict = predict if (fast and rows) else None
        # row map (zhip_rows_map): per (selection, unit, step) destinations for the
        # two-unit row decode; None when the layout does not admit one
        rowmap = _rows_map_host(self.plan, sels) if fast and rows else None
        if rowmap is not None and _whole_sels(layout, sels):
            self.flags |= N.DF_WHOLE
        # every table in one host -> device copy; statuses and workspaces in
        # one zeroed buffer.  The launches take plain addresses (p_*); the d_*
        # tensor views are built on demand (result checks, tests, tools).
        up = _Upload(device, pooled)
        sels = sels if len(sels) else np.zeros(1, SEL_DT)
        i_ch = up.add(chunks)
        i_sel = up.add(sels)
        i_idx = up.add(index_chunks) if self.n_idx else None
        i_map = up.add(rowmap) if rowmap is not None else None
        ptrs = up.commit(_stream_handle(device))
        self._tb = up.dev
        self._tparts = {"chunks": (ptrs[i_ch], chunks.nbytes), "sels": (ptrs[i_sel], sels.nbytes)}
        self.p_chunks, self.p_sels = ptrs[i_ch], ptrs[i_sel]
        self.p_idx_chunks = ptrs[i_idx] if i_idx is not None else None
        self.p_rowmap = ptrs[i_map] if i_map is not None else None
        if i_idx is not None:
            self._tparts["idx_chunks"] = (ptrs[i_idx], index_chunks.nbytes)
        if i_map is not None:
            self._tparts["rowmap"] = (ptrs[i_map], rowmap.nbytes)
        nw = max(self.n, 1) * 4
        self.ws_words = max(4, self.plan.workspace_words)  # zhip_plan_info
        nws = max(self.n, 1) * self.ws_words
        ni = self.n_idx * 4
        # [statuses][error word, pad to 256 B][workspace][index statuses]: the
        # error word and the chunks' deferred-verdict words (the first 4 words
        # per chunk of the workspace, zarrhip.h) are one contiguous range, read
        # back with one copy after a launch
        # pooled per region split, not per total size: after a clean launch the
        # workspace is zero again (self-resetting) but the statuses are not, so
        # a buffer may only go to a launch whose statuses and workspace sit at
        # the same offsets -- there every status is rewritten, as on any
        # relaunch of one program (a split-blind pool handed one program's
        # statuses to another as verdict words: a false CRC mismatch, found by
        # the rectilinear fuzz, tests/test_gpu_fuzz.py)
        self._zkind = f"z:{nw}:{nws}:{ni}"
        z = _pool_take(self._zkind, nw + 64 + nws + ni, device, torch.int32) if pooled else \
            torch.zeros(nw + 64 + nws + ni, dtype=torch.int32, device=device)
        self._z = z
        self._zl = (nw, nws, ni)
        self._bufs = (up.dev, z) if pooled else None
        zp = z.data_ptr()
        self.p_status, self.p_err, self.p_ws = zp, zp + 4 * nw, zp + 4 * (nw + 64)
        self.p_idx_status = zp + 4 * (nw + 64 + nws) if self.n_idx else None
        # error word .. last chunk's verdict words
        self.verdict_range = (self.p_err, 4 * (64 + 4 * self.n))
        self._bank = 0  # deferred-verdict bank of the next launch (alternates)
        self._ranges: list = []  # (first, count) of launch_range calls since the last statuses()

    def _tview(self, name: str):
        part = self._tparts.get(name)
        if part is None:
            return None
        off = part[0] - self._tb.data_ptr()
        return self._tb[off: off + max(part[1], 16)]

    d_chunks = property(lambda self: self._tview("chunks"))
    d_sels = property(lambda self: self._tview("sels"))
    d_idx_chunks = property(lambda self: self._tview("idx_chunks"))
    d_rowmap = property(lambda self: self._tview("rowmap"))
    d_status = property(lambda self: self._z[: self._zl[0]])
    d_err = property(lambda self: self._z[self._zl[0]: self._zl[0] + 4])
    d_ws = property(lambda self: self._z[self._zl[0] + 64: self._zl[0] + 64 + self._zl[1]])
    d_verdict = property(lambda self: self._z[self._zl[0]: self._zl[0] + 64 + 4 * self.n])
    d_idx_status = property(lambda self: self._z[self._zl[0] + 64 + self._zl[1]:
                                                 self._zl[0] + 64 + self._zl[1] + self._zl[2]])

    def launch(self, stream: int | None = None) -> None:
        if self.n == 0:
            return
        LAUNCHES[0] += 1
        s = _stream_handle(self.device) if stream is None else stream
        out_ptr = self.out.data_ptr() if self.out is not None else None
        # deferred CRC verdicts (zarrhip.h): consecutive launches publish into
        # alternate workspace banks (also while captured into a graph)
        flags = self.flags | (N.DF_BANK1 if self._bank else 0)
        self._bank ^= 1
        src = self.src.data_ptr()
        if self.p_rowmap is not None:
            N.check(N.lib().zhip_decode_mapped(
                self.plan.handle, src, self.src_size, out_ptr, self.p_chunks, self.n, self.p_sels,
                self.p_status, self.p_ws, self.p_err, self.p_idx_chunks, self.n_idx, self.p_idx_status, flags,
                self.predict, self.p_rowmap, s), "zhip_decode_mapped")
            return
        if self.predict is not None:
            N.check(N.lib().zhip_decode_predicted(
                self.plan.handle, src, self.src_size, out_ptr, self.p_chunks, self.n, self.p_sels,
                self.p_status, self.p_ws, self.p_err, self.p_idx_chunks, self.n_idx, self.p_idx_status, flags,
                self.predict, s), "zhip_decode_predicted")
            return
        if self.n_idx:
            N.check(N.lib().zhip_decode_indexed(
                self.plan.handle, src, self.src_size, out_ptr, self.p_chunks, self.n, self.p_sels,
                self.p_status, self.p_ws, self.p_err, self.p_idx_chunks, self.n_idx, self.p_idx_status, flags,
                s), "zhip_decode_indexed")
            return
        N.check(N.lib().zhip_decode(self.plan.handle, src, self.src_size, out_ptr, self.p_chunks, self.n,
                                    self.p_sels, self.p_status, self.p_ws, self.p_err, flags, s), "zhip_decode")

    def launch_range(self, first: int, count: int, src, src_size: int, stream: int | None = None) -> None:
        """Chunks [first, first + count) of the table, reading from `src` (the
        slab pipeline: one plan, one staging buffer per slab).  Statuses and
        workspace regions are the same slices a whole launch uses.  Plain
        launches only (no fused index checks, no load prediction)."""
        if count == 0:
            return
        LAUNCHES[0] += 1
        assert self.n_idx == 0 and self.predict is None
        self._ranges.append((first, count))  # where this range's verdict words live (statuses())
        s = _stream_handle(self.device) if stream is None else stream
        out_ptr = self.out.data_ptr() if self.out is not None else None
        chunks = self.p_chunks + first * CHUNK_DT.itemsize
        status = self.p_status + first * 16
        ws = self.p_ws + first * self.ws_words * 4
        flags = self.flags | (N.DF_BANK1 if self._bank else 0)
        if self.p_rowmap is not None:
            N.check(N.lib().zhip_decode_mapped(
                self.plan.handle, src.data_ptr(), src_size, out_ptr, chunks, count, self.p_sels,
                status, ws, self.p_err, None, 0, None, flags, None, self.p_rowmap, s), "zhip_decode_mapped")
            return
        N.check(N.lib().zhip_decode(self.plan.handle, src.data_ptr(), src_size, out_ptr, chunks, count,
                                    self.p_sels, status, ws, self.p_err, flags, s), "zhip_decode")

    def release(self) -> None:
        """Give pooled buffers back (after a clean result check; the launch
        must not be used again)."""
        if self._bufs is not None:
            tb, z = self._bufs
            self._bufs = None
            if tb is not None:
                _pool_give("t", tb)
            _pool_give(self._zkind, z)

    def statuses(self) -> np.ndarray:
        """Per-chunk statuses with the deferred CRC verdicts merged in: a
        nonzero verdict word w of bank b is a mismatch with stored trailer s_b,
        computed w ^ s_b (zarrhip.h); such words are cleared, so the next
        launch starts clean."""
        SYNCS[0] += 1
        st = self.d_status[: self.n * 4].cpu().numpy().view(STATUS_DT).copy()
        if self._ranges:  # range launches: chunk first + c's words at first * wsw + 4 c
            wsw = self.ws_words
            for first, count in self._ranges:
                self.merge_verdicts(st[first: first + count],
                                    self.d_ws[first * wsw: first * wsw + 4 * count].cpu().numpy().view(np.uint32),
                                    self.d_ws[first * wsw: first * wsw + 4 * count])
            self._ranges = []
        else:
            self.merge_verdicts(st, self.d_ws[: self.n * 4].cpu().numpy().view(np.uint32))
        return st

    def merge_verdicts(self, st: np.ndarray, ws: np.ndarray, dev_ws=None) -> bool:
        """Fold verdict words (the workspace's first 4 words per chunk, host
        copy) into host statuses; True (and the device words cleared) when one
        was set."""
        w = ws.reshape(-1, 4)
        bad = (w[:, 0] != 0) | (w[:, 2] != 0)
        if not bad.any():
            return False
        for c in np.nonzero(bad)[0]:
            b = 0 if w[c, 0] != 0 else 2
            st[c]["code"] = N.ST_CRC_MISMATCH
            st[c]["stored"] = w[c, b + 1]
            st[c]["computed"] = w[c, b] ^ w[c, b + 1]
        (self.d_ws[: self.n * 4] if dev_ws is None else dev_ws).view(-1, 4)[:, 0::2].zero_()
        return True

    def index_statuses(self) -> np.ndarray:
        SYNCS[0] += 1
        return self.d_idx_status[: self.n_idx * 4].cpu().numpy().view(STATUS_DT)

    def errflag(self) -> int:
        SYNCS[0] += 1
        return int(self.d_err[0].item())

    def reset_errflag(self):
        self.d_err.zero_()


@dataclass
class DecodeProgram:
    """A planned batch: resident tables + launches; launch() is the hot path."""

    tables: Tables
    data: DecodeLaunch
    index: DecodeLaunch | None
    n_items: int
    sharded: bool
    item_missing: np.ndarray
    keepalive: list = field(default_factory=list)
    pending: Any = None  # staging.Pending: host bytes still on their way to HBM
    clean: bool = False  # the last results_fast found no error
    # ((DeviceArena, gen), ...) of the device stores the batch reads: a launch
    # after any of them changed placements would read moved or reused bytes
    generations: tuple = ()

    def stale(self) -> bool:
        return any(a.gen != g for a, g in self.generations)

    def check_fresh(self) -> None:
        if self.stale():
            raise RuntimeError("the device store changed since this read was planned (a key was written or "
                               "deleted, its bytes may have moved): plan the read again")

    def launch(self, stream: int | None = None) -> None:
        self.check_fresh()
        if self.pending is not None:
            self.pending.finish(stream)  # the launch stream waits for the staged copies
            self.pending = None
        if self.index is not None:
            self.index.launch(stream)
        self.data.launch(stream)

    def retarget(self, out) -> None:
        """Point the data launch at another out of the same shape, strides,
        dtype and 16-byte alignment class (the tables hold out offsets, not
        addresses; the kernel choice depends only on the alignment), or at
        None to drop the reference (the per-call plan cache keeps programs,
        not outs)."""
        self.data.out = out

    def results_fast(self) -> tuple[GetResult, ...]:
        """results() for the per-call path: synchronise on ONE copy back per
        launch -- the data launch's error word and its chunks' deferred CRC
        verdict words (one contiguous range, zarrhip.h), the index launch's
        error word -- and read the full status table only when one is set.
        Missing items are known on the host at planning (absent keys, absent
        shards), so the GetResults are prebuilt."""
        w = getattr(self, "_err_ranges", None)
        if w is None:
            w = self._err_ranges = _RangeSet(self.wait_ranges())
        return self.results_from_words(w.wait(self.data.device))

    def wait_ranges(self) -> list:
        """The device ranges results_fast reads back: (pointer, bytes)."""
        rngs = [self.data.verdict_range]
        if self.index is not None:
            rngs.append((self.index.p_err, 4))
        return rngs

    def results_from_words(self, host: np.ndarray) -> tuple[GetResult, ...]:
        """results_fast's verdict on the host copy of wait_ranges()."""
        nv = self.data.verdict_range[1] // 4
        err = int(host[0]) | (int(host[nv]) if self.index is not None else 0)
        dv = host[64:nv]
        if err or (dv.size and (dv[0::2].any())):
            self.data.reset_errflag()
            if self.index is not None:
                self.index.reset_errflag()
            return self.results()
        ok = getattr(self, "_ok_results", None)
        if ok is None:
            ok = tuple(GetResult(status="missing" if m else "present") for m in self.item_missing)
            self._ok_results = ok
        self.clean = True
        return ok

    def release(self) -> None:
        """Pooled buffers back to the per-call pool (the program is done)."""
        self.data.release()
        if self.index is not None:
            self.index.release()

    def results(self) -> tuple[GetResult, ...]:
        """Synchronise, then raise like the reference or return per-item statuses."""
        data_st = self.data.statuses()  # first: consumes (clears) the deferred verdicts
        st = None
        if self.index is not None:
            st = self.index.statuses()
        elif self.data.n_idx:
            st = self.data.index_statuses()
        if st is not None:
            bad = np.nonzero(st["code"] != N.ST_OK)[0]
            if len(bad):
                r = st[bad[0]]
                raise ValueError(crc_error_message(int(r["stored"]), int(r["computed"])))
        st = data_st
        codes = st["code"]
        bad = np.nonzero((codes != N.ST_OK) & (codes != N.ST_MISSING))[0]
        if len(bad):
            j = bad[0]
            r = st[j]
            if r["code"] == N.ST_CRC_MISMATCH:
                raise ValueError(crc_error_message(int(r["stored"]), int(r["computed"])))
            if r["code"] == N.ST_INDEX_OOB:
                raise ValueError("shard index entry points outside the shard blob")
            raise ValueError("encoded chunk length does not match the fixed-size codec chain "
                             f"(chunk {int(self.tables.item_of_chunk[j])})")
        out = []
        if self.sharded:
            for i in range(self.n_items):
                out.append(GetResult(status="missing" if self.item_missing[i] else "present"))
        else:  # one entry per item (entries may be reordered: item_of_chunk maps back)
            by_item = np.full(self.n_items, N.ST_OK, np.uint32)
            by_item[self.tables.item_of_chunk] = codes
            for i in range(self.n_items):
                out.append(GetResult(status="missing" if by_item[i] == N.ST_MISSING else "present"))
        return tuple(out)


class ProgramGroup:
    """The planned read of a batch whose items carry different chunk specs
    (spec_groups): one DecodeProgram per spec group, all over the same out
    (the groups' out selections are disjoint), launched back to back on one
    stream; results come back in the batch's item order."""

    def __init__(self, programs: list, groups: list, n_items: int):
        self.programs = programs
        self.groups = groups
        self.n_items = n_items

    @property
    def data_launches(self) -> list:
        return [d for p in self.programs for d in getattr(p, "data_launches", [p.data])]

    @property
    def data(self):
        return self.programs[0].data

    @property
    def clean(self) -> bool:
        return all(p.clean for p in self.programs)

    def stale(self) -> bool:
        return any(p.stale() for p in self.programs)

    def check_fresh(self) -> None:
        for p in self.programs:
            p.check_fresh()

    def launch(self, stream: int | None = None) -> None:
        for p in self.programs:
            p.launch(stream)

    def retarget(self, out) -> None:
        for p in self.programs:
            p.retarget(out)

    def release(self) -> None:
        for p in self.programs:
            p.release()

    def _merge(self, per_group) -> tuple:
        out = [None] * self.n_items
        for idx, res in zip(self.groups, per_group):
            for i, r in zip(idx, res):
                out[i] = r
        return tuple(out)

    def results(self) -> tuple[GetResult, ...]:
        return self._merge([p.results() for p in self.programs])

    def results_fast(self) -> tuple[GetResult, ...]:
        """Every group's error word and verdict words come back in ONE
        synchronisation (one zhip_wait_ranges over all the programs' ranges);
        the status tables are read only for a group that reports an error."""
        progs = self.programs
        if not all(isinstance(p, DecodeProgram) for p in progs):
            return self._merge([p.results_fast() for p in progs])
        w = getattr(self, "_err_ranges", None)
        if w is None:
            per = [p.wait_ranges() for p in progs]
            w = self._err_ranges = (_RangeSet([r for rs in per for r in rs]),
                                    [sum(r[1] for r in rs) // 4 for rs in per])
        host = w[0].wait(progs[0].data.device)
        res, pos = [], 0
        for p, n in zip(progs, w[1]):
            res.append(p.results_from_words(host[pos: pos + n]))
            pos += n
        return self._merge(res)


# host-side count of decode launches issued (DecodeLaunch.launch /
# launch_range): tests check that a batch costs one launch per spec group
LAUNCHES = [0]
# host-side count of the read path's blocking device-to-host readbacks
# (_RangeSet.wait, status tables, error words): tests check that a batch of
# several spec groups costs ONE synchronisation
SYNCS = [0]


class _RangeSet:
    """Device ranges (pointer, bytes) read back by ONE zhip_wait_ranges: the
    stream's work drains, then every range lands in one host array (uint32)."""

    def __init__(self, rngs: list):
        import ctypes

        n = len(rngs)
        self.ptrs = (ctypes.c_void_p * n)(*[r[0] for r in rngs])
        self.lens = (ctypes.c_uint64 * n)(*[r[1] for r in rngs])
        self.n = n
        self.host = np.zeros(sum(r[1] for r in rngs) // 4, np.uint32)

    def wait(self, device) -> np.ndarray:
        SYNCS[0] += 1
        N.check(N.lib().zhip_wait_ranges(self.ptrs, self.lens, self.n, self.host.ctypes.data,
                                         _stream_handle(device)), "zhip_wait_ranges")
        return self.host


def _dv_refs(launches: list, device):
    """A device array of zhip_dv_ref (zarrhip.h) for DecodeLaunches."""
    torch = _torch()
    dt = np.dtype([("ws", "<u8"), ("status", "<u8"), ("err", "<u8"), ("n", "<u4"), ("pad", "<u4")])
    a = np.zeros(len(launches), dt)
    for i, d in enumerate(launches):
        a[i] = (d.p_ws, d.p_status, d.p_err, d.n, 0)
    return torch.from_numpy(a.view(np.uint8).copy()).to(device)


class ReadGraph:
    """A read loop captured once as a hipGraph and replayed with one launch.

    ``programs`` are planned reads (``prepare_read``); the graph holds
    ``repeats`` launches cycling over them, in order, on one stream.  Replaying
    it does exactly the work of the eager loop (every launch a full decode with
    CRC verification and statuses), without one host-side launch per batch —
    the HIP-graph counterpart of re-issuing the same read in a data-loader
    loop.  Statuses accumulate in each program's device tables; call
    ``results()`` to raise like the reference after a replay.
    """

    def __init__(self, programs: list, repeats: int, device=None):
        torch = _torch()
        if not programs or repeats < 1:
            raise ValueError("ReadGraph needs at least one program and one repeat")
        self.programs = list(programs)
        self.repeats = int(repeats)
        self.device = device if device is not None else self.programs[0].data.device
        self.graph = torch.cuda.CUDAGraph()
        self.stream = torch.cuda.Stream(self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        # deferred CRC verdicts (zarrhip.h): consecutive launches of a program
        # alternate banks and each checks the previous one; a program launched
        # an odd number of times would start the next replay in the bank its
        # last launch left unchecked, so the graph then ends with one
        # zhip_dv_check node over every program's workspace
        counts = [len(range(j, self.repeats, len(self.programs))) for j in range(len(self.programs))]
        launches = [getattr(p, "data_launches", None) or [getattr(p, "data", None)] for p in self.programs]
        odd = any(c % 2 for c, ds in zip(counts, launches) for d in ds if d is not None and hasattr(d, "d_ws"))
        self._dv_refs = _dv_refs([d for ds in launches for d in ds if d is not None], self.device) if odd \
            else None
        with torch.cuda.device(self.device):
            with torch.cuda.graph(self.graph, stream=self.stream):
                for i in range(self.repeats):
                    self.programs[i % len(self.programs)].launch()
                if self._dv_refs is not None:
                    N.check(N.lib().zhip_dv_check(self._dv_refs.data_ptr(), self._dv_refs.numel() // 32,
                                                  int(self.stream.cuda_stream)), "zhip_dv_check")

    def replay(self) -> None:
        for p in self.programs:  # the graph holds the programs' planned offsets
            chk = getattr(p, "check_fresh", None)  # (any object with launch / results replays)
            if chk is not None:
                chk()
        self.graph.replay()

    def results(self) -> list:
        _torch().cuda.synchronize(self.device)
        return [p.results() for p in self.programs]


def _parse_devices(devices) -> tuple:
    """A device list (ints, "cuda:i" strings or torch devices, or a comma
    string "0,1,2") -> tuple of device indices."""
    if devices is None or devices == "" or devices == ():
        return ()
    if isinstance(devices, str):
        devices = [d for d in devices.replace(" ", "").split(",") if d]
    out = []
    for d in devices:
        if isinstance(d, str):
            out.append(int(d.split(":")[-1]))
        elif isinstance(d, (int, np.integer)):
            out.append(int(d))
        else:  # a torch.device
            out.append(int(d.index or 0))
    return tuple(out)


def _config_devices() -> tuple:
    """zarr's config key "hip.devices" when zarr is importable, else its
    environment form ZARR_HIP__DEVICES (donfig's mapping of nested keys)."""
    v = os.environ.get("ZARR_HIP__DEVICES")
    z = _ZARR_CONFIG.get("z", 0)
    if z == 0:  # import once (absent on this image's Python)
        try:
            import zarr as z
        except Exception:
            z = None
        _ZARR_CONFIG["z"] = z
    if z is not None:
        try:
            v = z.config.get("hip.devices", v)
        except Exception:
            pass
    return _parse_devices(v)


_ZARR_CONFIG: dict = {}


IL_PREDICT = os.environ.get("ZARR_HIP_IL_PREDICT", "0") == "1"

# entries of the per-call plan cache (per pipeline instance); 0 disables it
READ_CACHE_SIZE = int(os.environ.get("ZARR_HIP_READ_CACHE", "16"))


def _sel_key(sel):
    """A hashable image of a basic selection (slices are unhashable before
    Python 3.12); None for selections the cache does not key (arrays)."""
    out = []
    for s in sel:
        t = type(s)
        if t is slice:
            out.append((s.start, s.stop, s.step))
        elif t is int or isinstance(s, (int, np.integer)):
            out.append(int(s))
        else:
            return None
    return tuple(out)


def _read_key(batch: list, dev_out, drop_axes):
    """Cache key of a device-resident read, or None when it is not cacheable
    (getters without a store path, array selections).  The out enters by
    geometry and 16-byte alignment only (see DecodeProgram.retarget)."""
    spec = batch[0][1]
    fv = spec.fill_value
    parts = [spec.shape, spec.dtype.str, type(fv).__name__, repr(fv), spec.config, tuple(drop_axes),
             tuple(dev_out.shape), tuple(dev_out.stride()), str(dev_out.dtype), dev_out.data_ptr() % 16,
             str(dev_out.device)]
    for it in batch:
        bg = it[0]
        st = getattr(bg, "store", None)
        if not isinstance(st, DeviceStore):
            return None
        cs, os_ = _sel_key(it[2]), _sel_key(it[3])
        if cs is None or os_ is None or it[1] is not spec and it[1] != spec:
            return None
        # the store enters by weak reference: a dead store's key never matches a
        # new store that happens to reuse its address (dead weakrefs compare by
        # identity), and _read_cached drops entries whose store died
        parts.append((_store_ref(st), bg.path, cs, os_, bool(it[4])))
    return tuple(parts)


def _one_device_store(batch: list, device):
    """(store, srcs) when every item is a StorePath into ONE DeviceStore on
    `device` (the per-call read of a device-resident array): the placements
    straight from its index, no per-item getter chain; else None."""
    from .store import StorePath

    bg0 = batch[0][0]
    if type(bg0) is not StorePath:
        return None
    st = bg0.store
    if type(st) is not DeviceStore or not _same_device(st.device, device):
        return None
    idx = st._index
    srcs = []
    for it in batch:
        bg = it[0]
        if type(bg) is not StorePath or bg.store is not st:
            return None
        v = idx.get(bg.path)
        srcs.append((0, 0, True) if v is None else (v[0], v[1], False))
    if all(s[2] for s in srcs):
        return None  # nothing present: the general path's zero-source handling
    return st, srcs


def _store_ref(st):
    r = getattr(st, "_zhip_wref", None)
    if r is None or r() is not st:
        r = weakref.ref(st)
        try:
            st._zhip_wref = r
        except AttributeError:
            pass
    return r


def _key_alive(key) -> bool:
    return all(p[0]() is not None for p in key[11:])


def _generations(batch: list) -> tuple:
    """((arena, gen), ...) of the DeviceStore arenas a batch reads."""
    seen: dict = {}
    for it in batch:
        bg = it[0]
        st = getattr(bg, "store", None)
        arena = st.arena if isinstance(st, DeviceStore) else (
            bg.value.arena if isinstance(bg, _Raw) and isinstance(bg.value, DeviceRef) else None)
        if arena is not None and id(arena) not in seen:
            seen[id(arena)] = (arena, arena.gen)
    return tuple(seen.values())


def _same_arenas(prog, batch: list) -> bool:
    """The arenas a cached program was planned against are the batch's arenas
    now (object identity, not addresses)."""
    now = _generations(batch)
    return len(now) == len(prog.generations) and all(
        a is b for (a, _), (b, _) in zip(now, prog.generations))


def _same_device(a, b) -> bool:
    torch = _torch()
    ia = a.index if a.index is not None else torch.cuda.current_device()
    ib = b.index if b.index is not None else torch.cuda.current_device()
    return a.type == b.type and ia == ib


def _device_resident(batch: list, device=None) -> bool:
    """True when every ByteGetter reads from a DeviceStore (bytes already in HBM)
    -- on `device`, when given: another GPU's bytes are copied, never read
    across the fabric by the kernel; raw getters holding nothing (absent
    chunks) go with either."""
    def dev(it):
        bg = it[0]
        st = getattr(bg, "store", None)
        if isinstance(st, DeviceStore):
            return device is None or _same_device(st.device, device)
        if isinstance(bg, _Raw):
            if bg.value is None:
                return True
            return isinstance(bg.value, DeviceRef) and (device is None or
                                                        _same_device(bg.value.arena.device, device))
        return False

    return all(dev(it) for it in batch) and any(
        not (isinstance(it[0], _Raw) and it[0].value is None) for it in batch)


@dataclass(frozen=True)
class HipCodecPipeline:
    """CodecPipeline whose codec compute runs in HIP kernels on MI355X."""

    codecs: tuple
    array_array_codecs: tuple
    array_bytes_codec: Any
    bytes_bytes_codecs: tuple
    batch_size: int = 1 << 30
    # load-address prediction for whole-row batches (planner.predict_rows);
    # ZARR_HIP_PREDICT=0 turns it off (measurements only)
    predict_loads: bool = field(default_factory=lambda: os.environ.get("ZARR_HIP_PREDICT", "1") != "0")
    # GPUs a read / write is split over (parallel.read_multi / write_multi):
    # () = one device (the out's, the store's or the current one).  Default
    # from zarr's config key "hip.devices" (env ZARR_HIP__DEVICES="0,1,...")
    devices: tuple = field(default_factory=lambda: _config_devices())
    # per-call plan cache for device-resident reads (read_sync): batch key ->
    # DecodeProgram; entries hold tables, never outs (retargeted per call)
    _read_cache: dict = field(default_factory=dict, compare=False, hash=False, repr=False)
    _aux: dict = field(default_factory=dict, compare=False, hash=False, repr=False)

    @classmethod
    def from_codecs(cls, codecs: Iterable, *, batch_size: int | None = None,
                    devices=None, warn: bool = True) -> "HipCodecPipeline":
        """warn=False: the package's own internal pipelines over an array's
        codecs (the writer's merge read) skip the advisory zarr already gave
        when the array was made."""
        codecs = tuple(codecs)
        cl = tuple(parse_codecs(codecs))
        if warn and any(isinstance(c, ShardingCodec) for c in cl) and len(cl) > 1:
            # codecs_from_list's advisory (codec_pipeline.py:859-883)
            warnings.warn("Combining a `sharding_indexed` codec disables partial reads and writes, which "
                          "may lead to inefficient performance.", UserWarning, stacklevel=2)
        aa, ab, bb = split_codecs(cl)
        p = cls(cl, aa, ab, bb, batch_size or (1 << 30))
        if devices is not None:
            p = replace(p, devices=_parse_devices(devices), _read_cache={}, _aux={})
        if any(is_v2_codec(c) for c in codecs):
            p._aux["v2"] = True  # the chunk spec's order decides the stored layout (evolve)
        return p

    @classmethod
    def from_array_metadata_and_store(cls, array_metadata, store) -> "HipCodecPipeline":
        """The hook create_codec_pipeline tries first (src/zarr/core/array.py:221-228,
        src/zarr/abc/codec.py:352-369): the v3 metadata's codecs evolved against
        its chunk spec (array.py:237-254).  v2 metadata and irregular chunk grids
        raise NotImplementedError, which sends zarr down its from_codecs path
        (and, for codecs off the GPU path, to a loud NotImplementedError there)."""
        codecs = getattr(array_metadata, "codecs", None)
        grid = getattr(array_metadata, "chunk_grid", None)
        chunk_shape = getattr(grid, "chunk_shape", None)
        if codecs is None or chunk_shape is None:
            raise NotImplementedError(
                "HipCodecPipeline.from_array_metadata_and_store needs v3 metadata on a regular grid")
        dtype = getattr(array_metadata, "data_type", None)
        if dtype is None:
            dtype = getattr(array_metadata, "dtype")
        spec = ArraySpec(tuple(chunk_shape), dtype, getattr(array_metadata, "fill_value", None))
        return cls.from_codecs(codecs).evolve_from_array_spec(spec)

    def evolve_from_array_spec(self, array_spec) -> "HipCodecPipeline":
        array_spec = coerce_spec(array_spec)
        codecs = self.codecs
        if self._aux.get("v2"):
            # zarr v2 (V2Codec): the raw chunk is the array in the spec's order
            # (_v2.py:66-68); F order is the v3 chain with a reversing transpose
            if array_spec.dtype.byteorder == ">":
                raise NotImplementedError("zarr v2 big-endian dtypes")
            if array_spec.order == "F" and array_spec.ndim > 1:
                codecs = (TransposeCodec(order=tuple(reversed(range(array_spec.ndim)))),) + codecs
        ev = evolve_codecs(codecs, array_spec)
        aa, ab, bb = split_codecs(ev)
        return type(self)(ev, aa, ab, bb, self.batch_size, self.predict_loads, self.devices)

    def __iter__(self):
        return iter(self.codecs)

    # ---------------------------------------------------------- host stage
    def _host_split(self):
        """None for an all-GPU chain, else (outer host stage, inner host stage of
        the sharding codec, the GPU pipeline for reads -- the chain without the
        outer stage, its sharding codec still naming the inner stage, which
        prepare_read runs per inner chunk -- and the GPU pipeline for writes,
        without either stage: hoststage.TranscodingByteSetter converts).
        Compression codecs stay on the host (hoststage.py)."""
        aux = self._aux
        if "split" not in aux:
            fixed, outer = split_host_tail(self.codecs)
            ab = self.array_bytes_codec
            inner = split_host_tail(ab.codecs)[1] if isinstance(ab, ShardingCodec) else ()
            if not outer and not inner:
                aux["split"] = None
            else:
                read_pipe = self._sub(fixed) if outer else None
                wfixed = tuple(replace(c, codecs=split_host_tail(c.codecs)[0]) if isinstance(c, ShardingCodec)
                               else c for c in fixed)
                aux["split"] = (outer, inner, read_pipe, self._sub(wfixed))
        return aux["split"]

    def _nested(self):
        """The outer ShardingCodec of a nested-sharding chain, else None."""
        aux = self._aux
        if "nested" not in aux:
            from . import nested

            aux["nested"] = nested.nested_split(self)
        return aux["nested"]

    def _sub(self, codecs) -> "HipCodecPipeline":
        aa, ab, bb = split_codecs(codecs)
        return type(self)(tuple(codecs), aa, ab, bb, self.batch_size, self.predict_loads, ())

    def _host_read_batch(self, batch: list, outer: tuple) -> list:
        """Items whose getters return the stored bytes -> items over the
        fixed-size bytes the outer host stage yields (decoded once per stored
        object, on the host-stage pool)."""
        from . import hoststage

        keys, firsts = {}, []
        for it in batch:
            bg = it[0]
            k = (id(getattr(bg, "store", None)), getattr(bg, "path", None)) if getattr(bg, "path", None) \
                is not None else ("obj", id(bg))
            if k not in keys:
                keys[k] = len(firsts)
                firsts.append(bg)
        spec = batch[0][1]

        def one(bg):
            raw = bg.get_sync(prototype=None) if hasattr(bg, "get_sync") else bg
            if raw is None:
                return None
            return hoststage.decode_tail(staging.staged_host(raw), outer, spec)

        dec = hoststage.map_host(one, firsts)
        out = []
        for it in batch:
            bg = it[0]
            k = (id(getattr(bg, "store", None)), getattr(bg, "path", None)) if getattr(bg, "path", None) \
                is not None else ("obj", id(bg))
            out.append((_Raw(dec[keys[k]]),) + tuple(it[1:]))
        return out

    def _inner_decoder(self, chain, spec):
        """The per-inner-chunk host stage of a sharded chain, as the staging
        hook (list of stored inner-chunk bytes -> fixed-size bytes)."""
        if not chain.inner_host:
            return None
        from . import hoststage

        tail = chain.inner_host
        ispec = chain.shard.inner_spec(spec)

        def dec(bufs):
            return hoststage.decode_many(list(bufs), tail, ispec)

        return dec

    @property
    def supports_partial_decode(self) -> bool:
        """pipeline_supports_partial_decode (codec_pipeline.py:143-166)."""
        return isinstance(self.array_bytes_codec, ShardingCodec) and not (
            self.array_array_codecs or self.bytes_bytes_codecs)

    @property
    def supports_partial_encode(self) -> bool:
        return self.supports_partial_decode

    def validate(self, *, shape, dtype=None, chunk_grid=None, chunk_shape=None) -> None:
        if chunk_shape is None and chunk_grid is not None and getattr(chunk_grid, "is_regular", True):
            chunk_shape = getattr(chunk_grid, "chunk_shape", None)  # (rectilinear grids: per edge)
        for c in self.codecs:
            c.validate(shape=shape, dtype=dtype, chunk_grid=chunk_grid, chunk_shape=chunk_shape)

    def compute_encoded_size(self, byte_length: int, array_spec=None) -> int:
        array_spec = None if array_spec is None else coerce_spec(array_spec)
        for c in self.codecs:
            byte_length = c.compute_encoded_size(byte_length, array_spec)
        return byte_length

    # ------------------------------------------------- transposes around sharding
    def _shard_space(self, batch: list, arr, drop_axes: tuple):
        """Transposes in front of a sharding codec (the codec then sees the
        permuted shard, chunk_utils.py:304-363): the same read / write expressed
        in that stored space -- selections, spec and the out / value tensor
        permuted (a strided view, no copy) -- for the pipeline of the sharding
        codec alone.  None when the chain has no such transposes."""
        if not self.array_array_codecs or not isinstance(self.array_bytes_codec, ShardingCodec):
            return None
        spec: ArraySpec = batch[0][1]
        perm = analyze_chain(self.codecs, spec).perm
        if perm == tuple(range(len(perm))):
            return None
        if drop_axes:
            raise NotImplementedError("drop_axes with transposes around sharding_indexed")
        torch = _torch()
        spec_s = replace(spec, shape=tuple(spec.shape[p] for p in perm))
        pipe = HipCodecPipeline.from_codecs((self.array_bytes_codec,), batch_size=self.batch_size)
        pipe = replace(pipe.evolve_from_array_spec(spec_s), predict_loads=self.predict_loads)
        is_int = [isinstance(c, (int, np.integer)) for c in batch[0][2]]
        kept = [d for d in range(len(perm)) if not is_int[d]]      # decoded dims present in out
        out_dim = {d: i for i, d in enumerate(kept)}
        order = [out_dim[perm[i]] for i in range(len(perm)) if not is_int[perm[i]]]
        batch_s = []
        for bg, sp, csel, osel, complete in batch:
            if [isinstance(c, (int, np.integer)) for c in csel] != is_int:
                raise NotImplementedError("mixed int selections in one batch")
            batch_s.append((bg, replace(sp, shape=spec_s.shape), tuple(csel[p] for p in perm),
                            tuple(osel[i] for i in order) if len(osel) == len(order) else osel, complete))
        if isinstance(arr, torch.Tensor) and arr.dim() == len(order):
            arr = arr.permute(order)
        elif isinstance(arr, np.ndarray) and arr.ndim == len(order):
            arr = arr.transpose(order)
        return pipe, batch_s, arr

    def _chain(self, spec: ArraySpec) -> ChainInfo:
        """analyze_chain of this pipeline's codecs for a chunk spec (memoised per
        shape and dtype: the per-call read path)."""
        key = (spec.shape, spec.dtype.str)
        cache = self._aux.setdefault("chains", {})
        c = cache.get(key)
        if c is None:
            c = analyze_chain(self.codecs, spec)
            if len(cache) < 64:
                cache[key] = c
        return c

    # ---------------------------------------------------------------- read
    def prepare_read(self, batch_info: Iterable, out, drop_axes: tuple = (),
                     item_out_extra=None, pooled: bool = False) -> DecodeProgram:
        """Plan a batch once: tables uploaded, launches ready.  `out` is a device
        tensor; item_out_extra (bytes per item) shifts each item's out position,
        so one launch can decode a batch into the slices of a stacked out."""
        torch = _torch()
        batch = normalize_batch(batch_info)
        if not batch:
            raise ValueError("empty batch")
        if not isinstance(out, torch.Tensor) or not out.is_cuda:
            raise TypeError("HipCodecPipeline.read needs a device-resident out (torch CUDA tensor)")
        groups = spec_groups(batch)
        if groups is not None:  # chunks of different specs (rectilinear grids): a program per spec
            progs = [self.prepare_read([batch[i] for i in idx], out, drop_axes,
                                       None if item_out_extra is None else np.asarray(item_out_extra)[idx],
                                       pooled) for idx in groups]
            return ProgramGroup(progs, groups, len(batch))
        ns = self._nested()
        if ns is not None:  # the inner pipeline's program over the touched inner shards
            from . import nested

            inner, items, _, _ = nested.read_batch(self, ns, batch)
            return inner.prepare_read(items, out, drop_axes, item_out_extra)
        hs = self._host_split()
        if hs is not None and hs[0]:
            return hs[2].prepare_read(self._host_read_batch(batch, hs[0]), out, drop_axes, item_out_extra)
        ss = self._shard_space(batch, out, drop_axes)
        if ss is not None:
            pipe, batch_s, out_s = ss
            return pipe.prepare_read(batch_s, out_s, drop_axes, item_out_extra)
        spec: ArraySpec = batch[0][1]
        device = out.device
        itemsize = out.element_size()
        if np.dtype(spec.dtype).itemsize != itemsize:
            raise TypeError("out dtype itemsize does not match the array dtype")
        chain: ChainInfo = self._chain(spec)
        resolved = None
        one = None if chain.inner_host else _one_device_store(batch, device)
        # host-resident bytes are packed and copied on the stager thread while
        # this thread plans; the launch waits for them (DecodeProgram.pending)
        # (a sharded chain whose inner chunks pass a host stage always reads
        # through the host: the touched inner chunks are decoded there first)
        if one is not None:  # one DeviceStore: its arena is the source
            arena = one[0].arena
            src, size, srcs, keep, pending = arena.buf, arena.top, one[1], [arena.buf], None
        elif chain.shard is not None and (chain.inner_host or not _device_resident(batch, device)):
            sh = chain.shard
            cps = sh.chunks_per_shard(spec.shape)
            src, size, item_missing, resolved, keep, pending = staging.gather_sharded_partial(
                batch, sh, cps, int(np.prod(cps)), sh.chunk_shape, spec, device, defer=True,
                inner_decode=self._inner_decoder(chain, spec))
            srcs = [(0, 0, bool(m)) for m in item_missing]
        else:
            src, size, srcs, keep, pending = staging.gather_sources(batch, device, defer=True)
        try:
            items = [(o, n, miss, it[2], it[3]) for (o, n, miss), it in zip(srcs, batch)]
            ostr = [int(s) * itemsize for s in out.stride()]
            with torch.cuda.device(device):
                t = plan_decode(chain, spec, items, ostr, out.data_ptr(), drop_axes, resolved, item_out_extra)
                # (k_decode_il resolves its own units: no prediction to build;
                # ZARR_HIP_IL_PREDICT=1 builds one for it too -- measurement arms)
                if self.predict_loads and t.rows and (IL_PREDICT or not (_kernel_flags(t.layout) & N.PK_IL)):
                    predict_rows(t, chain, spec, size)
                # fuse the shard-index CRC checks into the data launch
                # (zhip_decode_indexed: needs the CRC tables, i.e. an inner crc32c, and
                # the non-tiled kernel); else a second NO_WRITE launch
                fuse = (t.index_layout is not None and resolved is None and chain.inner.crc
                        and not t.tile)
                # inner chunks without a CRC (zarr's default sharding codecs):
                # leading index-check workgroups of the mapped pair decode
                # (k_decode_lead), whole-row layouts of <= 1 MiB chunks
                lead = (t.index_layout is not None and resolved is None and not chain.inner.crc
                        and not t.tile and t.fast and t.rows
                        and get_plan(t.layout).units_per_chunk <= 32)
                # (pooled: the per-call read hands the buffers back after a clean check)
                pooled = pooled and pending is None
                data = DecodeLaunch(t.layout, t.chunks, t.sels, src, size, out, t.fast, device, t.tile,
                                    t.index_chunks if (fuse or lead) else None, t.rows, t.predict, pooled)
                if lead and data.p_rowmap is None:  # the library declined the row map
                    data = DecodeLaunch(t.layout, t.chunks, t.sels, src, size, out, t.fast, device, t.tile,
                                        None, t.rows, t.predict)
                    lead = False
                fuse = fuse or lead
                index = None
                if t.index_layout is not None and not fuse:
                    index = DecodeLaunch(t.index_layout, t.index_chunks, np.zeros(1, SEL_DT), src, size,
                                         None, False, device)
        except BaseException:
            if pending is not None:
                pending.abort()  # the staging job must not outlive the buffers it fills
            raise
        return DecodeProgram(t, data, index, len(batch), chain.shard is not None,
                             np.array([s[2] for s in srcs], bool), keepalive=keep, pending=pending,
                             generations=((one[0].arena, one[0].arena.gen),) if one is not None
                             else _generations(batch))

    def read_sync(self, batch_info: Iterable, out, drop_axes: tuple = (),
                  max_workers: int = 1) -> tuple[GetResult, ...]:
        """FusedCodecPipeline.read_sync (codec_pipeline.py:1095-1172) on the GPU.

        `out` is a device tensor, this package's NDBuffer, any NDBuffer whose
        ``as_ndarray_like()`` is a ROCm tensor / DLPack capsule (decoded in
        place), or a host NDBuffer / numpy array: then the batch decodes into an
        HBM twin of `out` and the result is copied back (the regions no item
        selects are carried through unchanged)."""
        batch = normalize_batch(batch_info)
        if not batch:
            return ()
        groups = spec_groups(batch)
        if groups is not None:  # chunks of different specs (rectilinear grids)
            return self._read_groups(batch, groups, out, drop_axes)
        if len(self.devices) > 1:  # items split over several GPUs (parallel.read_multi)
            from . import parallel

            res = parallel.read_multi(self, batch, out, drop_axes)
            if res is not None:
                return res
        ns = self._nested()
        if ns is not None:  # nested sharding: outer level routed on the host (nested.py)
            from . import nested

            return nested.read_sync(self, ns, batch, out, drop_axes)
        hs = self._host_split()
        if hs is not None and hs[0]:  # the outer host stage first, then the GPU chain
            return hs[2].read_sync(self._host_read_batch(batch, hs[0]), out, drop_axes)
        dev_out, host_out = _resolve_out(out, batch, drop_axes)
        if host_out is None and READ_CACHE_SIZE and hs is None:
            key = _read_key(batch, dev_out, drop_axes)
            if key is not None:
                return self._read_cached(key, batch, dev_out, drop_axes)
        direct = host_out is not None and _pinned_host(host_out, dev_out)
        if host_out is not None and not drop_axes and not _device_resident(batch):
            groups = _slab_groups(batch, dev_out)
            if groups is not None:
                return self._read_slabs(batch, groups, dev_out, host_out, direct)
        prog = self.prepare_read(batch, dev_out, drop_axes)
        prog.launch()
        res = prog.results_fast()  # one 4-byte error word back (the statuses only on an error)
        if direct:
            _d2h(dev_out, host_out, 0, dev_out.numel() * dev_out.element_size())
            _torch().cuda.current_stream(dev_out.device).synchronize()
        elif host_out is not None:
            from .buffer import copy_to_host

            copy_to_host(dev_out, host_out)
        return res

    def _read_groups(self, batch, groups, out, drop_axes) -> tuple[GetResult, ...]:
        """read_sync of a batch whose items carry different chunk specs
        (rectilinear grids: zarr hands one spec per item, array.py:5469-5486):
        one plan and one launch per spec group into the same device out, whose
        regions the groups split between them, every group launched back to
        back on one stream, then ONE synchronisation for all their error and
        verdict words (ProgramGroup.results_fast); a host out is copied back
        once, after the last group.  Several devices keep one read per group."""
        dev_out, host_out = _resolve_out(out, batch, drop_axes)
        if len(self.devices) > 1:
            res: list = [None] * len(batch)
            for idx in groups:
                for i, r in zip(idx, self.read_sync([batch[i] for i in idx], dev_out, drop_axes)):
                    res[i] = r
        else:
            prog = self.prepare_read(batch, dev_out, drop_axes, pooled=True)
            prog.launch()
            res = prog.results_fast()
            if prog.clean:  # nothing raised or flagged: the pooled buffers are zero again
                prog.release()
        if host_out is not None:
            from .buffer import copy_to_host

            copy_to_host(dev_out, host_out)
        return tuple(res)

    def _read_cached(self, key, batch, dev_out, drop_axes) -> tuple[GetResult, ...]:
        """A device-resident read through the per-call plan cache: a repeated
        read of the same selection (same keys, selections, spec, out geometry,
        no write to the store since: the arena generation) skips planning and
        table uploads -- one launch, one 4-byte error word back.  The
        reference re-plans every read (codec_pipeline.py:1257-1319); its
        plans are Python objects, these are device tables."""
        cache = self._read_cache
        lock = self._aux.setdefault("cache_lock", threading.Lock())
        # checked out while in use: a concurrent read of the same key (another
        # thread, another stream) plans its own program instead of sharing
        # this one's status and arrival workspace
        with lock:
            prog = cache.pop(key, None)
        if prog is not None and (prog.stale() or not _same_arenas(prog, batch)):
            prog = None
        if prog is None:
            if not _device_resident(batch, dev_out.device):
                return self._read_uncached(batch, dev_out, drop_axes)
            prog = self.prepare_read(batch, dev_out, drop_axes)
        prog.retarget(dev_out)
        try:
            prog.launch()
            res = prog.results_fast()
        finally:
            prog.retarget(None)
        with lock:
            for k in [k for k in cache if not _key_alive(k)]:  # stores gone: free their programs
                del cache[k]
            while len(cache) >= READ_CACHE_SIZE:  # oldest first (insertion order = LRU)
                del cache[next(iter(cache))]
            cache[key] = prog
        return res

    def _read_uncached(self, batch, dev_out, drop_axes) -> tuple[GetResult, ...]:
        prog = self.prepare_read(batch, dev_out, drop_axes, pooled=True)
        prog.launch()
        res = prog.results_fast()
        if prog.clean:  # nothing raised or flagged: the buffers are zero again
            prog.release()
        return res

    def _read_slabs_one_plan(self, batch, groups, dev_out, host_out, direct: bool):
        """_read_slabs for unsharded chains: the batch is planned ONCE (in slab
        order), each slab's bytes are staged into its own buffer (every slab's
        staging job begun at once; the library runs them in order), and each
        slab is one range launch over the shared tables.  None when the chain is
        sharded (per-slab prepare_read then)."""
        torch = _torch()
        spec: ArraySpec = batch[0][1]
        if isinstance(self.array_bytes_codec, ShardingCodec):
            return None
        chain = analyze_chain(self.codecs, spec)
        dev = dev_out.device
        order = [i for _, _, idx in groups for i in idx]
        staged = []
        for _, _, idx in groups:
            src, size, srcs, keep, starter = staging.gather_sources([batch[i] for i in idx], dev, start=False)
            staged.append([src, size, srcs, keep, starter, None])
        itemsize = dev_out.element_size()
        if np.dtype(spec.dtype).itemsize != itemsize:
            raise TypeError("out dtype itemsize does not match the array dtype")

        def start(g):
            st = staged[g]
            if st[0] is None:  # host-sourced: begin its staging job now
                st[0], keep, st[5] = st[4]()
                st[3] = keep
        compute = torch.cuda.current_stream(dev)
        d2h = _d2h_stream(dev)
        nbytes = dev_out.numel() * dev_out.element_size()
        try:
            for g in range(len(groups)):  # the library packs and copies them in this order
                start(g)
            items = []
            for (_, _, idx), st in zip(groups, staged):
                items += [(o, n, miss, batch[i][2], batch[i][3]) for (o, n, miss), i in zip(st[2], idx)]
            ostr = [int(x) * itemsize for x in dev_out.stride()]
            with torch.cuda.device(dev):
                t = plan_decode(chain, spec, items, ostr, dev_out.data_ptr(), (), None, None)
                launch = DecodeLaunch(t.layout, t.chunks, t.sels, None, 0, dev_out, t.fast, dev, t.tile, None,
                                      t.rows, None)
            bounce = None if direct else torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            first = 0
            for g, ((a, b, idx), st) in enumerate(zip(groups, staged)):
                if st[5] is not None:
                    st[5].finish()  # the launch stream waits for this slab's copies
                launch.launch_range(first, len(idx), st[0], st[1])
                first += len(idx)
                _slab_back(compute, d2h, dev_out, host_out, bounce, a, b, direct)
            if not direct:
                _fill_gaps(d2h, dev_out, bounce, groups, nbytes)
            prog = DecodeProgram(t, launch, None, len(items), False,
                                 np.array([m for st in staged for (_, _, m) in st[2]], bool),
                                 keepalive=[st[0] for st in staged] + [k for st in staged for k in st[3]])
            res = prog.results()
        finally:
            # every begun slab job ends here, consumed or not (a failed slab
            # leaves the later ones running in the library's threads)
            for st in staged:
                if st[5] is not None:
                    st[5].abort()
            compute.synchronize()
            d2h.synchronize()
        if not direct:
            from .buffer import copy_to_host_from_pinned

            copy_to_host_from_pinned(bounce, host_out)
        out = [None] * len(batch)
        for j, i in enumerate(order):
            out[i] = res[j]
        return tuple(out)

    def _read_slabs(self, batch, groups, dev_out, host_out, direct: bool) -> tuple[GetResult, ...]:
        """A host-sourced read into a host out, pipelined over row slabs of
        out: slab k's chunks decode on the compute stream while slab k+1's
        bytes cross PCIe on the copy stream (staging), and slab k's rows go
        back on a D2H stream meanwhile -- H2D, decode and D2H overlap (PCIe
        is full duplex).  The result is what one whole-batch read gives:
        slabs are disjoint, every chunk lands in exactly one."""
        r = self._read_slabs_one_plan(batch, groups, dev_out, host_out, direct)
        if r is not None:
            return r
        torch = _torch()
        dev = dev_out.device
        compute = torch.cuda.current_stream(dev)
        d2h = _d2h_stream(dev)
        nbytes = dev_out.numel() * dev_out.element_size()
        bounce = None if direct else torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        done = []
        results: list = [None] * len(batch)
        try:
            for a, b, idx in groups:
                prog = self.prepare_read([batch[i] for i in idx], dev_out)
                prog.launch()
                _slab_back(compute, d2h, dev_out, host_out, bounce, a, b, direct)
                done.append((prog, idx))
            if not direct:
                _fill_gaps(d2h, dev_out, bounce, groups, nbytes)
            for prog, idx in done:
                for i, r in zip(idx, prog.results()):
                    results[i] = r
        finally:
            compute.synchronize()
            d2h.synchronize()
        if not direct:
            from .buffer import copy_to_host_from_pinned

            copy_to_host_from_pinned(bounce, host_out)
        return tuple(results)

    async def read(self, batch_info: Iterable, out, drop_axes: tuple = ()) -> tuple[GetResult, ...]:
        # one thread hop per batch, as FusedCodecPipeline.read (codec_pipeline.py:1287-1289)
        return await asyncio.to_thread(self.read_sync, list(batch_info), out, drop_axes)

    # --------------------------------------------------------------- write
    def write_sync(self, batch_info: Iterable, value, drop_axes: tuple = (),
                   max_workers: int = 1) -> None:
        """FusedCodecPipeline.write_sync (codec_pipeline.py:1174-1253) on the GPU.
        `value` is a device tensor, an NDBuffer (device or host), a numpy array
        or a scalar."""
        return self._write_sync(batch_info, value, drop_axes, partial_encode=True)

    def _write_sync(self, batch_info, value, drop_axes=(), partial_encode=True) -> None:
        from .writer import ChunkWriter

        torch = _torch()
        batch = normalize_batch(batch_info)
        if not batch:
            return
        value = _resolve_value(value)
        groups = spec_groups(batch)
        if groups is not None:  # chunks of different specs (rectilinear grids)
            if self._plain_unsharded():
                # every group's merge reads and encodes launched first, then ONE
                # readback of all their checks and non-empty flags, then the commits
                from .writer import ChunkWriter, PendingWrites

                from .writer import _value_tensor

                device = _write_device(batch, value)
                pend = PendingWrites()
                with torch.cuda.device(device):
                    if not isinstance(value, torch.Tensor) or not value.is_cuda:  # one upload for all groups
                        value = _value_tensor(value, batch[0][1].dtype, device)
                    for idx in groups:
                        sub = [batch[i] for i in idx]
                        spec = sub[0][1]
                        ChunkWriter(self.codecs, spec, spec.shape, device).write(
                            sub, value, self.codecs, drop_axes, partial_encode=partial_encode, pending=pend)
                    pend.finish(device)
                return
            for idx in groups:  # one write per spec
                self._write_sync([batch[i] for i in idx], value, drop_axes, partial_encode)
            return
        if len(self.devices) > 1:  # items split over several GPUs (parallel.write_multi)
            from . import parallel

            if parallel.write_multi(self, batch, value, drop_axes, partial_encode):
                return
        ns = self._nested()
        if ns is not None:  # nested sharding: outer level assembled on the host (nested.py)
            from . import nested

            return nested.write_sync(self, ns, batch, value, drop_axes)
        hs = self._host_split()
        if hs is not None and (hs[0] or not self.array_array_codecs):
            return self._host_write(batch, value, drop_axes, partial_encode, hs)
        ss = self._shard_space(batch, value, drop_axes)
        if ss is not None:
            pipe, batch_s, value_s = ss
            # with array->array codecs around it the sharding codec encodes whole
            # shards (ChunkTransform -> ShardingCodec._encode_sync, sharding.py:716-772),
            # not the partial-encode path (codec_pipeline.py:1212)
            return pipe._write_sync(batch_s, value_s, drop_axes, partial_encode=False)
        spec: ArraySpec = batch[0][1]
        device = _write_device(batch, value)
        with torch.cuda.device(device):
            w = ChunkWriter(self.codecs, spec, None or spec.shape, device)
            w.write(batch, value, self.codecs, drop_axes, partial_encode=partial_encode)

    def _plain_unsharded(self) -> bool:
        """One device, no sharding codec, no host stage, no nesting: the
        chain ChunkWriter encodes unsharded (the two-phase mixed-spec write)."""
        return (len(self.devices) <= 1 and self._nested() is None and self._host_split() is None
                and not isinstance(self.array_bytes_codec, ShardingCodec))

    def _host_write(self, batch, value, drop_axes, partial_encode, hs) -> None:
        """Writes through a host stage: the GPU encodes the fixed-size chain;
        each setter converts between that and the stored form on the host
        (hoststage.TranscodingByteSetter: the outer stage, and for a sharding
        codec with an inner stage the shard re-pack)."""
        from . import hoststage

        outer, inner, _, wpipe = hs
        spec: ArraySpec = batch[0][1]
        tr = None
        if inner:
            ab = self.array_bytes_codec
            tr = hoststage.ShardTranscoder(replace(ab, codecs=split_host_tail(ab.codecs)[0]), spec.shape,
                                           inner, ab.inner_spec(spec))
        wrapped = [(hoststage.TranscodingByteSetter(it[0], outer, tr, spec),) + tuple(it[1:]) for it in batch]
        # a bytes->bytes codec around a sharding codec hides the index: whole
        # shards are re-encoded (no partial encode, codec_pipeline.py:1212 with
        # pipeline_supports_partial_encode false)
        return wpipe._write_sync(wrapped, value, drop_axes, partial_encode and not outer)

    async def write(self, batch_info: Iterable, value, drop_axes: tuple = ()) -> None:
        await asyncio.to_thread(self.write_sync, list(batch_info), value, drop_axes)

    def decode_sync(self, chunk_bytes_and_specs: Iterable) -> list:
        """Decode standalone chunks (Buffer | None, ArraySpec) -> NDBuffer | None
        (abc/codec.py:417-434; BatchedCodecPipeline.decode_batch,
        codec_pipeline.py:679-706, decodes the whole list per call).  The
        chunks of one spec are ONE read: stacked along axis 0 of one device
        array (chunk i is rows [i s0, (i + 1) s0)), one plan, one launch; each
        result is an NDBuffer view of its rows (this package's device NDBuffer
        when the spec names no prototype)."""
        torch = _torch()
        from .buffer import torch_dtype

        items = list(chunk_bytes_and_specs)
        res: list = [None] * len(items)
        groups: dict = {}
        own: dict = {}  # each result is wrapped with its item's own spec (prototype included)
        for i, (raw, spec) in enumerate(items):
            if raw is not None:
                spec = own[i] = coerce_spec(spec)
                groups.setdefault(_spec_key(spec), (spec, []))[1].append(i)
        for spec, idx in groups.values():
            raws = []
            dev = None
            for i in idx:
                raw = items[i][0]
                raw = raw if isinstance(raw, (DeviceRef, bytes, bytearray, memoryview)) else \
                    staging.staged_bytes(raw)
                if dev is None:
                    dev = raw.arena.device if isinstance(raw, DeviceRef) else (
                        raw.device if isinstance(raw, torch.Tensor) else None)
                raws.append(raw)
            dev = dev or torch.device("cuda", torch.cuda.current_device())
            full = tuple(slice(0, s, 1) for s in spec.shape)
            if spec.ndim == 0:  # 0-d chunks cannot stack along an axis: one read each
                for i, raw in zip(idx, raws):
                    out = torch.empty((), dtype=torch_dtype(spec.dtype), device=dev)
                    self.read_sync([(_Raw(raw), spec, (), (), True)], out)
                    res[i] = _as_nd_buffer(out, own[i])
                continue
            s0 = spec.shape[0]
            out = torch.empty((len(idx) * s0,) + tuple(spec.shape[1:]), dtype=torch_dtype(spec.dtype), device=dev)
            batch = [(_Raw(raw), spec, full, (slice(j * s0, (j + 1) * s0),) + full[1:], True)
                     for j, raw in enumerate(raws)]
            self.read_sync(batch, out)
            for j, i in enumerate(idx):
                res[i] = _as_nd_buffer(out[j * s0:(j + 1) * s0], own[i])
        return res

    async def decode(self, chunk_bytes_and_specs: Iterable) -> list:
        return await asyncio.to_thread(self.decode_sync, list(chunk_bytes_and_specs))

    def encode_sync(self, chunk_arrays_and_specs: Iterable) -> list:
        """Encode standalone chunks (NDBuffer | None, ArraySpec) -> Buffer | None
        (abc/codec.py:436-453; BatchedCodecPipeline.encode_batch,
        codec_pipeline.py:716-745, encodes the whole list per call).  The
        chunks of one spec are ONE write: stacked along axis 0 of one device
        array, each chunk a complete chunk region of it, one GPU encode.  Empty
        chunks are None unless write_empty_chunks (chunk_utils.py:43-58); each
        result is a Buffer of the spec's prototype (this package's device
        Buffer when the spec names none: the encoded bytes stay in HBM)."""
        torch = _torch()
        from .writer import _value_tensor

        items = list(chunk_arrays_and_specs)
        res: list = [None] * len(items)
        groups: dict = {}
        own: dict = {}  # each result is wrapped with its item's own spec (prototype included)
        for i, (arr, spec) in enumerate(items):
            if arr is not None:
                spec = own[i] = coerce_spec(spec)
                groups.setdefault(_spec_key(spec), (spec, []))[1].append(i)
        for spec, idx in groups.values():
            full = tuple(slice(0, s, 1) for s in spec.shape)
            vals = [_resolve_value(items[i][0]) for i in idx]
            dev = next((v.device for v in vals if isinstance(v, torch.Tensor) and v.is_cuda), None) or \
                torch.device("cuda", torch.cuda.current_device())
            if spec.ndim == 0:
                for i, v in zip(idx, vals):
                    sink = _CollectSetter()
                    self._write_sync([(sink, spec, (), (), True)], v, partial_encode=False)
                    res[i] = None if sink.value is None else _as_buffer(sink.value, own[i])
                continue
            s0 = spec.shape[0]
            stacked = torch.cat([_value_tensor(v, spec.dtype, dev).reshape(spec.shape) for v in vals], 0)
            sinks = [_CollectSetter() for _ in idx]
            batch = [(sink, spec, full, (slice(j * s0, (j + 1) * s0),) + full[1:], True)
                     for j, sink in enumerate(sinks)]
            self._write_sync(batch, stacked, partial_encode=False)
            for i, sink in zip(idx, sinks):
                res[i] = None if sink.value is None else _as_buffer(sink.value, own[i])
        return res

    async def encode(self, chunk_arrays_and_specs: Iterable) -> list:
        return await asyncio.to_thread(self.encode_sync, list(chunk_arrays_and_specs))


def normalize_batch(batch_info: Iterable) -> list:
    """batch_info with every spec as this package's ArraySpec (zarr's ArraySpec
    carries a ZDType dtype, array_spec.py:137-186)."""
    items = batch_info if isinstance(batch_info, list) else list(batch_info)
    if all(type(it) is tuple and type(it[1]) is ArraySpec for it in items):
        return items  # already normalized (read_sync -> prepare_read)
    out = []
    seen: dict = {}  # one coerced spec per caller spec object (a regular grid shares one)
    for it in items:
        it = tuple(it)
        _check_basic(it[2])
        _check_basic(it[3])
        sp = seen.get(id(it[1]))
        if sp is None:
            sp = seen[id(it[1])] = coerce_spec(it[1])
        out.append((it[0], sp) + it[2:])
    return out


def _check_basic(selection) -> None:
    """The GPU path takes BasicIndexer selections (SURVEY §8 a16,
    indexing.py:571-621): per dim a slice or an integer.  zarr's orthogonal,
    coordinate and mask indexers (OrthogonalIndexer, CoordinateIndexer,
    MaskIndexer: indexing.py:902-1046, 1171-1400) hand integer arrays or
    boolean masks; those are refused here, by name, instead of failing
    somewhere in the planner."""
    for s in selection:
        if not isinstance(s, (slice, int, np.integer)):
            raise NotImplementedError(
                "only BasicIndexer selections (slices and integers) are on the GPU path; got "
                f"{type(s).__name__} (zarr's orthogonal / coordinate / mask selections are not)")


def _spec_key(spec: ArraySpec) -> tuple:
    return (spec.shape, spec.dtype.str, spec.fill_bytes(), spec.config)


def spec_groups(batch: list) -> list | None:
    """Item indices grouped by chunk spec (shape, dtype, fill, config), in
    first-seen order, or None when every item shares the first item's spec.
    zarr hands a batch one ArraySpec per chunk, and on a rectilinear grid
    their shapes differ (_get_chunk_spec, src/zarr/core/array.py:5373-5390,
    5469-5486): each group is planned and launched with its own spec."""
    s0 = batch[0][1]
    for it in batch:
        if it[1] is not s0:
            break
    else:
        return None
    k0 = _spec_key(s0)
    groups: dict = {}
    for i, it in enumerate(batch):
        sp = it[1]
        groups.setdefault(k0 if sp is s0 else _spec_key(sp), []).append(i)
    return None if len(groups) == 1 else list(groups.values())


def _selection_items(osel) -> int:
    n = 1
    for s in osel:
        if isinstance(s, slice):
            a, b, st = s.start or 0, s.stop, s.step or 1
            n *= max(0, -((a - b) // st))
    return n


def _resolve_out(out, batch, drop_axes):
    """(device tensor decoded into, host array to copy back into | None)."""
    torch = _torch()
    t = device_tensor(out)
    if t is not None:
        return t, None
    h = host_array(out)
    if h is None:
        raise TypeError(f"cannot decode into a {type(out).__name__}")
    if not h.flags.writeable:
        raise ValueError("out is read-only")
    from .buffer import torch_dtype

    dev = None
    for it in batch:
        st = getattr(it[0], "store", None)
        dev = getattr(st, "device", None)
        if dev is not None:
            break
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    twin = torch.empty(h.shape, dtype=torch_dtype(h.dtype), device=dev)
    covered = sum(_selection_items(it[3]) for it in batch)
    if covered < h.size:  # regions no chunk writes keep their host values
        twin.copy_(torch.from_numpy(np.ascontiguousarray(h).astype(h.dtype.newbyteorder("="))))
    return twin, h


_D2H_STREAMS: dict = {}


def _d2h_stream(device):
    torch = _torch()
    key = torch.device(device).index
    st = _D2H_STREAMS.get(key)
    if st is None:
        st = _D2H_STREAMS[key] = torch.cuda.Stream(device=device)
    return st


def _pinned_host(h: np.ndarray, dev_out) -> bool:
    """A C-contiguous host out in page-locked memory, byte-compatible with the
    device twin: the D2H DMA can write it directly."""
    return (h.flags.c_contiguous and h.dtype.isnative and h.nbytes == dev_out.numel() * dev_out.element_size()
            and h.nbytes > 0 and N.lib().zhip_host_pinned(h.ctypes.data) == 1)


def _d2h(dev_out, host_out: np.ndarray, a: int, b: int) -> None:
    """Bytes [a, b) of the (contiguous) device twin into the pinned host out,
    on the current stream."""
    torch = _torch()
    if b <= a:
        return
    flat = dev_out.reshape(-1).view(torch.uint8)
    dst = torch.from_numpy(host_out.reshape(-1).view(np.uint8))
    dst[a:b].copy_(flat[a:b], non_blocking=True)


def _slab_back(compute, d2h, dev_out, host_out, bounce, a: int, b: int, direct: bool) -> None:
    """Bytes [a, b) of a decoded slab back to the host on the D2H stream, after
    the slab's launch on `compute`: straight into a pinned host out, else into
    the pinned bounce image."""
    torch = _torch()
    ev = torch.cuda.Event()
    ev.record(compute)
    d2h.wait_event(ev)
    with torch.cuda.stream(d2h):
        if direct:
            _d2h(dev_out, host_out, a, b)
        else:
            flat = dev_out.reshape(-1).view(torch.uint8)
            bounce[a:b].copy_(flat[a:b], non_blocking=True)


def _fill_gaps(d2h, dev_out, bounce, groups, nbytes: int) -> None:
    """The bounce image is copied to the host out whole: the bytes no slab
    covers (rows before, between and after the groups) come from the device
    twin, which holds the out's own values there (_resolve_out prefilled it),
    so regions no item selects are carried through unchanged."""
    torch = _torch()
    flat = dev_out.reshape(-1).view(torch.uint8)
    at = 0
    with torch.cuda.stream(d2h):
        for a, b, _ in sorted(groups, key=lambda g: g[0]):
            if a > at:
                bounce[at:a].copy_(flat[at:a], non_blocking=True)
            at = max(at, b)
        if at < nbytes:
            bounce[at:nbytes].copy_(flat[at:nbytes], non_blocking=True)


def _slab_groups(batch: list, dev_out, min_bytes: int = 8 << 20, max_groups: int = 8):
    """Items grouped by disjoint row slabs of a C-contiguous out (out dim 0):
    [(byte_lo, byte_hi, item indices)], at least two groups of about
    max(min_bytes, out / max_groups) bytes each; None when the batch does not
    split that way (one chunk row, strided rows, small outs)."""
    if dev_out.dim() == 0 or not dev_out.is_contiguous() or dev_out.shape[0] == 0:
        return None
    row_bytes = dev_out[0].numel() * dev_out.element_size()
    total = row_bytes * dev_out.shape[0]
    if total < 2 * min_bytes:
        return None
    rows: dict = {}
    for i, it in enumerate(batch):
        osel = it[3]
        if not osel or not isinstance(osel[0], slice) or (osel[0].step or 1) != 1:
            return None
        rows.setdefault((osel[0].start or 0, osel[0].stop), []).append(i)
    keys = sorted(rows)
    if len(keys) < 2 or any(k1[0] < k0[1] for k0, k1 in zip(keys, keys[1:])):
        return None
    target = max(min_bytes, total // max_groups)
    groups, cur, lo = [], [], None
    for a, b in keys:
        lo = a if lo is None else lo
        cur += rows[(a, b)]
        if (b - lo) * row_bytes >= target:
            groups.append((lo * row_bytes, b * row_bytes, cur))
            cur, lo = [], None
    if cur:
        groups.append((lo * row_bytes, keys[-1][1] * row_bytes, cur))
    return groups if len(groups) >= 2 else None


def _write_device(batch, value):
    """The device a write encodes on: the value's, else the first item's
    store's, else the current one."""
    torch = _torch()
    if isinstance(value, torch.Tensor) and value.is_cuda:
        return value.device
    st = getattr(batch[0][0], "store", None)
    return getattr(st, "device", None) or torch.device("cuda", torch.cuda.current_device())


def _resolve_value(value):
    """A write's value as a device tensor or a host numpy array / scalar."""
    t = device_tensor(value)
    if t is not None:
        return t
    if isinstance(value, np.ndarray) or np.isscalar(value):
        return value
    h = host_array(value)
    return value if h is None else h


class _CollectSetter:
    """A ByteSetter that keeps what the writer stores (encode())."""

    value = None

    def get_sync(self, prototype=None, byte_range=None):
        return None

    def set_sync(self, value) -> None:
        self.value = value

    def delete_sync(self) -> None:
        self.value = None


def _as_nd_buffer(t, spec):
    from .buffer import NDBuffer, to_numpy

    proto = getattr(spec, "prototype", None)
    cls = getattr(proto, "nd_buffer", None)
    if cls is None or cls is NDBuffer:
        return NDBuffer(t)
    return cls.from_numpy_array(to_numpy(t, spec.dtype))


def _as_buffer(value, spec):
    from .buffer import Buffer
    from .interop import byte_payload

    proto = getattr(spec, "prototype", None)
    cls = getattr(proto, "buffer", None)
    if cls is None or cls is Buffer:
        return Buffer(byte_payload(value))
    return cls.from_bytes(byte_payload(value, host=True).tobytes())


@dataclass(frozen=True)
class _Raw:
    """Wrap raw bytes / DeviceRef as a ByteGetter."""

    value: Any

    def get_sync(self, prototype=None, byte_range=None):
        v = self.value
        if v is not None and not isinstance(v, (DeviceRef, bytes, bytearray, memoryview)):
            v = staging.staged_bytes(v)  # zarr Buffers, device tensors -> bytes / tensor
        if byte_range is None or v is None:
            return v
        n = v.numel() if hasattr(v, "numel") else len(v)
        a, b = _resolve_range(byte_range, n)
        if isinstance(v, DeviceRef):
            return DeviceRef(v.arena, v.offset + a, b - a)
        if isinstance(v, (bytes, bytearray, memoryview)):
            return memoryview(v)[a:b]
        return v[a:b]

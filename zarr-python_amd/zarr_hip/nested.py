"""Nested sharding: a ``sharding_indexed`` codec whose inner chain is itself a
single ``sharding_indexed`` codec (the reference runs the inner chain as a
nested pipeline over each inner chunk: ShardingCodec._get_inner_pipeline,
src/zarr/codecs/sharding.py:491-528; scenario ``nested-sharding``,
tests/test_codec_pipeline_suite.py:308-320).

The OUTER level is byte routing on the host: the outer index is read by one
suffix (or prefix) range request and its CRC checked with the host CRC-32C
(_decode_shard_index_sync, sharding.py:624-631), and every touched inner
shard becomes one batch item of the inner pipeline over its byte range of the
outer blob -- a DeviceRef into the same HBM arena for a DeviceStore, a range
request for host stores.  The INNER level (its index parse and CRC, sub-chunk
extraction, the inner chunks' CRC / byteswap, the scatter) is the ordinary
sharded GPU decode of the inner pipeline.

Writes run the inner pipeline's GPU encode against one collector per touched
inner shard (the old inner shard's bytes served for read-modify-write), then
assemble the outer blob: inner shards in the outer codec's subchunk write
order (untouched ones keep their bytes), the index re-encoded with its CRC
(_encode_sync / _encode_partial_sync, sharding.py:716-950); an outer shard
whose inner shards are all empty is deleted, as the reference deletes an
empty shard.
"""

from __future__ import annotations

from dataclasses import replace

import numpy as np

from .codecs import ShardingCodec
from .indexing import basic_projections, subchunk_order, to_chunk_selection
from .interop import byte_payload, is_own_store, request_classes, wrap_for_setter
from .store import DeviceRef, _resolve_range

MAX_U64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def nested_split(pipe):
    """(outer ShardingCodec, inner pipeline factory) when ``pipe``'s chain is
    nested sharding, else None.  Only the form the reference's suite uses is
    taken: the outer codec is the whole chain and its inner chain is exactly
    one sharding codec; anything around either raises NotImplementedError."""
    ab = pipe.array_bytes_codec
    if not isinstance(ab, ShardingCodec) or not any(isinstance(c, ShardingCodec) for c in ab.codecs):
        return None
    if pipe.array_array_codecs or pipe.bytes_bytes_codecs or len(ab.codecs) != 1:
        raise NotImplementedError("nested sharding with codecs around either sharding level")
    return ab


def _inner_pipeline(pipe, outer: ShardingCodec, spec):
    from .pipeline import HipCodecPipeline

    p = HipCodecPipeline.from_codecs(outer.codecs, batch_size=pipe.batch_size)
    return replace(p.evolve_from_array_spec(outer.inner_spec(spec)), predict_loads=pipe.predict_loads)


def _host_bytes(raw) -> np.ndarray | None:
    if raw is None:
        return None
    if isinstance(raw, DeviceRef):
        return np.frombuffer(raw.to_bytes(), np.uint8)
    return byte_payload(raw, host=True)


def _read_index(outer: ShardingCodec, bg, shard_shape):
    """The outer index of one outer shard (or None when the shard is absent),
    CRC-checked with the reference's message."""
    from .hoststage import ShardTranscoder

    tr = ShardTranscoder(outer, tuple(shard_shape), (), None)
    Range, Suffix = request_classes(getattr(bg, "store", None))
    req = Suffix(tr.index_size) if outer.index_location == "end" else Range(0, tr.index_size)
    raw = _host_bytes(bg.get_sync(prototype=None, byte_range=req))
    if raw is None:
        return None
    return tr.read_index(raw)


def _compose(osel: tuple, cell_osel: tuple) -> tuple:
    """A cell's out selection relative to its item's, as absolute slices."""
    if len(osel) != len(cell_osel):
        raise NotImplementedError("nested sharding with this out selection")
    out = []
    for o, c in zip(osel, cell_osel):
        if not isinstance(o, slice) or (o.step or 1) != 1:
            raise NotImplementedError("nested sharding with a strided out selection")
        a = o.start or 0
        out.append(slice(a + c.start, a + c.stop))
    return tuple(out)


def _cells(outer: ShardingCodec, spec, csel):
    """(linear cell id, cell chunk selection, cell out selection relative to
    the item, complete) for every inner shard a chunk selection touches."""
    cps = outer.chunks_per_shard(spec.shape)
    pr = basic_projections(tuple(csel), spec.shape, outer.chunk_shape)
    strides = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
    out = []
    for i in range(len(pr.coords)):
        cell = int((pr.coords[i] * strides).sum())
        c_csel, c_osel = to_chunk_selection(pr, i)
        out.append((cell, c_csel, c_osel, bool(pr.complete[i])))
    return cps, out


def read_batch(pipe, outer: ShardingCodec, batch: list):
    """The inner pipeline and its batch for a nested read, plus which of the
    new items belong to which outer item and which outer shards are absent."""
    from .pipeline import _Raw

    spec = batch[0][1]
    inner = _inner_pipeline(pipe, outer, spec)
    spec_in = outer.inner_spec(spec)
    items, owner, absent = [], [], []
    for k, (bg, sp, csel, osel, _complete) in enumerate(batch):
        cps, cells = _cells(outer, sp, csel)
        idx = _read_index(outer, bg, sp.shape)
        absent.append(idx is None)
        Range = request_classes(getattr(bg, "store", None))[0]
        for cell, c_csel, c_osel, c_complete in cells:
            getter = _Raw(None)
            if idx is not None:
                o, n = idx[cell]
                if not (o == MAX_U64 and n == MAX_U64):
                    getter = _Raw(bg.get_sync(prototype=None, byte_range=Range(int(o), int(o) + int(n))))
            items.append((getter, spec_in, c_csel, _compose(tuple(osel), c_osel), c_complete))
            owner.append(k)
    return inner, items, owner, absent


def read_sync(pipe, outer: ShardingCodec, batch: list, out, drop_axes: tuple = ()):
    """HipCodecPipeline.read_sync for a nested chain: one GetResult per outer
    item ("missing" when its outer shard is absent)."""
    from .spec import GetResult

    inner, items, owner, absent = read_batch(pipe, outer, batch)
    if items:
        inner.read_sync(items, out, drop_axes)
    return tuple(GetResult(status="missing" if a else "present") for a in absent)


class _Cell:
    """One inner shard of an outer shard being written: serves its old bytes
    (read-modify-write of a partial inner shard) and collects the new ones."""

    def __init__(self, old):
        self.old = old
        self.value = old
        self.written = False

    def get_sync(self, prototype=None, byte_range=None):
        v = self.old
        if v is None or byte_range is None:
            return None if v is None else bytes(v)
        a, b = _resolve_range(byte_range, len(v))
        return bytes(v[a:b])

    def set_sync(self, value) -> None:
        self.value = byte_payload(value, host=True).tobytes()
        self.written = True

    def delete_sync(self) -> None:
        self.value = None
        self.written = True


def write_sync(pipe, outer: ShardingCodec, batch: list, value, drop_axes: tuple = ()) -> None:
    """HipCodecPipeline.write_sync for a nested chain (one outer shard per item)."""
    from .hoststage import ShardTranscoder

    spec = batch[0][1]
    inner = _inner_pipeline(pipe, outer, spec)
    spec_in = outer.inner_spec(spec)
    plans = []
    items = []
    for bg, sp, csel, osel, complete in batch:
        cps, cells = _cells(outer, sp, csel)
        n = int(np.prod(cps))
        tr = ShardTranscoder(outer, sp.shape, (), sp)
        old = None if complete else _host_bytes(bg.get_sync(prototype=None))
        idx = tr.read_index(old) if old is not None else None
        parts = [None] * n
        if idx is not None:
            for c in range(n):
                o, m = idx[c]
                if not (o == MAX_U64 and m == MAX_U64):
                    parts[c] = old[int(o): int(o) + int(m)]
        touched = {}
        for cell, c_csel, c_osel, c_complete in cells:
            io = _Cell(parts[cell])
            touched[cell] = io
            items.append((io, spec_in, c_csel, _compose(tuple(osel), c_osel), c_complete))
        plans.append((bg, sp, cps, tr, parts, touched))
    if items:
        inner.write_sync(items, value, drop_axes)
    for bg, sp, cps, tr, parts, touched in plans:
        for cell, io in touched.items():
            parts[cell] = None if io.value is None else np.frombuffer(io.value, np.uint8)
        if all(p is None for p in parts):
            # deleted whether or not it was read first: a complete write (not
            # read) of nothing but empty inner shards replaces whatever the key
            # held (sharding.py:882-883 deletes unconditionally)
            bg.delete_sync()
            continue
        order = subchunk_order(tuple(cps), outer.subchunk_write_order)
        strides = np.array([int(np.prod(cps[d + 1:])) for d in range(len(cps))], np.int64)
        lin = (np.asarray(order, np.int64) * strides).sum(axis=1)
        idx = np.full((len(parts), 2), MAX_U64, np.uint64)
        at = tr.index_size if tr.at_start else 0
        body = []
        for c in lin:
            p = parts[int(c)]
            if p is None:
                continue
            idx[int(c)] = (at, p.size)
            at += p.size
            body.append(p.tobytes())
        ib = tr.write_index(idx)
        blob = ib + b"".join(body) if tr.at_start else b"".join(body) + ib
        st = getattr(bg, "store", None)
        bg.set_sync(blob if is_own_store(st) else wrap_for_setter(blob, sp.prototype))

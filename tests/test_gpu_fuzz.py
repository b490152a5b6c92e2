"""Seeded randomized parity: random shapes, chunk grids (edge chunks
included), dtypes, endianness, crc32c on/off, transposes, sharding (inner
shape, index location, transposes inside the shard), fill values and
selections (slices with steps, integers); each case (C or F order, write_empty_chunks on or off) writes the whole array,
overwrites two random selections (an array and a scalar), then reads the whole
array and two random selections.  The store's bytes are compared with the
oracle's after every write, and every read as raw bytes -- through whichever
kernels the planner picks for that geometry."""

import os

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import BE, CRC, LE, SHARD, T, _data

pytestmark = pytest.mark.gpu

DTYPES = ["float32", "int16", "uint8", "float64", "int32", "uint16"]


def _rand_sel(rng, shape):
    sel = []
    for n in shape:
        r = rng.random()
        if r < 0.2 and n > 0:
            sel.append(int(rng.integers(0, n)))
        elif r < 0.35:
            sel.append(slice(None))
        else:
            a = int(rng.integers(0, n))
            b = int(rng.integers(a + 1, n + 1))
            st = int(rng.choice([1, 1, 2, 3]))
            sel.append(slice(a, b, st))
    return tuple(sel)


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    nd = int(rng.choice([1, 2, 2, 3, 3, 3]))
    dtype = str(rng.choice(DTYPES))
    sharded = nd >= 2 and rng.random() < 0.4
    aligned = rng.random() < 0.3  # power-of-two geometries: the row / tile kernels' layouts
    if aligned:
        inner = tuple(int(rng.choice([8, 16, 32, 64])) for _ in range(nd))
        per = tuple(int(rng.integers(1, 3)) for _ in range(nd)) if sharded else (1,) * nd
        chunks = tuple(i * p for i, p in zip(inner, per))
        shape = tuple(int(c * rng.integers(1, 3) + (0 if rng.random() < 0.7 else rng.integers(1, c)))
                      for c in chunks)
        if int(np.prod(shape)) > (1 << 21):  # keep the oracle fast
            shape = tuple(min(s, 64) for s in shape)
    elif sharded:
        inner = tuple(int(rng.integers(2, 9)) for _ in range(nd))
        per = tuple(int(rng.integers(1, 4)) for _ in range(nd))
        chunks = tuple(i * p for i, p in zip(inner, per))
    else:
        chunks = tuple(int(rng.integers(1, 17)) for _ in range(nd))
    if not aligned:
        shape = tuple(int(rng.integers(1, 3 * c + 2)) for c in chunks)
    endian = BE if (rng.random() < 0.3 and np.dtype(dtype).itemsize > 1) else LE
    crc = rng.random() < 0.7
    chain = []
    if nd >= 2 and rng.random() < 0.4:
        chain.append(T(tuple(int(x) for x in rng.permutation(nd))))
    chain.append(endian)
    if crc:
        chain.append(CRC)
    if sharded:
        codecs = [SHARD(inner, chain, str(rng.choice(["end", "start"])))]
    else:
        codecs = chain
    fill = 0
    if np.dtype(dtype).kind == "f" and rng.random() < 0.3:
        fill = float("nan")
    elif rng.random() < 0.3:
        fill = 7
    return rng, shape, chunks, dtype, codecs, fill


# ZARR_HIP_FUZZ_FIRST / ZARR_HIP_FUZZ_SEEDS widen the sweep for stress runs
# (profiles/r03/fuzz_stress.log); the default suite runs seeds 0..159
_FIRST = int(os.environ.get("ZARR_HIP_FUZZ_FIRST", "0"))
_SEEDS = int(os.environ.get("ZARR_HIP_FUZZ_SEEDS", "160"))


@pytest.mark.parametrize("seed", range(_FIRST, _FIRST + _SEEDS))
def test_random_roundtrip(device, seed):
    import zarr_hip
    from zarr_hip.spec import ArrayConfig

    rng, shape, chunks, dtype, codecs, fill = _case(seed)
    wec = seed % 5 == 0
    order = "F" if seed % 3 == 0 else "C"
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs, write_empty_chunks=wec)
    host = {}
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs,
                                config=ArrayConfig(order=order, write_empty_chunks=wec))

    def check_store():
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store()
    # an array overwrite and a scalar overwrite of random selections
    sel = _rand_sel(rng, shape)
    want_shape = O.read(host, meta, sel).shape
    val = _data(want_shape, dtype, seed + 7) if want_shape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store()
    sel = _rand_sel(rng, shape)
    scalar = np.array(fill if rng.random() < 0.5 else 3, dtype=dtype)[()]
    O.write(host, meta, sel, scalar)
    arr[sel] = scalar
    check_store()
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


_LARGE = int(os.environ.get("ZARR_HIP_FUZZ_LARGE", "8"))


@pytest.mark.parametrize("seed", range(_LARGE))
def test_random_host_reads_large(device, tmp_path, seed):
    """Host-sourced reads big enough for the slab pipeline (>= 16 MiB outs):
    random chunking (sharded or not, transposed or not), host stores of the
    three kinds, random selections, compared with the oracle."""
    import zarr_hip

    rng = np.random.default_rng(5000 + seed)
    dtype = str(rng.choice(["float32", "int16", "float64"]))
    it = np.dtype(dtype).itemsize
    shape = (int(rng.choice([160, 256, 320])), 128, int(rng.choice([96, 128])) * 4 // it)
    chunks = tuple(int(rng.choice([16, 32, 64])) for _ in range(3))
    chain = ([T(tuple(int(x) for x in rng.permutation(3)))] if rng.random() < 0.5 else []) + [LE, CRC]
    codecs = [SHARD(chunks, chain)] if rng.random() < 0.4 else chain
    if codecs is not chain:
        chunks = tuple(2 * c for c in chunks)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), 0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), _data(shape, dtype, seed))
    kind = seed % 3
    if kind == 0:
        store = zarr_hip.MemoryStore(dict(host))
    elif kind == 1:
        store = zarr_hip.PinnedMemoryStore(dict(host))
    else:
        store = zarr_hip.LocalStore(str(tmp_path))
        for k, v in host.items():
            store.set_sync(k, v)
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, 0, codecs=codecs)
    for sel in [(Ellipsis,), _rand_sel(rng, shape), (slice(3, shape[0] - 5), slice(None), slice(1, None, 2))]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


def _il_case(seed):
    """Whole-row chunks of 256 KiB - 1 MiB (steps that tile into groups of eight
    workgroups): the k_decode_il / k_decode_ilw512 / k_encode_il geometry, with
    random dtype, endianness, sharding, fill, edge chunks and selections."""
    rng = np.random.default_rng(9000 + seed)
    dtype = str(rng.choice(["float32", "int16", "float64", "uint8", "int32"]))
    it = np.dtype(dtype).itemsize
    row = int(rng.choice([128, 256, 512]))          # bytes per innermost row
    c = row // it
    b = int(rng.choice([32, 64]))                   # rows per plane (a multiple of 4096 / row)
    chunk_bytes = int(rng.choice([256, 512, 1024])) << 10
    a = chunk_bytes // (b * row)
    chunks = (a, b, c)
    sharded = rng.random() < 0.4
    per = tuple(int(rng.integers(1, 3)) for _ in range(3)) if sharded else (1, 1, 1)
    outer = tuple(ch * p for ch, p in zip(chunks, per))
    shape = tuple(int(o * rng.integers(1, 3) - (0 if rng.random() < 0.6 else rng.integers(1, ch)))
                  for o, ch in zip(outer, chunks))
    while int(np.prod(shape)) * it > (24 << 20):  # keep the oracle fast
        shape = (max(1, shape[0] // 2),) + shape[1:]
    endian = BE if (it > 1 and rng.random() < 0.3) else LE
    chain = [endian, CRC]
    codecs = [SHARD(chunks, chain, str(rng.choice(["end", "start"])))] if sharded else chain
    fill = float("nan") if (np.dtype(dtype).kind == "f" and rng.random() < 0.3) else (7 if rng.random() < 0.3 else 0)
    return rng, shape, outer, dtype, codecs, fill


_IL_FIRST = int(os.environ.get("ZARR_HIP_FUZZ_IL_FIRST", "0"))


@pytest.mark.parametrize("seed", range(_IL_FIRST, _IL_FIRST + int(os.environ.get("ZARR_HIP_FUZZ_IL", "16"))))
def test_random_il_geometry(device, seed):
    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _il_case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    host = {}
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)

    def check_store():
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    # one chunk-sized region entirely fill (an elided chunk / inner chunk)
    data[tuple(slice(0, min(s, ch)) for s, ch in zip(shape, (chunks if not isinstance(codecs[0], dict)
                                                             or codecs[0]["name"] != "sharding_indexed"
                                                             else codecs[0]["configuration"]["chunk_shape"])))] = fill
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store()
    sel = _rand_sel(rng, shape)
    want_shape = O.read(host, meta, sel).shape
    val = _data(want_shape, dtype, seed + 7) if want_shape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store()
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


def _edges(rng, extent_unit, max_edges, max_mult):
    """A varying dimension: 1..max_edges edges, each a multiple of extent_unit."""
    return [int(extent_unit * rng.integers(1, max_mult + 1)) for _ in range(int(rng.integers(1, max_edges + 1)))]


def _rect_case(seed):
    """Rectilinear chunk grids (row n3): per dimension either a regular chunk or
    a list of edges (RLE-free, lengths repeating or not), the extent ending
    inside the last edge (an overhanging last chunk) or on it; optionally
    sharded (rectilinear shards whose edges are multiples of a regular inner
    chunk, sharding.py:567-593), with a random chain (transpose, endianness,
    crc32c) and fill."""
    rng = np.random.default_rng(13000 + seed)
    nd = int(rng.choice([1, 2, 2, 3]))
    dtype = str(rng.choice(DTYPES))
    sharded = rng.random() < 0.35
    inner = tuple(int(rng.integers(2, 7)) for _ in range(nd)) if sharded else None
    grid, shape = [], []
    for d in range(nd):
        unit = inner[d] if sharded else 1
        if rng.random() < 0.25:  # a regular dimension
            c = unit * int(rng.integers(1, 4 if sharded else 13))
            grid.append(c)
            shape.append(int(rng.integers(1, 3 * c + 1)))
        else:
            e = _edges(rng, unit, 4 if sharded else 6, 3 if sharded else 12)
            grid.append(e)
            lo = sum(e[:-1])
            shape.append(int(rng.integers(lo + 1, lo + e[-1] + 1)))
    endian = BE if (rng.random() < 0.3 and np.dtype(dtype).itemsize > 1) else LE
    chain = []
    if nd >= 2 and rng.random() < 0.3:
        chain.append(T(tuple(int(x) for x in rng.permutation(nd))))
    chain.append(endian)
    if rng.random() < 0.7:
        chain.append(CRC)
    fill = 0
    if np.dtype(dtype).kind == "f" and rng.random() < 0.3:
        fill = float("nan")
    elif rng.random() < 0.3:
        fill = 7
    return rng, tuple(shape), tuple(grid), inner, dtype, chain, fill


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_RECT_FIRST", "0")),
                                       int(os.environ.get("ZARR_HIP_FUZZ_RECT_FIRST", "0")) +
                                       int(os.environ.get("ZARR_HIP_FUZZ_RECT", "64"))))
def test_random_rectilinear_grid(device, seed):
    """Seeded rectilinear parity: whole write, an array and a scalar write into
    random selections, whole and random reads; store bytes after every write and
    every read compared with the oracle.  A read from a device store is one
    host synchronisation whatever the number of spec groups (pipeline.SYNCS)."""
    import zarr_hip
    from zarr_hip import pipeline as P

    rng, shape, grid, inner, dtype, chain, fill = _rect_case(seed)
    loc = str(rng.choice(["end", "start"]))
    codecs = chain if inner is None else [SHARD(inner, chain, loc)]
    meta = O.ArrayMeta(shape, grid, np.dtype(dtype), fill, codecs=codecs)
    host = {}
    dev = seed % 2 == 0
    store = zarr_hip.DeviceStore(device) if dev else zarr_hip.MemoryStore()
    if inner is None:
        arr = zarr_hip.Array.create(store, shape, grid, dtype, fill, codecs=chain)
    else:
        arr = zarr_hip.Array.create(store, shape, inner, dtype, fill, codecs=chain, shards=grid, index_location=loc)

    def check_store(what):
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (what, shape, grid, inner, codecs)
        for k in host:
            assert got[k] == host[k], (what, k, shape, grid, inner, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store("whole")
    sel = _rand_sel(rng, shape)
    want_shape = O.read(host, meta, sel).shape
    val = _data(want_shape, dtype, seed + 7) if want_shape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store(("array", sel))
    sel = _rand_sel(rng, shape)
    sval = _data((1,), dtype, seed + 11)[0]
    O.write(host, meta, sel, sval)
    arr[sel] = sval
    check_store(("scalar", sel))
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, grid, inner, codecs)
        want = np.ascontiguousarray(want)
        assert got.tobytes() == want.tobytes(), (sel, shape, grid, inner, codecs)
        if dev:
            arr.get(sel)  # plans and pooled buffers exist
            s0 = P.SYNCS[0]
            g = arr.get(sel)
            assert P.SYNCS[0] - s0 == 1, (sel, P.SYNCS[0] - s0, shape, grid)
            assert g.cpu().numpy().tobytes() == want.tobytes(), (sel, shape, grid, inner, codecs)


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_CORRUPT", "48"))))
def test_random_single_bit_corruption(device, seed):
    """One flipped bit in one stored object (an inner chunk, its CRC trailer,
    a shard index or its CRC), geometries of test_random_roundtrip (odd seeds:
    the il geometries): a whole read and a random read raise the oracle's
    exception with its exact message (crc32c_.py:46-49; sharding.py's index
    check), or -- for chains without a CRC -- return the same corrupted bytes;
    once the object is restored the same reads are exact again (nothing left
    dirty by the failed launch: pooled buffers, arrival words, cached plans)."""
    import zarr_hip

    if seed % 2:
        rng, shape, chunks, dtype, codecs, fill = _il_case(seed)
    else:
        rng, shape, chunks, dtype, codecs, fill = _case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 4 < 2 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    data = _data(shape, dtype, seed)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    if not host:
        pytest.skip("every chunk is fill: nothing stored")
    r = np.random.default_rng(7000 + seed)
    key = sorted(host)[int(r.integers(len(host)))]
    good = host[key]
    bad = bytearray(good)
    bad[int(r.integers(len(bad)))] ^= 1 << int(r.integers(8))
    sels = [(Ellipsis,), _rand_sel(rng, shape)]

    def outcome(fn):
        try:
            return ("ok", np.ascontiguousarray(fn()).tobytes())
        except Exception as e:  # noqa: BLE001 -- compared type and message
            return (type(e).__name__, str(e))

    for stored in (bytes(bad), good):
        host[key] = stored
        store.set_sync(key, stored)
        for sel in sels:
            want = outcome(lambda: O.read(host, meta, sel))
            got = outcome(lambda: arr[sel])
            assert got == want, (key, sel, shape, chunks, codecs, got[0], want[0])


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_CORRUPT_W", "48"))))
def test_random_corruption_then_write(device, seed):
    """One flipped bit in one stored object, then a random write (array or
    scalar) over it: a write that must merge with the corrupted bytes raises
    the oracle's exception and message (merge_and_encode_chunk decodes the
    existing chunk, chunk_utils.py:115-190; a partial shard write decodes only
    the touched, partially written inner chunks and carries the others' bytes
    over verbatim, sharding.py:774-885); any other write leaves a store
    byte-identical with the oracle's, corrupted object included, and the
    whole read afterwards has the oracle's outcome."""
    import zarr_hip

    if seed % 2:
        rng, shape, chunks, dtype, codecs, fill = _il_case(seed)
    else:
        rng, shape, chunks, dtype, codecs, fill = _case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 4 < 2 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    data = _data(shape, dtype, seed)
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    if not host:
        pytest.skip("every chunk is fill: nothing stored")
    r = np.random.default_rng(9100 + seed)
    key = sorted(host)[int(r.integers(len(host)))]
    bad = bytearray(host[key])
    bad[int(r.integers(len(bad)))] ^= 1 << int(r.integers(8))
    host[key] = bytes(bad)
    store.set_sync(key, bytes(bad))
    sel = _rand_sel(rng, shape)
    if r.random() < 0.5:
        val = np.array(3, dtype=dtype)[()]
    else:
        shp = O.read({}, meta, sel).shape
        val = _data(shp, dtype, seed + 5) if shp else _data((1,), dtype, seed + 5)[0]

    def outcome(fn):
        try:
            fn()
            return ("ok", "")
        except Exception as e:  # noqa: BLE001 -- compared type and message
            return (type(e).__name__, str(e))

    want = outcome(lambda: O.write(host, meta, sel, val))
    got = outcome(lambda: arr.__setitem__(sel, val))
    assert got == want, (key, sel, shape, chunks, codecs)
    if want[0] != "ok":
        return  # (which other chunks a failed write stored is not specified)
    stored = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert stored == host, (key, sel, shape, chunks, codecs)

    def read_outcome(fn):
        try:
            return ("ok", np.ascontiguousarray(fn()).tobytes())
        except Exception as e:  # noqa: BLE001
            return (type(e).__name__, str(e))

    assert read_outcome(lambda: arr[...]) == read_outcome(lambda: O.read(host, meta)), (key, sel)


def _with_gzip(rng, codecs):
    """A gzip (numcodecs.GZip restated by the oracle, mtime 0) inserted after the
    bytes codec -- before or after a crc32c -- of the chain, or of the shard's
    inner chain, or (sharded, 1 in 4) around the whole sharding codec."""
    gz = {"name": "gzip", "configuration": {"level": int(rng.integers(1, 10))}}
    if codecs and codecs[0].get("name") == "sharding_indexed":
        if rng.random() < 0.25:
            return codecs + [gz]
        inner = list(codecs[0]["configuration"]["codecs"])
        cfg = dict(codecs[0]["configuration"], codecs=_with_gzip(rng, inner))
        return [dict(codecs[0], configuration=cfg)]
    pos = next(i for i, c in enumerate(codecs) if c.get("name") == "bytes") + 1
    pos += int(rng.integers(0, len(codecs) - pos + 1))
    return codecs[:pos] + [gz] + codecs[pos:]


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_GZ", "24"))))
def test_random_compressed_roundtrip(device, seed):
    """test_random_roundtrip's geometries with a compressor in the chain: the
    host stage (gzip) beside the GPU chain, whole and random writes, whole and
    random reads, stores byte-identical with the oracle's."""
    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _case(seed)
    codecs = _with_gzip(rng, codecs)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}

    def check_store(what):
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (what, shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (what, k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store("whole")
    sel = _rand_sel(rng, shape)
    wshape = O.read(host, meta, sel).shape
    val = _data(wshape, dtype, seed + 7) if wshape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store(("array", sel))
    sel = (Ellipsis,) if rng.random() < 0.3 else _rand_sel(rng, shape)  # (whole: every chunk emptied)
    sval = np.array(fill if rng.random() < 0.5 else 3, dtype=dtype)[()]
    O.write(host, meta, sel, sval)
    arr[sel] = sval
    check_store(("scalar", sel))
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


def _nested_case(seed):
    """Nested sharding (suite:308-320 generalised): inner chunks c2, inner
    shards c1 = k1 * c2 whose codec is itself sharding_indexed, outer shards
    c0 = k0 * c1; random chain, index locations, dtype, fill, edge shards."""
    rng = np.random.default_rng(17000 + seed)
    nd = int(rng.choice([1, 2, 2, 3]))
    dtype = str(rng.choice(DTYPES))
    c2 = tuple(int(rng.integers(2, 6)) for _ in range(nd))
    c1 = tuple(c * int(rng.integers(1, 4)) for c in c2)
    c0 = tuple(c * int(rng.integers(1, 4)) for c in c1)
    shape = tuple(int(rng.integers(1, int(2.5 * c) + 2)) for c in c0)
    endian = BE if (rng.random() < 0.3 and np.dtype(dtype).itemsize > 1) else LE
    chain = [endian] + ([CRC] if rng.random() < 0.7 else [])
    inner_shard = SHARD(c2, chain, str(rng.choice(["end", "start"])))
    codecs = [SHARD(c1, [inner_shard], str(rng.choice(["end", "start"])))]
    fill = float("nan") if (np.dtype(dtype).kind == "f" and rng.random() < 0.3) else (7 if rng.random() < 0.3 else 0)
    return rng, shape, c0, dtype, codecs, fill


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_NESTED", "24"))))
def test_random_nested_sharding(device, seed):
    """Whole, array and scalar writes, whole and random reads of nested-sharded
    arrays (the outer level routed on the host, zarr_hip/nested.py; the inner
    shards on the GPU), stores and reads compared with the oracle."""
    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _nested_case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}

    def check_store(what):
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (what, shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (what, k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store("whole")
    sel = _rand_sel(rng, shape)
    wshape = O.read(host, meta, sel).shape
    val = _data(wshape, dtype, seed + 7) if wshape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store(("array", sel))
    sel = _rand_sel(rng, shape)
    sval = np.array(fill if rng.random() < 0.5 else 3, dtype=dtype)[()]
    O.write(host, meta, sel, sval)
    arr[sel] = sval
    check_store(("scalar", sel))
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


@pytest.mark.parametrize("kind", ["device", "memory"])
def test_nested_whole_fill_write_deletes_shards(kind, device):
    """A complete write of the fill value over nested-sharded data (found by
    test_random_nested_sharding): every outer shard is deleted, as the
    reference deletes an empty shard (sharding.py:882-883) -- it was left
    holding the old bytes, so a read returned the old data instead of fill."""
    import zarr_hip

    inner = SHARD((4, 4), [LE, CRC])
    codecs = [SHARD((8, 8), [inner])]
    store = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, (32, 16), (16, 16), "float32", 0.0, codecs=codecs)
    arr[...] = _data((32, 16), "float32", 1)
    assert len([k for k in store.to_dict() if not k.endswith("zarr.json")]) == 2
    arr[...] = np.float32(0.0)
    assert [k for k in store.to_dict() if not k.endswith("zarr.json")] == []
    assert not np.asarray(arr[...]).any()


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_STORES", "24"))))
def test_random_roundtrip_file_and_pinned_stores(device, tmp_path, seed):
    """test_random_roundtrip's geometries on the two other stores: LocalStore
    (files: pread into pinned windows, writes as files) and PinnedMemoryStore
    (page-locked arena: DMA straight from it, writes into it); whole, array and
    scalar writes, whole and random reads, stores and reads as the oracle's."""
    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.LocalStore(str(tmp_path)) if seed % 2 == 0 else zarr_hip.PinnedMemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}

    def check_store(what):
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (what, shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (what, k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store("whole")
    sel = _rand_sel(rng, shape)
    wshape = O.read(host, meta, sel).shape
    val = _data(wshape, dtype, seed + 7) if wshape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store(("array", sel))
    sel = (Ellipsis,) if rng.random() < 0.3 else _rand_sel(rng, shape)
    sval = np.array(fill if rng.random() < 0.5 else 3, dtype=dtype)[()]
    O.write(host, meta, sel, sval)
    arr[sel] = sval
    check_store(("scalar", sel))
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_VIEWS", "24"))))
def test_read_sync_into_views(device, seed):
    """read_sync straight into caller outs that are views: an offset window of
    a larger tensor, a stepped view, a transposed (F-order-like) view, and a
    numpy host view; the regions the batch selects equal the oracle's and every
    other byte of the underlying buffer is untouched -- or the read is refused
    with an error, never silently misplaced."""
    import torch

    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}
    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    sel = _rand_sel(rng, shape) if rng.random() < 0.6 else (Ellipsis,)
    batch, out_shape = arr.batch_info(sel)
    if not out_shape or not batch:
        pytest.skip("scalar selection")
    want = np.ascontiguousarray(O.read(host, meta, sel))
    tdt = torch.from_numpy(np.zeros(1, dtype)).dtype
    sentinel = np.array(5, dtype)
    nd = len(out_shape)
    kind = ["window", "stepped", "transposed", "host_window"][seed % 4]
    if kind == "transposed":
        base = torch.full(tuple(reversed(out_shape)), 5, dtype=tdt, device=device)
        view = base.permute(*reversed(range(nd)))
    else:
        big = tuple(n * (2 if (kind == "stepped" and d == 0) else 1) + 3 for d, n in enumerate(out_shape))
        base_np = np.full(big, sentinel)
        base = base_np if kind == "host_window" else torch.from_numpy(base_np).to(device)
        if kind == "stepped":
            view = base[tuple(slice(1, 1 + 2 * n, 2) if d == 0 else slice(2, 2 + n) for d, n in enumerate(out_shape))]
        else:
            view = base[tuple(slice(2, 2 + n) for n in out_shape)]
    try:
        arr.codec_pipeline.read_sync(batch, view)
    except (NotImplementedError, ValueError):
        return  # refused: acceptable, as long as nothing was written (checked below)
    else:
        got = view.cpu().numpy() if isinstance(view, torch.Tensor) else view
        assert np.ascontiguousarray(got).tobytes() == want.tobytes(), (kind, sel, shape, chunks, codecs)
    finally:
        b = base.cpu().numpy() if isinstance(base, torch.Tensor) else base
        mask = np.ones(b.shape, bool)
        if kind == "transposed":
            mask[...] = False
        elif kind == "stepped":
            mask[tuple(slice(1, 1 + 2 * n, 2) if d == 0 else slice(2, 2 + n) for d, n in enumerate(out_shape))] = False
        else:
            mask[tuple(slice(2, 2 + n) for n in out_shape)] = False
        outside = b[mask]
        assert (outside.view(np.uint8) == np.full(outside.shape, sentinel).view(np.uint8)).all(), (kind, sel)


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_VIEWS", "24"))))
def test_write_from_views(device, seed):
    """Array writes whose value is a view: an offset window, a stepped view
    and a transposed view of a larger array, as numpy (host) or torch (device)
    -- the encode reads the value through its strides; stores equal the
    oracle's (which is given the same values, contiguous)."""
    import torch

    import zarr_hip

    rng, shape, chunks, dtype, codecs, fill = _case(seed)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}
    for sel in [(Ellipsis,), _rand_sel(rng, shape)]:
        vshape = O.read(host, meta, sel).shape
        if not vshape:
            continue
        nd = len(vshape)
        src = _data((2 * max(vshape) + 3,) * nd, dtype, seed + len(host))  # every view fits
        kind = ["window", "stepped", "transposed"][int(rng.integers(0, 3))]
        if kind == "window":
            v = src[tuple(slice(1, 1 + n) for n in vshape)]
        elif kind == "stepped":
            v = src[tuple(slice(0, 2 * n, 2) for n in vshape)]
        else:
            t = np.ascontiguousarray(src[tuple(slice(0, n) for n in reversed(vshape))])
            v = t.transpose(tuple(reversed(range(nd))))
        assert v.shape == vshape
        val = torch.from_numpy(np.ascontiguousarray(src)).to(device) if rng.random() < 0.5 else None
        if val is not None:  # the same view taken of a device tensor
            if kind == "window":
                val = val[tuple(slice(1, 1 + n) for n in vshape)]
            elif kind == "stepped":
                val = val[tuple(slice(0, 2 * n, 2) for n in vshape)]
            else:
                val = torch.from_numpy(np.ascontiguousarray(t)).to(device).permute(*reversed(range(nd)))
        O.write(host, meta, sel, np.ascontiguousarray(v))
        arr[sel] = v if val is None else val
        got = {k: bytes(b) for k, b in store.to_dict().items() if not k.endswith("zarr.json")}
        assert got == host, (kind, sel, shape, chunks, codecs, val is not None)


@pytest.mark.parametrize("kind", ["device", "memory"])
@pytest.mark.parametrize("codecs_name", ["plain", "crc", "sharded"])
def test_empty_and_degenerate_shapes(kind, codecs_name, device):
    """Degenerate cases the reference handles: a zero-length dimension (no
    chunk exists; reads return empty arrays, writes store nothing), empty
    selections (arr[3:3], a step past the end), a one-element array, chunks
    larger than the array; stores and reads as the oracle's / numpy's."""
    import zarr_hip

    chains = {"plain": [LE], "crc": [LE, CRC]}
    for shape, chunks in [((0, 5), (4, 4)), ((1,), (1,)), ((3, 2), (8, 8)), ((5, 0, 2), (2, 2, 2))]:
        if codecs_name == "sharded":
            inner = tuple(max(1, c // 2) for c in chunks)
            codecs = [SHARD(inner, [LE, CRC])]
        else:
            codecs = chains[codecs_name]
        meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 1.5, codecs=codecs)
        store = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
        arr = zarr_hip.Array.create(store, shape, chunks, "float32", 1.5, codecs=codecs)
        host: dict = {}
        data = _data(shape, "float32", 3)
        O.write(host, meta, (Ellipsis,), data)
        arr[...] = data
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert got == host, (shape, chunks, codecs)
        full = O.read(host, meta)
        assert np.asarray(arr[...]).shape == full.shape
        assert np.asarray(arr[...]).tobytes() == full.tobytes()
        nd = len(shape)
        for sel in [(slice(3, 3),) + (slice(None),) * (nd - 1), (slice(shape[0] + 5, None),) + (slice(None),) * (nd - 1),
                    (slice(0, shape[0], 7),) + (slice(None),) * (nd - 1)]:
            want = full[sel]
            g = arr[sel]
            assert g.shape == want.shape, (shape, sel)
            assert np.ascontiguousarray(g).tobytes() == np.ascontiguousarray(want).tobytes(), (shape, sel)
            if want.size:
                continue
            arr[sel] = np.zeros(want.shape, np.float32)  # an empty write stores nothing
            O.write(host, meta, sel, np.zeros(want.shape, np.float32))
            got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
            assert got == host, (shape, sel)


@pytest.mark.parametrize("seed", range(int(os.environ.get("ZARR_HIP_FUZZ_TSHARD", "24"))))
def test_random_transpose_around_shards(device, seed):
    """A transpose OUTSIDE the sharding codec ([transpose, sharding_indexed]):
    the sharding codec is no longer alone, so the reference reads and writes
    whole shards (no partial decode / encode, codec_pipeline.py:143-166); whole,
    array and scalar writes and random reads against the oracle."""
    import zarr_hip

    rng = np.random.default_rng(23000 + seed)
    nd = int(rng.choice([2, 3]))
    dtype = str(rng.choice(DTYPES))
    inner = tuple(int(rng.integers(2, 7)) for _ in range(nd))
    chunks = tuple(i * int(rng.integers(1, 4)) for i in inner)
    perm = tuple(int(x) for x in rng.permutation(nd))
    # ShardingCodec.validate checks the inner chunk against the array's own
    # (untransposed) chunk edges (sharding.py:567-595), while the codec then
    # tiles the transposed shard: a valid inner edge divides both
    import math

    if seed % 2 == 0:
        inner_t = tuple(math.gcd(chunks[d], chunks[perm[d]]) for d in range(nd))
    else:
        inner_t = tuple(int(rng.integers(1, 7)) for _ in range(nd))
        bad = [d for d in range(nd) if chunks[d] % inner_t[d]]
        if bad:  # the reference refuses it at validation, and so must we, with its message
            d = bad[0]
            with pytest.raises(ValueError) as e:
                zarr_hip.Array.create(zarr_hip.MemoryStore(), tuple(2 * c for c in chunks), chunks, dtype, 0,
                                      codecs=[T(perm), SHARD(inner_t, [LE])])
            assert str(e.value) == (f"Chunk edge length {chunks[d]} in dimension {d} is not divisible by the "
                                    f"shard's inner chunk size {inner_t[d]}.")
            return
        if any(chunks[perm[d]] % inner_t[d] for d in range(nd)):
            pytest.skip("valid for ShardingCodec.validate, not a tiling of the transposed shard")
    shape = tuple(int(rng.integers(1, 3 * c + 2)) for c in chunks)
    endian = BE if (rng.random() < 0.3 and np.dtype(dtype).itemsize > 1) else LE
    codecs = [T(perm), SHARD(inner_t, [endian] + ([CRC] if rng.random() < 0.7 else []),
                             str(rng.choice(["end", "start"])))]
    fill = float("nan") if (np.dtype(dtype).kind == "f" and rng.random() < 0.3) else (7 if rng.random() < 0.3 else 0)
    meta = O.ArrayMeta(shape, chunks, np.dtype(dtype), fill, codecs=codecs)
    store = zarr_hip.DeviceStore(device) if seed % 2 == 0 else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs)
    host: dict = {}

    def check_store(what):
        got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host), (what, shape, chunks, codecs)
        for k in host:
            assert got[k] == host[k], (what, k, shape, chunks, codecs)

    data = _data(shape, dtype, seed)
    O.write(host, meta, (Ellipsis,), data)
    arr[...] = data
    check_store("whole")
    sel = _rand_sel(rng, shape)
    wshape = O.read(host, meta, sel).shape
    val = _data(wshape, dtype, seed + 7) if wshape else _data((1,), dtype, seed + 7)[0]
    O.write(host, meta, sel, val)
    arr[sel] = val
    check_store(("array", sel))
    sel = _rand_sel(rng, shape)
    sval = np.array(fill if rng.random() < 0.5 else 3, dtype=dtype)[()]
    O.write(host, meta, sel, sval)
    arr[sel] = sval
    check_store(("scalar", sel))
    for sel in [(Ellipsis,), _rand_sel(rng, shape), _rand_sel(rng, shape)]:
        want = O.read(host, meta, sel)
        got = arr[sel]
        assert got.shape == want.shape, (sel, shape, chunks, codecs)
        assert got.tobytes() == np.ascontiguousarray(want).tobytes(), (sel, shape, chunks, codecs)

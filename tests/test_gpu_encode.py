"""GPU parity of the write path: zarr_hip encode (HIP kernels through the C ABI)
must produce byte-identical stores to the CPU oracle (same keys, same bytes,
same elided empty chunks, same Morton-ordered shards) for the same sequence
of writes, and read back bit-exactly."""

import numpy as np
import pytest

from oracle import oracle as O
from conftest import set_tuning

pytestmark = pytest.mark.gpu

LE = {"name": "bytes", "configuration": {"endian": "little"}}
BE = {"name": "bytes", "configuration": {"endian": "big"}}
CRC = {"name": "crc32c"}


def T(order):
    return {"name": "transpose", "configuration": {"order": list(order)}}


def SHARD(inner_shape, codecs, loc="end", index=(LE, CRC)):
    return {"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(inner_shape), "codecs": list(codecs), "index_codecs": list(index),
        "index_location": loc}}


def _data(shape, dtype, seed=0):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        a = rng.standard_normal(shape).astype(dt)
        flat = a.reshape(-1)
        if flat.size > 8:
            flat[3] = -0.0
            flat[5] = np.nan
        return a
    info = np.iinfo(dt)
    return rng.integers(info.min, info.max, size=shape, dtype=dt, endpoint=True)


def _stores_equal(dev_store, host):
    got = {k: v for k, v in dev_store.to_dict().items() if not k.endswith("zarr.json")}
    assert sorted(got) == sorted(host), (sorted(set(got) ^ set(host)))[:10]
    for k in host:
        assert got[k] == host[k], f"bytes differ for {k}"


def _run(device, shape, chunks, dtype, codecs, fill, writes, write_empty=False, host_store=False):
    import zarr_hip
    from zarr_hip.spec import ArrayConfig

    meta = O.ArrayMeta(tuple(shape), tuple(chunks), np.dtype(dtype), fill, codecs=codecs,
                       write_empty_chunks=write_empty)
    host = {}
    store = zarr_hip.MemoryStore() if host_store else zarr_hip.DeviceStore(device)
    arr = zarr_hip.Array.create(store, shape, chunks, dtype, fill, codecs=codecs,
                                config=ArrayConfig(write_empty_chunks=write_empty))
    for sel, val in writes:
        O.write(host, meta, sel, val)
        arr[sel] = val
    if host_store:
        got = {k: v for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
        assert sorted(got) == sorted(host)
        for k in host:
            assert got[k] == host[k], k
    else:
        _stores_equal(store, host)
    full = O.read(host, meta)
    assert arr[...].tobytes() == full.tobytes()
    return arr, host


@pytest.mark.parametrize("dtype", ["float32", "int16", "uint8", "float64", "int32"])
def test_full_write_bytes_crc(device, dtype):
    _run(device, (40, 33, 20), (16, 16, 8), dtype, [LE, CRC], 0,
         [((Ellipsis,), _data((40, 33, 20), dtype))])


@pytest.mark.parametrize("dtype", ["float32", "int16", "float64"])
def test_big_endian_write(device, dtype):
    _run(device, (21, 34), (8, 16), dtype, [BE, CRC], 0, [((Ellipsis,), _data((21, 34), dtype))])


@pytest.mark.parametrize("order", [(2, 1, 0), (1, 2, 0), (0, 2, 1)])
def test_transpose_write(device, order):
    _run(device, (10, 20, 30), (5, 10, 15), "float32", [T(order), LE, CRC], np.nan,
         [((Ellipsis,), _data((10, 20, 30), "float32"))])


def test_empty_chunk_elision_and_fill_rules(device):
    d = _data((32, 32), "float32")
    d[0:8, 0:8] = 0.0          # == fill 0.0 -> elided
    d[8:16, 0:8] = -0.0        # -0.0 != 0.0 bitwise -> kept
    _run(device, (32, 32), (8, 8), "float32", [LE, CRC], 0.0, [((Ellipsis,), d)])
    e = _data((32, 32), "float32")
    e[0:8, 8:16] = np.nan      # NaN fill: any NaN equals -> elided
    e[16:24, 16:24] = np.float32(np.nan) * -1
    _run(device, (32, 32), (8, 8), "float32", [LE, CRC], np.nan, [((Ellipsis,), e)])


def test_write_empty_chunks_true(device):
    d = np.zeros((16, 16), "int16")
    _run(device, (16, 16), (8, 8), "int16", [LE, CRC], 0, [((Ellipsis,), d)], write_empty=True)


def test_partial_writes_sequence(device):
    shape, chunks = (37, 29), (8, 10)
    w = [((Ellipsis,), _data(shape, "float32", 1)),
         ((slice(3, 17), slice(None, None, 3)), _data((14, 10), "float32", 2)),
         ((5, slice(2, 30, 7)), _data((4,), "float32", 3)),
         ((slice(30, 37), slice(20, 29)), 0.0),
         ((slice(0, 8), slice(0, 10)), 0.0)]
    _run(device, shape, chunks, "float32", [LE, CRC], 0.0, w)


def test_scalar_and_fresh_partial(device):
    _run(device, (20, 20), (8, 8), "int32", [LE, CRC], 7,
         [((slice(2, 11), slice(5, 19)), 3), ((slice(0, 4), 0), np.array([1, 2, 3, 4], "int32"))])


def test_host_store_write(device):
    _run(device, (24, 24), (8, 8), "int16", [LE, CRC], 0,
         [((Ellipsis,), _data((24, 24), "int16"))], host_store=True)


@pytest.mark.parametrize("loc", ["end", "start"])
@pytest.mark.parametrize("inner", [[LE, CRC], [LE], [T((1, 0, 2)), LE, CRC]])
def test_sharded_write(device, loc, inner):
    _run(device, (32, 32, 32), (16, 16, 16), "float32", [SHARD((8, 8, 8), inner, loc)], 0.0,
         [((Ellipsis,), _data((32, 32, 32), "float32"))])


def test_sharded_elision_partial_and_delete(device):
    shape = (16, 24)
    codecs = [SHARD((4, 4), [LE, CRC])]
    d = _data(shape, "int16")
    d[0:4, 4:8] = -1
    d[8:16, 16:24] = -1
    w = [((Ellipsis,), d),
         ((slice(3, 13), slice(2, 23, 3)), _data((10, 7), "int16", 5)),
         ((slice(8, 16), slice(16, 24)), -1)]
    _run(device, shape, (8, 8), "int16", codecs, -1, w)


def test_sharded_edge_and_nonsquare(device):
    # non-square chunks_per_shard -> Morton vs lexicographic layouts differ
    _run(device, (20, 14), (6, 4), "int32", [SHARD((2, 2), [LE])], -1,
         [((Ellipsis,), _data((20, 14), "int32"))])


def test_roundtrip_c2_like(device):
    _run(device, (128, 128, 128), (64, 64, 64), "float32", [LE, CRC], 0.0,
         [((Ellipsis,), _data((128, 128, 128), "float32"))])


def test_sharded_c4_like(device):
    _run(device, (128, 128, 128), (64, 64, 64), "float32", [SHARD((16, 16, 16), [LE, CRC])], 0.0,
         [((Ellipsis,), _data((128, 128, 128), "float32"))])


# ---- k_encode_pair regular pairing (even units per chunk): non-empty flags and
#      trailers written by the last arrival of each chunk

@pytest.mark.parametrize("codecs", [[LE, CRC], [LE], [BE, CRC]])
@pytest.mark.parametrize("fill", [0.0, np.nan])
def test_encode_pair_elision_and_merges(device, codecs, fill):
    shape, chunks = (32, 64, 128), (8, 64, 64)  # 128 KiB chunks: 4 units each
    d = _data(shape, "float32")
    d[0:8, :, 0:64] = fill        # one chunk entirely fill -> elided
    d[16:24, :, 64:128] = fill    # another
    d[24, 3, 70] = -0.0 if fill == 0.0 else d[24, 3, 70]   # bitwise != fill: that chunk is kept
    w = [((Ellipsis,), d),
         ((slice(8, 16), slice(None), slice(64, 128)), fill),             # a full chunk back to fill
         ((slice(3, 29), slice(5, 60), slice(10, 100)), _data((26, 55, 90), "float32", 3))]
    _run(device, shape, chunks, "float32", codecs, fill, w)
    _run(device, shape, chunks, "float32", codecs, fill, w[:2], write_empty=True)


def test_encode_pair_sharded_empty_inner(device):
    shape = (32, 64, 64)
    codecs = [SHARD((8, 64, 64), [LE, CRC])]   # 128 KiB inner chunks
    d = _data(shape, "float32")
    d[8:16] = 0.0
    d[24:32] = 0.0
    _run(device, shape, (16, 64, 64), "float32", codecs, 0.0,
         [((Ellipsis,), d), ((slice(0, 8),), 0.0), ((slice(2, 30, 3), slice(1, 63)), 5.0)])


# ---- k_encode_il: chunks of 8 k units (>= 256 KiB), one unit per workgroup,
#      steps interleaved in groups of eight; the last arrival of each chunk
#      writes trailer, status and the non-empty flag (ORed by non-fill waves)

IL_ENC_CASES = [
    ((64, 64, 128), (32, 64, 32), "float32", [LE, CRC], 0.0),     # 256 KiB chunks: one group of eight
    ((64, 64, 128), (64, 64, 64), "float32", [BE, CRC], np.nan),  # 1 MiB: the headline's chunk
    ((64, 128, 64), (64, 64, 32), "int16", [LE, CRC], 0),
    ((32, 64, 64), (32, 32, 32), "float64", [LE, CRC], 0.0),
]


@pytest.mark.parametrize("case", range(len(IL_ENC_CASES)))
def test_encode_il(device, case):
    from zarr_hip import _native as N

    shape, chunks, dtype, codecs, fill = IL_ENC_CASES[case]
    d = _data(shape, dtype)
    c0 = tuple(slice(0, c) for c in chunks)
    d[c0] = fill                                   # one chunk entirely fill: elided
    c1 = (slice(0, chunks[0]), slice(0, chunks[1]), slice(chunks[2], 2 * chunks[2]))
    d[c1] = fill                                   # another: fill except one element
    if np.issubdtype(np.dtype(dtype), np.floating) and not np.isnan(fill):
        d[chunks[0] - 1, chunks[1] - 1, 2 * chunks[2] - 1] = -0.0   # bitwise != fill: kept
    else:
        d[chunks[0] - 1, chunks[1] - 1, 2 * chunks[2] - 1] = 1
    part = (slice(3, shape[0] - 5), slice(7, shape[1]), slice(1, shape[2] - 9))
    psh = tuple(s.stop - s.start for s in part)
    w = [((Ellipsis,), d),
         (part, _data(psh, dtype, 3)),                                  # merges into every chunk
         ((slice(0, chunks[0]), slice(0, chunks[1]), slice(shape[2] - chunks[2], shape[2])), fill)]  # back to fill
    arr, _ = _run(device, shape, chunks, dtype, codecs, fill, w)
    arr[...] = d
    assert N.lib().zhip_last_kernel().decode() == "k_encode_il"
    _run(device, shape, chunks, dtype, codecs, fill, w[:1], write_empty=True)


@pytest.mark.tuning
@pytest.mark.parametrize("case", [0, 1])
def test_encode_il_affine_arm(device, case):
    """Tuning arm 46: k_encode_il takes whole-chunk writes' destinations from
    the plan's affine form of the row map (ZHIP_DF_WHOLE) instead of the map:
    stores byte-identical with the oracle, partial writes (the map) between."""
    from zarr_hip import _native as N

    shape, chunks, dtype, codecs, fill = IL_ENC_CASES[case]
    d = _data(shape, dtype)
    part = (slice(3, shape[0] - 5), slice(7, shape[1]), slice(1, shape[2] - 9))
    psh = tuple(s.stop - s.start for s in part)
    set_tuning(6, 46)
    try:
        arr, _ = _run(device, shape, chunks, dtype, codecs, fill,
                      [((Ellipsis,), d), (part, _data(psh, dtype, 3)), ((Ellipsis,), d)])
        arr[...] = d
        assert N.lib().zhip_last_kernel().decode() == "k_encode_il"
    finally:
        set_tuning(6, 0)


def test_encode_il_sharded(device):
    from zarr_hip import _native as N

    shape = (64, 64, 128)
    codecs = [SHARD((32, 64, 32), [LE, CRC])]       # 256 KiB inner chunks
    d = _data(shape, "float32")
    d[0:32, :, 32:64] = 0.0
    arr, _ = _run(device, shape, (64, 64, 64), "float32", codecs, 0.0,
                  [((Ellipsis,), d), ((slice(5, 60), slice(2, 63), slice(9, 100)), 2.5), ((slice(32, 64),), 0.0)])
    arr[...] = d
    assert N.lib().zhip_last_kernel().decode() == "k_encode_il"


# ---- k_encode_quad: chunks of <= 16 KiB, four per workgroup (trailer, status
#      and non-empty flag written by the workgroup that owns the chunk);
#      ZHIP_TUNE_ARM 11 runs k_encode_pair on the same writes

QUAD_CASES = [
    ((256, 256), (64, 64), "int32", [LE, CRC], 0),                    # the reference example's inner chunk
    ((48, 32, 64), (3, 16, 64), "float32", [LE, CRC], np.nan),        # 12 KiB: an empty head step
    ((16, 64, 32), (4, 16, 32), "float64", [BE, CRC], 0.0),
    ((96, 128), (16, 128), "int16", [BE], 0),                         # 4 KiB, 6 chunks: a partial quad
    ((256, 256), (128, 128), "int32", [SHARD((64, 64), [LE])], 0),     # zarr's default sharding codecs
]


@pytest.mark.tuning
@pytest.mark.parametrize("arm", [0, 11])
@pytest.mark.parametrize("shape,chunks,dtype,codecs,fill", QUAD_CASES)
def test_encode_quad_small_chunks(device, arm, shape, chunks, dtype, codecs, fill):
    from zarr_hip import _native as N

    d = _data(shape, dtype)
    d[tuple(slice(0, c) for c in chunks)] = fill   # first chunk all fill -> elided
    sub = tuple(slice(1, s - 2) for s in shape[:-1]) + (slice(None),)
    w = [((Ellipsis,), d),
         (sub, _data(tuple(s - 3 for s in shape[:-1]) + (shape[-1],), dtype, 4)),   # merges with fill
         (tuple(slice(c, 2 * c) for c in chunks), fill)]                          # a chunk back to fill
    set_tuning(6, arm)
    try:
        _run(device, shape, chunks, dtype, codecs, fill, w)
    finally:
        set_tuning(6, 0)


# ---- k_encode_tile4: transposed chunks with full 64-row x 256-byte tiles

ENC_TILE4_CASES = [
    ("float32", LE, (64, 64, 64), (128, 128, 64)),
    ("float64", BE, (32, 16, 64), (64, 48, 128)),
    ("int16", LE, (128, 8, 64), (256, 16, 64)),
    ("uint8", LE, (256, 8, 64), (256, 24, 128)),
]


@pytest.mark.parametrize("dtype,endian,chunks,shape", ENC_TILE4_CASES)
def test_encode_tile4(device, dtype, endian, chunks, shape):
    from zarr_hip import _native as N
    from zarr_hip.planner import _make_layout

    codecs = [T((2, 1, 0)), endian, CRC]
    d = _data(shape, dtype)
    fill = 0
    sl = tuple(slice(0, c) for c in chunks)  # one chunk entirely fill -> elided
    d[sl] = fill
    arr, _ = _run(device, shape, chunks, dtype, codecs, fill, [((Ellipsis,), d)])
    arr[...] = d  # (two tiles per workgroup: the production form for CRC layouts)
    assert N.lib().zhip_last_kernel() == b"k_encode_tile2"
    # the layout qualifies for the four-tile encode
    st = [chunks[p] for p in (2, 1, 0)]
    it = np.dtype(dtype).itemsize
    L = _make_layout(st, it, [it, shape[2] * it * 999, shape[2] * shape[1] * it], 0, b"\0")
    assert N.Plan(L, upload=False).kernel_flags & N.PK_TILE4_ENCODE


@pytest.mark.tuning
@pytest.mark.parametrize("dtype,endian,chunks,shape", ENC_TILE4_CASES)
def test_encode_tile4_four_tile_form(device, dtype, endian, chunks, shape):
    """k_encode_tile4's four-tile form (ZHIP_TUNE_ARM 38) writes the same
    bytes: elided fill chunk, partial writes merged."""
    from zarr_hip import _native as N

    codecs = [T((2, 1, 0)), endian, CRC]
    d = _data(shape, dtype)
    d[tuple(slice(0, c) for c in chunks)] = 0
    set_tuning(6, 38)
    try:
        arr, _ = _run(device, shape, chunks, dtype, codecs, 0,
                      [((Ellipsis,), d), ((slice(1, shape[0] - 1), slice(2, shape[1]), slice(0, 33)), 5)])
        arr[...] = d
        assert N.lib().zhip_last_kernel() == b"k_encode_tile4"
    finally:
        set_tuning(6, 0)


@pytest.mark.tuning
@pytest.mark.parametrize("order", [(2, 1, 0), (1, 2, 0)])
@pytest.mark.parametrize("dtype,endian", [("float32", LE), ("int16", BE)])
def test_encode_tileg_four_tile_form(device, order, dtype, endian):
    """k_encode_tileg (production: four tiles per workgroup) and its two-tile
    form (ZHIP_TUNE_ARM 36) write byte-identical stores (partial tiles, a
    fill chunk)."""
    from zarr_hip import _native as N

    shape, chunks = (96, 160, 160), (96, 80, 80)
    codecs = [T(order), endian, CRC]
    d = _data(shape, dtype)
    d[0:96, 0:80, 0:80] = 0
    for arm, kname in ((0, b"k_encode_tileg"), (36, b"k_encode_tileg2"), (47, b"k_encode_tilegs"),
                       (50, b"k_encode_tileg2s"), (63, b"k_encode_tileg_lb"), (68, b"k_encode_tileg_a4")):
        set_tuning(6, arm)
        try:
            arr, _ = _run(device, shape, chunks, dtype, codecs, 0,
                          [((Ellipsis,), d), ((slice(3, 90), slice(5, 150), slice(0, 77)), 7)])
            arr[...] = d
            assert N.lib().zhip_last_kernel() == kname
        finally:
            set_tuning(6, 0)


def test_encode_tile4_nan_fill_merges_and_no_crc(device):
    shape, chunks = (128, 64, 128), (64, 64, 64)
    d = _data(shape, "float32")
    d[64:128, :, 0:64] = np.nan
    w = [((Ellipsis,), d), ((slice(0, 64), slice(None), slice(64, 128)), np.nan),
         ((slice(10, 100), slice(3, 60), slice(5, 120)), 2.5)]
    _run(device, shape, chunks, "float32", [T((2, 1, 0)), LE, CRC], np.nan, w)
    _run(device, shape, chunks, "float32", [T((2, 1, 0)), LE], np.nan, w[:2], write_empty=True)


def test_encode_tile4_sharded_inner(device):
    _run(device, (128, 128, 64), (128, 128, 64), "float32",
         [SHARD((64, 64, 64), [T((2, 1, 0)), LE, CRC])], 0.0,
         [((Ellipsis,), _data((128, 128, 64), "float32")), ((slice(0, 64), slice(64, 128)), 0.0)])


# ---- k_encode_tile: the general transposed encode (partial tiles, > 64
# tiles per chunk, other base steps, prefix-box edge chunks)

def _record_encode_flags(monkeypatch):
    from zarr_hip import writer

    seen = []
    orig = writer.EncodeLaunch.launch

    def launch(self, stream=None):
        seen.append((self.flags, self.plan.kernel_flags))
        return orig(self, stream)
    monkeypatch.setattr(writer.EncodeLaunch, "launch", launch)
    return seen


def _took_general_tile(seen) -> bool:
    from zarr_hip import _native as N

    return any((f & (N.DF_TILE | N.DF_TILE_PREFIX)) and (kf & N.PK_TILE) and
               not ((f & N.DF_TILE) and (kf & N.PK_TILE4_ENCODE)) for f, kf in seen)


@pytest.mark.parametrize("order", [(2, 1, 0), (1, 2, 0), (0, 2, 1), (2, 0, 1)])
@pytest.mark.parametrize("dtype,endian", [("float32", LE), ("int16", BE), ("float64", LE), ("uint8", LE)])
def test_encode_tile_general(device, monkeypatch, order, dtype, endian):
    """Partial tiles and edge chunks (prefix selections): (100, 72, 48) over
    (64, 48, 32) chunks; stored rows stay 16-byte multiples for every order."""
    seen = _record_encode_flags(monkeypatch)
    shape, chunks = (100, 72, 48), (64, 48, 32)
    d = _data(shape, dtype)
    d[0:64, 0:48, 0:32] = 0  # one whole chunk of fill: elided
    _run(device, shape, chunks, dtype, [T(order), endian, CRC], 0, [((Ellipsis,), d)])
    assert _took_general_tile(seen)


def test_encode_tile_many_tiles_per_chunk(device, monkeypatch):
    """128 x 128 x 64 float32 chunks, order (2, 1, 0): 256 tiles per chunk."""
    seen = _record_encode_flags(monkeypatch)
    shape = (256, 128, 64)
    d = _data(shape, "float32")
    _run(device, shape, (128, 128, 64), "float32", [T((2, 1, 0)), LE, CRC], np.nan,
         [((Ellipsis,), d), ((slice(5, 200), slice(7, 100), slice(0, 33)), 1.5)])
    assert _took_general_tile(seen)


def test_encode_tile_no_crc_nan_fill_and_sharded(device, monkeypatch):
    seen = _record_encode_flags(monkeypatch)
    shape = (96, 80, 48)
    d = _data(shape, "float32")
    d[0:32, 0:40, 0:48] = np.nan
    _run(device, shape, (32, 40, 48), "float32", [T((2, 0, 1)), LE], np.nan, [((Ellipsis,), d)])
    _run(device, (96, 80, 48), (96, 80, 48), "float32", [SHARD((48, 40, 24), [T((1, 2, 0)), LE, CRC])], 0.0,
         [((Ellipsis,), d), ((slice(0, 48), slice(40, 80)), 0.0)])
    assert _took_general_tile(seen)


def _took(seen, kind) -> bool:
    """kind "g": k_encode_tileg engaged (full selections, a group dim)."""
    from zarr_hip import _native as N

    return any((f & N.DF_TILE) and (kf & N.PK_TILE) and not (kf & N.PK_TILE4_ENCODE) for f, kf in seen)


@pytest.mark.parametrize("order", [(2, 1, 0), (1, 2, 0), (0, 2, 1), (2, 0, 1)])
@pytest.mark.parametrize("dtype,endian", [("float32", LE), ("int16", BE), ("float64", LE), ("uint8", LE)])
def test_encode_tileg_full_chunks(device, monkeypatch, order, dtype, endian):
    """Full chunks, partial tiles (80 rows) and > 64 tiles per chunk: (96, 160,
    160) over (96, 80, 80) chunks -- every order has a stored dim with shape
    % 4 == 0 other than tq and the innermost, so the grouped kernel runs."""
    seen = _record_encode_flags(monkeypatch)
    shape, chunks = (96, 160, 160), (96, 80, 80)
    d = _data(shape, dtype)
    d[0:96, 0:80, 0:80] = 0  # one whole chunk of fill: elided
    _run(device, shape, chunks, dtype, [T(order), endian, CRC], 0, [((Ellipsis,), d)])
    assert _took(seen, "g")

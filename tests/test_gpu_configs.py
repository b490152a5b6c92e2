"""GPU parity at the exact geometries bench.py measures (BASELINE.json configs,
workloads.py), every output byte compared with the CPU oracle.

  headline  256^3 f32, 128^3 shards of 64^3 inner chunks, bytes+crc32c, index at end
  C4        C4's inner geometry (128^3 shards of 32^3 inner chunks) on a 256^3 array,
            full read and the round-robin per-rank partition (src/zarr/core/
            codec_pipeline.py:1104-1109, 1169-1171: disjoint out selections)
  C5        C5's geometry (256^3 int16 shards of 64^3 inner chunks) on a 512^3 array,
            the seeded 10 % inner-chunk batch built exactly as bench.py builds it
  big CRC   chunks over 1 MiB with crc32c on the row kernel (more than 32 units of
            32 KiB per chunk: the arrival word cannot hold every unit's bit, the
            run end takes the multi-word path)
"""

import os
import sys

import numpy as np
import pytest

from oracle import oracle as O

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402

pytestmark = pytest.mark.gpu


def SHARD(inner_shape, codecs, loc="end"):
    return {"name": "sharding_indexed", "configuration": {
        "chunk_shape": list(inner_shape), "codecs": list(codecs),
        "index_codecs": [W.LE, W.CRC], "index_location": loc}}


def _device_array(device, meta, host):
    import zarr_hip

    store = zarr_hip.DeviceStore.from_host(host, device)
    arr = zarr_hip.Array.create(store, meta.shape, meta.chunk_shape, meta.dtype, meta.fill_value,
                                codecs=meta.codecs)
    return store, arr


def _to_bytes(t):
    from zarr_hip.buffer import to_numpy

    return to_numpy(t, "uint8" if t.element_size() == 1 else {2: "int16", 4: "int32", 8: "int64"}[
        t.element_size()]).tobytes()


@pytest.fixture(scope="module")
def headline(device):
    g = W.HEADLINE
    meta = O.ArrayMeta(g["shape"], g["shards"], np.dtype(g["dtype"]), 0.0,
                       codecs=[SHARD(g["inner"], [W.LE, W.CRC])])
    host = {}
    O.write(host, meta, (Ellipsis,), W.synthetic(g["shape"], seed=0))
    return meta, host


def test_headline_exact_geometry(device, headline):
    meta, host = headline
    store, arr = _device_array(device, meta, host)
    prog, out = arr.prepare_read((Ellipsis,))
    # the headline kernel: whole-row decode with the 8 index CRCs fused into the launch
    assert prog.tables.rows and prog.index is None and prog.data.n_idx == 8
    assert prog.data.d_rowmap is not None
    prog.launch()
    prog.results()
    want = O.read(host, meta)
    assert _to_bytes(out) == want.view(np.int32).tobytes()


def test_headline_crc_mismatch(device, headline):
    meta, host = headline
    bad = dict(host)
    blob = bytearray(bad["c/1/0/1"])
    blob[3 * 1048580 + 777] ^= 0x20  # an inner chunk's payload
    bad["c/1/0/1"] = bytes(blob)
    with pytest.raises(ValueError) as want:
        O.read(bad, meta)
    store, arr = _device_array(device, meta, bad)
    with pytest.raises(ValueError) as got:
        arr[...]
    assert str(got.value) == str(want.value)


@pytest.fixture(scope="module")
def c4_small(device):
    shape = (256, 256, 256)
    meta = O.ArrayMeta(shape, W.C4["shards"], np.dtype("float32"), 0.0,
                       codecs=[SHARD(W.C4["inner"], [W.LE, W.CRC])])
    host = {}
    O.write(host, meta, (Ellipsis,), W.synthetic(shape, seed=4))
    return meta, host, O.read(host, meta)


def test_c4_inner_geometry(device, c4_small):
    meta, host, want = c4_small
    store, arr = _device_array(device, meta, host)
    prog, out = arr.prepare_read((Ellipsis,))
    assert prog.tables.rows and prog.data.n_idx == 8 and len(prog.tables.chunks) == 8 * 64
    prog.launch()
    prog.results()
    assert _to_bytes(out) == want.view(np.int32).tobytes()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode", ["round_robin", "contiguous"])
def test_c4_partitioned_union(device, c4_small, world, mode):
    """Every rank's sub-batch decoded in turn into ONE out: the union is the
    oracle's array, and each rank writes only its own shards."""
    import torch

    from zarr_hip import parallel

    meta, host, want = c4_small
    store, arr = _device_array(device, meta, host)
    out = torch.full(meta.shape, float("nan"), dtype=torch.float32, device=device)
    seen = np.zeros(meta.shape, bool)
    for rank in range(world):
        regions = parallel.owned_regions(arr, (Ellipsis,), world, rank, mode)
        assert regions, "every rank owns at least one shard of the 8"
        before = out.clone()
        parallel.read_partitioned(arr, (Ellipsis,), world, rank, out=out, mode=mode)
        changed = (before.view(torch.int32) != out.view(torch.int32)).cpu().numpy()
        mask = np.zeros(meta.shape, bool)
        for r in regions:
            mask[r] = True
        assert not (changed & ~mask).any(), "a rank wrote outside its own shards"
        assert not (seen & mask).any(), "two ranks own the same region"
        seen |= mask
    assert seen.all()
    assert _to_bytes(out) == want.view(np.int32).tobytes()


def test_c5_geometry_seeded_batch(device):
    """C5's shard/inner geometry (256^3 int16 shards of 64^3 inner chunks) on a
    512^3 array; the batch is bench.py's: rng(1) 10 % of the inner chunks, one
    item per inner chunk, each decoded into its region of a full-shape out."""
    import torch

    shape = (512, 512, 512)
    g = W.C5
    meta = O.ArrayMeta(shape, g["shards"], np.dtype("int16"), 0,
                       codecs=[SHARD(g["inner"], [W.LE, W.CRC])])
    rng = np.random.default_rng(5)
    data = rng.integers(-2 ** 15, 2 ** 15, size=shape, dtype=np.int16)
    host = {}
    O.write(host, meta, (Ellipsis,), data)
    want = O.read(host, meta)
    store, arr = _device_array(device, meta, host)
    grid = tuple(s // i for s, i in zip(shape, g["inner"]))
    coords = W.partial_selection(grid)
    assert len(coords) == int(np.ceil(0.1 * np.prod(grid)))
    batch = W.inner_chunk_batch(arr, store, coords, g["inner"])
    sentinel = torch.full(shape, -12345, dtype=torch.int16, device=device)
    out = sentinel.clone()
    prog = arr.codec_pipeline.prepare_read(batch, out)
    assert prog.tables.rows
    prog.launch()
    res = prog.results()
    assert all(r["status"] == "present" for r in res)
    got = out.cpu().numpy()
    mask = np.zeros(shape, bool)
    for c in coords:
        sl = tuple(slice(int(x) * i, int(x) * i + i) for x, i in zip(c, g["inner"]))
        assert got[sl].tobytes() == want[sl].tobytes()
        mask[sl] = True
    assert (got[~mask] == -12345).all(), "the decode wrote outside the selected inner chunks"


@pytest.mark.parametrize("shape,chunks,sel", [
    ((256, 128, 64), (128, 64, 64), (Ellipsis,)),                    # 2 MiB chunks, 256-byte rows
    ((256, 128, 64), (128, 64, 64), (slice(5, 250), slice(3, 128), slice(None))),
    ((2 ** 21 + 2 ** 19,), (2 ** 20,), (Ellipsis,)),                  # 4 MiB 1-D chunks + an edge chunk
])
def test_row_kernel_chunks_over_1mib(device, shape, chunks, sel):
    """More than 32 units per chunk on the row kernel (nseg > 32 run end)."""
    import zarr_hip

    meta = O.ArrayMeta(shape, chunks, np.dtype("float32"), 1.5, codecs=[W.LE, W.CRC])
    host = {}
    O.write(host, meta, (Ellipsis,), W.synthetic(shape, seed=2))
    store, arr = _device_array(device, meta, host)
    prog, _ = arr.prepare_read(sel)
    assert prog.tables.rows
    nbytes = int(prog.tables.layout.nbytes)
    assert nbytes > (1 << 20) and prog.data.plan.units_per_chunk > 32
    got = arr[sel]
    assert got.tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()
    # a flipped bit in a late unit of a >1 MiB chunk is reported like the reference
    key = sorted(k for k in host if k.startswith("c/"))[-1]
    bad = dict(host)
    blob = bytearray(bad[key])
    blob[len(blob) - 4 - 40000] ^= 0x01
    bad[key] = bytes(blob)
    with pytest.raises(ValueError) as want:
        O.read(bad, meta)
    store2 = zarr_hip.DeviceStore.from_host(bad, device)
    arr2 = zarr_hip.Array.create(store2, shape, chunks, "float32", 1.5, codecs=[W.LE, W.CRC])
    with pytest.raises(ValueError) as got_e:
        arr2[...]
    assert str(got_e.value) == str(want.value)


@pytest.mark.parametrize("index_crc", [True, False])
def test_truncated_shard_on_device_store(device, index_crc):
    """A shard blob shorter than its index raises before any kernel reads it."""
    import zarr_hip

    index = [W.LE, W.CRC] if index_crc else [W.LE]
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 8], "codecs": [W.LE, W.CRC], "index_codecs": index}}]
    meta = O.ArrayMeta((16, 16), (16, 16), np.dtype("float32"), 0.0, codecs=codecs)
    host = {}
    O.write(host, meta, (Ellipsis,), W.synthetic((16, 16)))
    host["c/0/0"] = host["c/0/0"][:20]
    store, arr = _device_array(device, meta, host)
    with pytest.raises(ValueError, match="shorter than its index"):
        arr[...]


@pytest.mark.parametrize("kind", ["memory", "device"])
def test_c1_exact_geometry(device, kind):
    """BASELINE configs[0] at its exact geometry: 1e7 float32 1-D in (2**20,)
    chunks, bytes codec only (no CRC): 10 chunks, the last a boundary chunk
    stored at the full 4 MiB (562,816 items in the array, the rest fill).  The
    GPU write gives the oracle's store byte for byte; the GPU read gives the
    oracle's values, whole and for a ragged selection."""
    import zarr_hip

    n, c = 10 ** 7, 2 ** 20
    meta = O.ArrayMeta((n,), (c,), np.dtype("float32"), 0.0, codecs=[W.LE])
    data = W.synthetic((n,), seed=0)
    host = {}
    O.write(host, meta, (Ellipsis,), data)
    assert len(host) == 10 and len(host["c/9"]) == 4 * c
    store = zarr_hip.DeviceStore(device, capacity=48 << 20) if kind == "device" else zarr_hip.MemoryStore()
    arr = zarr_hip.Array.create(store, (n,), (c,), "float32", 0.0, codecs=[W.LE])
    arr[...] = data
    got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert got.keys() == host.keys()
    for k in host:
        assert got[k] == host[k], k
    assert arr[...].tobytes() == data.tobytes()
    sel = (slice(123457, 9_876_543, 1),)
    assert arr[sel].tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()


# --------------------------------------------- C4 / C5 at their FULL sizes
# The oracle cannot decode 4 GiB in seconds, so the full-size checks are the
# size-independent properties the domain offers: the GPU encode -> GPU decode
# round trip is the source bit for bit, a sample of the stored shards is
# byte-identical to what the oracle encodes from the same source region and
# decodes back to it, and a corrupted inner chunk is caught with the
# reference's message.

def _full(device, g, dtype):
    import torch

    import zarr_hip

    gen = torch.Generator(device=device).manual_seed(11)
    if dtype == "int16":
        src = torch.randint(-2 ** 15, 2 ** 15, g["shape"], generator=gen, device=device, dtype=torch.int16)
    else:
        src = torch.randn(g["shape"], generator=gen, device=device, dtype=torch.float32)
    n_shards = int(np.prod([s // c for s, c in zip(g["shape"], g["shards"])]))
    per = int(np.prod(g["shards"])) * src.element_size() + int(np.prod(
        [s // i for s, i in zip(g["shards"], g["inner"])])) * (4 + 16) + 4
    store = zarr_hip.DeviceStore(device, capacity=n_shards * (per + 256) + (1 << 24))
    arr = zarr_hip.Array.create(store, g["shape"], g["inner"], dtype, 0, shards=g["shards"],
                                inner_codecs=[W.LE, W.CRC])
    sb, _ = arr.batch_info((Ellipsis,))
    for i in range(0, len(sb), 64):
        arr.codec_pipeline.write_sync(sb[i:i + 64], src)
    torch.cuda.synchronize(device)
    return src, store, arr


def _oracle_shard_check(store, g, dtype, src, key, coords):
    meta = O.ArrayMeta(tuple(g["shards"]), tuple(g["shards"]), np.dtype(dtype), 0,
                       codecs=[SHARD(g["inner"], [W.LE, W.CRC])])
    region = tuple(slice(c * s, (c + 1) * s) for c, s in zip(coords, g["shards"]))
    want_vals = src[region].cpu().numpy()
    host = {}
    O.write(host, meta, (Ellipsis,), want_vals)
    got = store.get_sync(key).to_bytes()
    assert got == host["c/0/0/0"], f"stored shard {key} differs from the oracle's encoding"
    back = O.read({"c/0/0/0": got}, meta)
    assert back.tobytes() == want_vals.tobytes()


@pytest.mark.parametrize("which", ["c4", "c5"])
def test_full_size_roundtrip_and_oracle_sample(device, which):
    import torch

    g = W.C4 if which == "c4" else W.C5
    dtype = "float32" if which == "c4" else "int16"
    src, store, arr = _full(device, g, dtype)
    try:
        if which == "c4":
            out = arr.get((Ellipsis,))
            assert torch.equal(out.view(torch.int32), src.view(torch.int32))
            del out
        else:  # bench.py's C5 batch: rng(1) 10 % of the inner chunks into a full-shape out
            grid = tuple(s // i for s, i in zip(g["shape"], g["inner"]))
            coords = W.partial_selection(grid)
            batch = W.inner_chunk_batch(arr, store, coords, g["inner"])
            out = torch.zeros(g["shape"], dtype=torch.int16, device=device)
            arr.codec_pipeline.read_sync(batch, out)
            for it in batch[::97]:
                osel = tuple(it[3])
                assert torch.equal(out[osel], src[osel])
            del out
        grid = [s // c for s, c in zip(g["shape"], g["shards"])]
        for coords in [(0, 0, 0), tuple(x - 1 for x in grid), (grid[0] // 2, 1, grid[2] - 2)]:
            key = "c/" + "/".join(str(c) for c in coords)
            _oracle_shard_check(store, g, dtype, src, key, coords)
    finally:
        del src, store, arr
        torch.cuda.empty_cache()


def test_full_size_c4_corruption_caught(device):
    """One flipped bit in one inner chunk of the 4 GiB C4 array: the full read
    raises the reference's checksum message (crc32c_.py:46-49)."""
    import torch

    g = W.C4
    src, store, arr = _full(device, g, "float32")
    try:
        key = "c/3/5/7"
        ref = store.get_sync(key)
        off = ref.offset + 123457
        store.arena.buf[off] ^= 0x10
        with pytest.raises(ValueError, match="Stored and computed checksum do not match"):
            arr.get((Ellipsis,))
    finally:
        del src, store, arr
        torch.cuda.empty_cache()

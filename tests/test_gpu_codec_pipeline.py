"""The GPU half of the reference's tests/test_codec_pipeline.py, restated
against HipCodecPipeline with zarr-shaped stores, specs and buffers
(tests/zarr_fakes.py; zarr cannot be imported here):

* test_read_returns_get_results (tests/test_codec_pipeline.py:54-110): the
  low-level ``read`` coroutine returns one GetResult per chunk with status
  "present" / "missing";
* test_write_empty_chunks_false_no_store (:118-138): with
  ``write_empty_chunks=False`` fill-only chunks are never stored and read back
  as the fill.

The reference runs them with zarr's default chain (``bytes`` + the default
compressor, zstd -- absent here: the compressor slot is taken by a gzip
instance on the host stage) and with ``compressors=None``; both are run."""

import asyncio

import numpy as np
import pytest

from oracle import oracle as O
from tests import zarr_fakes as Z

pytestmark = pytest.mark.gpu

LE = {"name": "bytes", "configuration": {"endian": "little"}}


def _pipe(spec, compressed: bool):
    from zarr_hip import HipCodecPipeline

    codecs = Z.zcodecs([LE]) + ((Z.GzipCodec(level=5),) if compressed else ())
    return HipCodecPipeline.from_codecs(codecs).evolve_from_array_spec(spec)


@pytest.mark.parametrize("compressed", [False, True], ids=["no-compressor", "gzip"])
@pytest.mark.parametrize(("write_slice", "read_slice", "expected"), [
    (slice(None), slice(None), ("present", "present", "present")),
    (slice(0, 2), slice(None), ("present", "missing", "missing")),
    (None, slice(None), ("missing", "missing", "missing")),
])
def test_read_returns_get_results(device, compressed, write_slice, read_slice, expected):
    shape, chunks = (6,), (2,)
    spec = Z.ArraySpec(chunks, Z.ZDType("int64"), np.int64(-1), Z.ArrayConfig(), Z.cpu_prototype)
    pipe = _pipe(spec, compressed)
    store = Z.MemoryStore()
    if write_slice is not None:
        batch, shp = Z.batch_for(shape, chunks, (write_slice,), store, spec)
        pipe.write_sync(batch, Z.NDBuffer(np.zeros(shp, np.int64)))
    batch, shp = Z.batch_for(shape, chunks, (read_slice,), store, spec)
    out = Z.NDBuffer.create(shape=shp, dtype="int64")
    results = asyncio.run(pipe.read(batch, out, drop_axes=()))
    assert len(results) == len(expected)
    assert tuple(r["status"] for r in results) == expected
    want = np.full(shape, -1, np.int64)
    if write_slice is not None:
        want[write_slice] = 0
    assert out.as_numpy_array().tobytes() == want[read_slice].tobytes()


@pytest.mark.parametrize("compressed", [False, True], ids=["no-compressor", "gzip"])
def test_write_empty_chunks_false_no_store(device, compressed):
    shape, chunks = (20,), (10,)
    spec = Z.ArraySpec(chunks, Z.ZDType("float64"), np.float64(0.0), Z.ArrayConfig(write_empty_chunks=False),
                       Z.cpu_prototype)
    pipe = _pipe(spec, compressed)
    store = Z.MemoryStore()
    batch, shp = Z.batch_for(shape, chunks, (slice(None),), store, spec)
    asyncio.run(pipe.write(batch, Z.NDBuffer(np.zeros(shp, np.float64)), ()))
    assert "c/0" not in store._store_dict
    assert "c/1" not in store._store_dict
    out = Z.NDBuffer.create(shape=shp, dtype="float64")
    res = pipe.read_sync(batch, out)
    assert [r["status"] for r in res] == ["missing", "missing"]
    np.testing.assert_array_equal(out.as_numpy_array(), np.zeros(20, dtype="float64"))
    # the oracle agrees: nothing stored for an all-fill write
    meta = O.ArrayMeta(shape, chunks, np.dtype("float64"), 0.0, codecs=[LE], write_empty_chunks=False)
    want = {}
    O.write(want, meta, (Ellipsis,), np.zeros(shape, np.float64))
    assert want == {}

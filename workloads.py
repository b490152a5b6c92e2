"""Benchmark workloads shared by bench.py and the GPU tests (test infrastructure:
it builds inputs and batches, it computes nothing that is measured).

The BASELINE.json configs are defined once here so that a GPU test can check a
config at exactly the geometry bench.py times it at:

  synthetic()            seeded f32 data with a planted NaN payload and -0.0
  partial_selection()    C5's seeded random 10 % of inner chunks
  inner_chunk_batch()    one CodecPipeline batch item per selected inner chunk
                         (the reference's batch_info tuple, src/zarr/abc/codec.py:456-485)
"""

from __future__ import annotations

import numpy as np

LE = {"name": "bytes", "configuration": {"endian": "little"}}
CRC = {"name": "crc32c"}

# BASELINE.json configs; shard / inner shapes where BASELINE leaves them open
# are DESIGN.md's choices.
HEADLINE = dict(shape=(256, 256, 256), shards=(128, 128, 128), inner=(64, 64, 64), dtype="float32")
C4 = dict(shape=(1024, 1024, 1024), shards=(128, 128, 128), inner=(32, 32, 32), dtype="float32")
C5 = dict(shape=(2048, 2048, 2048), shards=(256, 256, 256), inner=(64, 64, 64), dtype="int16")
# the reference's own timing harness for this boundary
# (examples/codec_pipeline_performance/codec_pipeline_performance.py:67-80):
# 4096^2 int32 = 64 MiB, 16 shards of 1024^2, 256 inner chunks of 64^2 each,
# zarr's default sharding codecs (inner: bytes + the compressors, index:
# bytes + crc32c at the end), compressors None or gzip-6, fill 0
CPP_EXAMPLE = dict(shape=(4096, 4096), shards=(1024, 1024), inner=(64, 64), dtype="int32")
GZIP6 = {"name": "gzip", "configuration": {"level": 6}}


def cpp_example_data(kind: str) -> np.ndarray:
    """The example's inputs (codec_pipeline_performance.py:149-156): `plain` =
    arange (uncompressed runs), `noisy` = rng(0) integers in [0, 2**24) (gzip)."""
    shape = CPP_EXAMPLE["shape"]
    if kind == "plain":
        return np.arange(int(np.prod(shape)), dtype=np.int32).reshape(shape)
    return np.random.default_rng(0).integers(0, 2**24, size=shape, dtype=np.int32)


def synthetic(shape, seed=0) -> np.ndarray:
    """seed-`seed` standard normal f32, -0.0 at flat index 7, NaN payload 0x7FC00001 at 11."""
    rng = np.random.default_rng(seed)
    a = rng.standard_normal(shape, dtype=np.float32)
    flat = a.reshape(-1)
    flat[7] = -0.0
    flat[11:12].view(np.uint32)[0] = 0x7FC00001
    return a


def partial_selection(inner_grid, frac: float = 0.1, seed: int = 1) -> np.ndarray:
    """C5's selection: ceil(frac * n) inner chunks drawn without replacement with
    rng(seed), returned as sorted inner-grid coordinates (n_sel, ndim)."""
    n = int(np.prod(inner_grid))
    rng = np.random.default_rng(seed)
    pick = rng.choice(n, size=int(np.ceil(frac * n)), replace=False)
    return np.stack(np.unravel_index(np.sort(pick), tuple(inner_grid)), axis=1)


def inner_chunk_batch(arr, store, coords, inner):
    """One batch item per selected inner chunk of a sharded array: the shard's
    StorePath, the shard spec, the inner chunk's selection inside the shard and
    its region of a full-shape out (ShardingCodec partial decode,
    src/zarr/codecs/sharding.py:1222-1309, driven item by item)."""
    from zarr_hip.store import StorePath

    shards = arr.chunks
    per = [s // i for s, i in zip(shards, inner)]
    batch = []
    for c in coords:
        sc = tuple(int(x) // p for x, p in zip(c, per))
        lo = [int(x) % p * i for x, p, i in zip(c, per, inner)]
        csel = tuple(slice(l, l + i, 1) for l, i in zip(lo, inner))
        osel = tuple(slice(int(x) * i, int(x) * i + i, 1) for x, i in zip(c, inner))
        batch.append((StorePath(store, arr._key(sc)), arr.spec, csel, osel, False))
    return batch

#!/usr/bin/env python
"""Generate tests/golden/chunks/*.json: small zarr v3 stores written by the CPU
oracle (oracle/oracle.py, itself pinned by the CRC-32C KATs and the reference's
Morton vectors) -- SURVEY.md §8(c)'s golden chunk fixtures: 8^3..32^3 chunks,
one 2x2x2 shard, big-endian, NaN / -0.0 payloads, a transpose and a gzip
chain.  Each file: the zarr.json document, every stored object (base64) and the
decoded array (base64, native order).  Re-run only to regenerate:

    python tests/golden/make_chunk_fixtures.py
"""

import base64
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

LE = {"name": "bytes", "configuration": {"endian": "little"}}
BE = {"name": "bytes", "configuration": {"endian": "big"}}
CRC = {"name": "crc32c"}


def planted(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        a = rng.standard_normal(shape).astype(dt)
        f = a.reshape(-1)
        f[1] = -0.0
        f[2] = np.nan
        if dt.itemsize == 4:
            f[3:4].view(np.uint32)[0] = 0x7FC00001  # a NaN payload
            f[4:5].view(np.uint32)[0] = 0xFF800001  # a signalling-pattern NaN
        return a
    info = np.iinfo(dt)
    return rng.integers(info.min, info.max, size=shape, dtype=dt, endpoint=True)


CASES = [
    ("f32_16c_8c_le_crc", (16, 16, 16), (8, 8, 8), "float32", "NaN", [LE, CRC]),
    ("i16_32x24_8x8_be", (32, 24), (8, 8), "int16", -1, [BE]),
    ("f64_20x13_8x8_be_crc_edge", (20, 13), (8, 8), "float64", 0.0, [BE, CRC]),
    ("f32_shard_2x2x2_of_8c", (16, 16, 16), (16, 16, 16), "float32", 0.0,
     [{"name": "sharding_indexed", "configuration": {"chunk_shape": [8, 8, 8], "codecs": [LE, CRC],
                                                     "index_codecs": [LE, CRC], "index_location": "end"}}]),
    ("u16_shard_index_start", (32, 32), (16, 32), "uint16", 7,
     [{"name": "sharding_indexed", "configuration": {"chunk_shape": [8, 8], "codecs": [BE, CRC],
                                                     "index_codecs": [LE, CRC], "index_location": "start"}}]),
    ("f32_transpose_210_crc", (32, 16, 8), (16, 8, 8), "float32", 0.0,
     [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, LE, CRC]),
    ("f32_gzip", (24, 24), (8, 12), "float32", 0.0, [LE, {"name": "gzip", "configuration": {"level": 1}}]),
]


def main():
    out_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "chunks")
    os.makedirs(out_dir, exist_ok=True)
    for i, (name, shape, chunks, dtype, fill, codecs) in enumerate(CASES):
        dt = np.dtype(dtype)
        fv = np.nan if fill == "NaN" else fill
        data = planted(shape, dtype, seed=100 + i)
        if name.startswith("f32_shard"):
            data[0:8, 8:16, 0:8] = 0.0  # one inner chunk equal to the fill: elided
        meta = O.ArrayMeta(shape, chunks, dt, fv, codecs=codecs)
        store = {}
        O.write(store, meta, (Ellipsis,), data)
        assert O.read(store, meta).tobytes() == data.tobytes()
        doc = {"zarr_format": 3, "node_type": "array", "shape": list(shape), "data_type": dt.name,
               "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": list(chunks)}},
               "chunk_key_encoding": {"name": "default", "configuration": {"separator": "/"}},
               "fill_value": fill, "codecs": codecs, "attributes": {}}
        rec = {"generator": "tests/golden/make_chunk_fixtures.py (oracle/oracle.py)", "zarr.json": doc,
               "store": {k: base64.b64encode(bytes(v)).decode() for k, v in sorted(store.items())},
               "decoded": {"dtype": dt.str, "shape": list(shape),
                           "bytes": base64.b64encode(np.ascontiguousarray(data).tobytes()).decode()}}
        with open(os.path.join(out_dir, name + ".json"), "w") as fh:
            json.dump(rec, fh, indent=0)
        print(name, len(store), "objects")


if __name__ == "__main__":
    main()

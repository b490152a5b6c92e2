"""GPU round trips of the arrays the reference's own v3 metadata fixtures
describe (tests/golden/metadata/, from packages/zarr-metadata/tests/v3/array/):
the zarr.json document is put in a store, the array opened from it, seeded
data written and read back through the GPU pipeline; values are compared bit
for bit and stores byte for byte with the CPU oracle (its keys mapped for the
v2 chunk key encoding)."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_decode import _data

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(__file__), "golden", "metadata")


@pytest.mark.parametrize("kind", ["memory", "device"])
@pytest.mark.parametrize("name", ["transpose_and_crc32c_codecs", "sharding_indexed_codec", "gzip_codec",
                                  "regular_grid_default_encoding", "regular_grid_v2_encoding",
                                  "with_optionals"])
def test_fixture_array_roundtrip(name, kind, device):
    import zarr_hip

    with open(os.path.join(HERE, name + ".json")) as fh:
        doc = json.load(fh)
    store = zarr_hip.MemoryStore() if kind == "memory" else zarr_hip.DeviceStore(device)
    store.set_sync("zarr.json", json.dumps(doc).encode())
    arr = zarr_hip.Array.open(store)
    md = arr.metadata
    data = _data(md.shape, md.dtype)
    arr[...] = data
    meta = O.ArrayMeta(md.shape, md.chunk_shape, md.dtype, md.fill_value, codecs=doc["codecs"])
    host: dict = {}
    O.write(host, meta, (Ellipsis,), data)
    got = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    if md.key_encoding == "v2":
        host = {md.chunk_key(tuple(int(c) for c in k.split("/")[1:])): v for k, v in host.items()}
    assert got == host
    assert arr[...].tobytes() == data.tobytes()
    sel = tuple(slice(s // 5, s - s // 7, 3) for s in md.shape)
    assert np.asarray(arr[sel]).tobytes() == np.ascontiguousarray(data[sel]).tobytes()

"""GPU decode and encode of the golden chunk fixtures (tests/golden/chunks/):
the stored objects decode to the recorded arrays bit for bit (NaN payloads,
-0.0, big-endian items, edge chunks, a 2x2x2 shard with an elided inner chunk,
an index at the shard start, a transpose, a gzip chain), from host and HBM
stores; writing the recorded array gives the recorded stored bytes."""

import json
import os

import pytest

from test_golden_chunks import FIX, load_fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["memory", "device"])
@pytest.mark.parametrize("path", FIX, ids=lambda p: os.path.basename(p)[:-5])
def test_gpu_decodes_and_encodes_fixture(path, kind, device):
    import numpy as np

    import zarr_hip

    doc, meta, store, want = load_fixture(path)
    host = dict(store)
    host["zarr.json"] = json.dumps(doc).encode()
    st = zarr_hip.DeviceStore.from_host(host, device) if kind == "device" else zarr_hip.MemoryStore(host)
    arr = zarr_hip.Array.open(st)
    assert arr[...].tobytes() == want.tobytes()
    sel = tuple(slice(1, s, 3) for s in want.shape)
    assert np.asarray(arr[sel]).tobytes() == np.ascontiguousarray(want[sel]).tobytes()
    fresh = zarr_hip.DeviceStore(device) if kind == "device" else zarr_hip.MemoryStore()
    fresh.set_sync("zarr.json", json.dumps(doc).encode())
    w = zarr_hip.Array.open(fresh)
    w[...] = want
    got = {k: bytes(v) for k, v in fresh.to_dict().items() if not k.endswith("zarr.json")}
    assert got == store

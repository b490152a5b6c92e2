"""The reference's own performance workload for this boundary, on the GPU
path (examples/codec_pipeline_performance/codec_pipeline_performance.py:
67-80, 95-130): a 4096^2 int32 array in 16 shards of 1024^2, 256 inner chunks
of 64^2 per shard, zarr's default sharding codecs, compressors None (arange
data) or gzip-6 (noisy data), on memory and local stores.  As the example
does, one full write then one full read; here the stored bytes are compared
with the CPU oracle's encoding of the same data (byte-identical store: same
keys, same shard blobs, gzip with mtime 0) and the read with the source, bit
for bit.  A device store runs the uncompressed chain end to end in HBM."""

import numpy as np
import pytest

import workloads as W
from oracle import oracle as O

pytestmark = pytest.mark.gpu

LE = {"name": "bytes", "configuration": {"endian": "little"}}


def _shard_meta(compressed: bool):
    g = W.CPP_EXAMPLE
    inner = [LE] + ([W.GZIP6] if compressed else [])
    codecs = [{"name": "sharding_indexed", "configuration": {"chunk_shape": list(g["inner"]), "codecs": inner,
                                                             "index_location": "end"}}]
    return O.ArrayMeta(g["shape"], g["shards"], np.dtype(g["dtype"]), 0, codecs=codecs), inner


@pytest.fixture(scope="module")
def oracle_stores():
    out = {}
    for compressed in (False, True):
        meta, _ = _shard_meta(compressed)
        data = W.cpp_example_data("noisy" if compressed else "plain")
        host: dict = {}
        O.write(host, meta, (Ellipsis,), data)
        out[compressed] = (meta, data, host)
    return out


@pytest.mark.parametrize("kind", ["memory", "local", "device"])
@pytest.mark.parametrize("compressed", [False, True], ids=["uncompressed", "gzip6"])
def test_cpp_example_write_then_read(kind, compressed, oracle_stores, tmp_path, device):
    import zarr_hip

    if kind == "device" and compressed:
        pytest.skip("compression runs on the host stage; the device store case is the uncompressed chain")
    g = W.CPP_EXAMPLE
    meta, data, host = oracle_stores[compressed]
    _, inner = _shard_meta(compressed)
    store = {"memory": lambda: zarr_hip.MemoryStore(), "local": lambda: zarr_hip.LocalStore(str(tmp_path / "s")),
             "device": lambda: zarr_hip.DeviceStore(device)}[kind]()
    arr = zarr_hip.Array.create(store, g["shape"], g["inner"], g["dtype"], 0, shards=g["shards"],
                                inner_codecs=inner)
    arr[...] = data
    stored = {k: bytes(v) for k, v in store.to_dict().items() if not k.endswith("zarr.json")}
    assert sorted(stored) == sorted(host)
    for k in host:
        assert stored[k] == host[k], k
    got = np.asarray(arr[...])
    assert got.dtype == np.int32 and got.tobytes() == data.tobytes()
    # a partial read crossing shard and inner-chunk edges, against the oracle
    sel = (slice(1000, 1100, 3), slice(60, 2100))
    assert np.asarray(arr[sel]).tobytes() == np.ascontiguousarray(O.read(host, meta, sel)).tobytes()


def test_cpp_example_device_resident_kernel(oracle_stores, device):
    """The uncompressed chain read from HBM by one launch (the index CRCs in
    the data launch's leading workgroups), bit-exact, and a flipped index bit
    raising the reference's message."""
    import torch

    import zarr_hip

    g = W.CPP_EXAMPLE
    meta, data, host = oracle_stores[False]
    store = zarr_hip.DeviceStore.from_host(host, device)
    arr = zarr_hip.Array.create(store, g["shape"], g["inner"], g["dtype"], 0, shards=g["shards"],
                                inner_codecs=[LE])
    out = torch.empty(g["shape"], dtype=torch.int32, device=device)
    prog, out = arr.prepare_read((Ellipsis,), out=out)
    prog.launch()
    prog.results()
    from zarr_hip import _native as N
    assert N.lib().zhip_last_kernel() == b"k_decode_lead4", "16 KiB inner chunks: four per workgroup"
    assert prog.index is None and prog.data.n_idx == 16, "index checks fused into the data launch"
    assert out.cpu().numpy().tobytes() == data.tobytes()
    bad = dict(host)
    b = bytearray(bad["c/2/1"])
    b[-100] ^= 0x01
    bad["c/2/1"] = bytes(b)
    with pytest.raises(ValueError) as want:
        O.read(bad, meta)
    arr2 = zarr_hip.Array.create(zarr_hip.DeviceStore.from_host(bad, device), g["shape"], g["inner"], g["dtype"],
                                 0, shards=g["shards"], inner_codecs=[LE])
    with pytest.raises(ValueError) as got:
        arr2[...]
    assert str(got.value) == str(want.value)

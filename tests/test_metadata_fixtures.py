"""CPU checks against the reference's own v3 metadata fixtures
(tests/golden/metadata/, copied from packages/zarr-metadata/tests/v3/array/):
each document parses into this package's ArrayMetadata and builds a
HipCodecPipeline through the zarr-side hook (from_array_metadata_and_store,
src/zarr/core/array.py:221-228); the documents that name codecs or grids off
this path are refused loudly.  GPU round trips of the same arrays:
tests/test_gpu_metadata_fixtures.py."""

import json
import math
import os

import numpy as np
import pytest

import zarr_fakes as Z

HERE = os.path.join(os.path.dirname(__file__), "golden", "metadata")


def load(name):
    with open(os.path.join(HERE, name + ".json")) as fh:
        return json.load(fh)


SUPPORTED = ["transpose_and_crc32c_codecs", "sharding_indexed_codec", "gzip_codec",
             "regular_grid_default_encoding", "regular_grid_v2_encoding", "with_optionals"]


@pytest.mark.parametrize("name", SUPPORTED)
def test_fixture_parses_and_builds_a_pipeline(name):
    from zarr_hip import ArrayMetadata, HipCodecPipeline

    d = load(name)
    md = ArrayMetadata.from_json(d)
    assert md.shape == tuple(d["shape"])
    assert md.chunk_shape == tuple(d["chunk_grid"]["configuration"]["chunk_shape"])
    assert md.dtype == np.dtype(d["data_type"])
    if d["fill_value"] == "NaN":
        assert math.isnan(float(md.fill_value))
    else:
        assert md.fill_value == d["fill_value"]
    # the zarr-side construction hook, with zarr-shaped metadata objects
    zmd = Z.ArrayV3Metadata(tuple(d["shape"]), Z.ZDType(d["data_type"]), Z.RegularChunkGrid(md.chunk_shape),
                            md.fill_value, Z.zcodecs(d["codecs"]))
    p = HipCodecPipeline.from_array_metadata_and_store(zmd, Z.MemoryStore())
    p.validate(shape=zmd.shape, dtype=zmd.data_type, chunk_grid=zmd.chunk_grid)
    assert [c.to_dict()["name"] for c in p.codecs] == [c["name"] for c in d["codecs"]]
    n = int(np.prod(md.chunk_shape)) * md.dtype.itemsize
    names = [c["name"] for c in d["codecs"]]
    if "gzip" in names or "sharding_indexed" in names:
        with pytest.raises(NotImplementedError):
            p.compute_encoded_size(n)
    else:
        assert p.compute_encoded_size(n) == n + 4 * names.count("crc32c")


def test_fixture_details():
    from zarr_hip import ArrayMetadata
    from zarr_hip.codecs import GzipCodec, ShardingCodec, TransposeCodec

    t = ArrayMetadata.from_json(load("transpose_and_crc32c_codecs"))
    assert isinstance(t.codecs[0], TransposeCodec) and t.codecs[0].order == (2, 1, 0)
    s = ArrayMetadata.from_json(load("sharding_indexed_codec"))
    sc = s.codecs[0]
    assert isinstance(sc, ShardingCodec) and sc.chunk_shape == (64, 64) and sc.index_location == "end"
    assert isinstance(sc.codecs[1], GzipCodec) and sc.codecs[1].level == 1
    assert sc.shard_index_size(16) == 16 * 16 + 4
    v2 = ArrayMetadata.from_json(load("regular_grid_v2_encoding"))
    assert v2.key_encoding == "v2" and v2.chunk_key((1,)) == "1"  # chunk_key_encodings.py:103-105
    dflt = ArrayMetadata.from_json(load("regular_grid_default_encoding"))
    assert dflt.chunk_key((3, 4)) == "c/3/4"
    o = ArrayMetadata.from_json(load("with_optionals"))
    assert o.attributes["tags"] == ["test", "metadata"]
    # the document written back keeps what the path needs
    back = ArrayMetadata.from_json(o.to_json())
    assert back.shape == o.shape and back.chunk_shape == o.chunk_shape and math.isnan(float(back.fill_value))


@pytest.mark.parametrize("name,exc,what", [
    ("zstd_codec", NotImplementedError, "zstd"),
    ("blosc_codec", NotImplementedError, "blosc"),
])
def test_fixture_off_the_path_is_refused(name, exc, what):
    from zarr_hip import ArrayMetadata

    with pytest.raises(exc, match=what):
        ArrayMetadata.from_json(load(name))


def test_named_config_dtype_refused():
    from zarr_hip import ArrayMetadata

    with pytest.raises((TypeError, NotImplementedError, ValueError)):
        ArrayMetadata.from_json(load("datatype_named_config"))

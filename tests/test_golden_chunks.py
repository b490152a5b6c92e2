"""CPU pin of the golden chunk fixtures (tests/golden/chunks/, written by
tests/golden/make_chunk_fixtures.py from the oracle): the oracle decodes every
fixture store to its recorded array and re-encodes that array to the same
stored bytes.  The GPU decodes / encodes them in tests/test_gpu_golden.py."""

import base64
import glob
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

FIX = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "chunks", "*.json")))


def load_fixture(path):
    with open(path) as fh:
        rec = json.load(fh)
    doc = rec["zarr.json"]
    fill = np.nan if doc["fill_value"] == "NaN" else doc["fill_value"]
    meta = O.ArrayMeta(tuple(doc["shape"]), tuple(doc["chunk_grid"]["configuration"]["chunk_shape"]),
                       np.dtype(doc["data_type"]), fill, codecs=doc["codecs"])
    store = {k: base64.b64decode(v) for k, v in rec["store"].items()}
    d = rec["decoded"]
    want = np.frombuffer(base64.b64decode(d["bytes"]), dtype=np.dtype(d["dtype"])).reshape(d["shape"])
    return doc, meta, store, want


def test_fixtures_present():
    assert len(FIX) >= 7


@pytest.mark.parametrize("path", FIX, ids=lambda p: os.path.basename(p)[:-5])
def test_oracle_pins_fixture(path):
    doc, meta, store, want = load_fixture(path)
    assert O.read(store, meta).tobytes() == want.tobytes()
    again = {}
    O.write(again, meta, (Ellipsis,), want)
    assert again == store

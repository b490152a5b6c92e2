"""Host logic of the multi-device pipeline (zarr_hip.parallel.device_bands /
outer_dim): the batch's items split into bands of the out along its outermost
dim, balanced, disjoint, covering."""

import numpy as np
import pytest

from oracle import oracle as O


def _batch(shape, chunks, sel):
    pr, out_shape = O.basic_indexer(sel, shape, chunks)
    return [(None, None, cs, os_, comp) for _, cs, os_, comp in pr], out_shape


@pytest.mark.parametrize("n_dev", [2, 3, 4, 8])
@pytest.mark.parametrize("sel", [(Ellipsis,), (slice(5, 120, 3), slice(None), slice(7, 60))])
def test_bands_cover_and_balance(n_dev, sel):
    from zarr_hip.parallel import device_bands

    batch, out_shape = _batch((128, 96, 64), (16, 32, 32), sel)
    groups = device_bands(batch, n_dev, 0)
    assert 1 <= len(groups) <= n_dev
    seen = sorted(j for _, _, idx in groups for j in idx)
    assert seen == list(range(len(batch)))
    at = 0
    for lo, hi, idx in groups:
        assert lo == at and hi > lo
        at = hi
        for j in idx:
            s = batch[j][3][0]
            assert lo <= s.start and s.stop <= hi
    assert at == out_shape[0]
    sizes = [len(idx) for _, _, idx in groups]
    assert max(sizes) - min(sizes) <= max(1, len(batch) // (4 * n_dev) * 4)


def test_outer_dim_and_unsplittable():
    from zarr_hip.parallel import device_bands, outer_dim

    assert outer_dim((4096, 64, 1), (10, 64, 64)) == 0
    assert outer_dim((1, 10, 640), (10, 64, 64)) == 2
    assert outer_dim((64, 64, 1), (1, 64, 64)) == 1  # a length-1 outer dim is skipped
    batch, _ = _batch((64, 64), (16, 16), (5, slice(None)))  # int selection: the out is 1-d
    assert [len(g[2]) for g in device_bands(batch, 2, 0)] == [2, 2]
    assert device_bands(batch, 2, 1) is None  # no such out dim
    one, _ = _batch((16, 64), (16, 16), (Ellipsis,))
    assert len(device_bands(one, 4, 0)) == 1  # one band: nothing to split


def test_devices_config():
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import BytesCodec
    from zarr_hip.pipeline import _parse_devices

    assert _parse_devices("0, 1,2") == (0, 1, 2)
    assert _parse_devices(["cuda:3", 4]) == (3, 4)
    assert _parse_devices(None) == ()
    p = HipCodecPipeline.from_codecs([BytesCodec()], devices="0,1")
    assert p.devices == (0, 1)
    assert p.evolve_from_array_spec(__import__("zarr_hip").spec.ArraySpec((4,), np.dtype("f4"), 0.0)).devices == (0, 1)

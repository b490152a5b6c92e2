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
    # a scalar selection: a 0-d out has no dim to band along (found by the
    # device-list fuzz, tests/test_gpu_multidevice.py::test_random_device_list)
    assert outer_dim((), ()) == 0
    scalar, shape = _batch((64, 64), (16, 16), (5, 7))
    assert shape == () and device_bands(scalar, 2, outer_dim((), shape)) is None


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


class _FakeArena:
    def __init__(self, index):
        import torch

        self.device = torch.device("cuda", index)


def _dev_store(index):
    """A DeviceStore on GPU `index` without touching a GPU (placement only
    reads the store's device)."""
    from zarr_hip.store import DeviceStore

    st = DeviceStore.__new__(DeviceStore)
    st.arena = _FakeArena(index)
    return st


class _Path:
    def __init__(self, store):
        self.store = store


@pytest.mark.parametrize("out_dev", [0, 1, None])
def test_placement_single_device_store(out_dev):
    """Every item of one DeviceStore on GPU 0 decodes on GPU 0, whatever the
    out's device: no encoded bytes move between GPUs (read_multi then moves
    only decoded bands)."""
    from zarr_hip.parallel import placement

    batch, _ = _batch((128, 96), (16, 32), (Ellipsis,))
    st = _dev_store(0)
    batch = [(_Path(st),) + it[1:] for it in batch]
    assert placement(batch, out_dev) == {0: list(range(len(batch)))}


def test_placement_mixed_sources():
    """Items on two GPUs stay where their bytes are; host-resident items go
    with the out's device (or, for a host out, the device holding most)."""
    from zarr_hip.parallel import placement

    batch, _ = _batch((128, 96), (16, 32), (Ellipsis,))
    s0, s3 = _dev_store(0), _dev_store(3)
    srcs = [s0, s3, None, s3, s3, None] * (len(batch) // 6 + 1)
    batch = [((_Path(s) if s is not None else _Path(None)),) + it[1:] for s, it in zip(srcs, batch)]
    by = placement(batch, 0)
    assert sorted(by) == [0, 3]
    assert all(srcs[j] is s3 for j in by[3])
    assert all(srcs[j] is not s3 for j in by[0])
    by_host = placement(batch, None)
    assert all(srcs[j] is not s0 for j in by_host[3])  # host items joined GPU 3 (most items)
    host_only = [(_Path(None),) + it[1:] for it in batch]
    assert placement(host_only, 0) is None


def test_item_bands_exclusive_and_interleaved():
    """Parts whose items form disjoint bands move one band per run; a part
    interleaved with another moves item by item (None)."""
    from zarr_hip.parallel import item_bands

    batch, _ = _batch((128, 96), (16, 32), (Ellipsis,))
    rows = [it[3][0].start // 16 for it in batch]
    top = [j for j, r in enumerate(rows) if r < 4]
    bottom = [j for j, r in enumerate(rows) if r >= 4]
    assert item_bands(batch, [top, bottom], 0) == [[(0, 64)], [(64, 128)]]
    even = [j for j, r in enumerate(rows) if r % 2 == 0]
    odd = [j for j, r in enumerate(rows) if r % 2 == 1]
    assert item_bands(batch, [even, odd], 0) == [[(0, 16), (32, 48), (64, 80), (96, 112)],
                                                [(16, 32), (48, 64), (80, 96), (112, 128)]]
    cols = [it[3][1].start // 32 for it in batch]
    left = [j for j, c in enumerate(cols) if c == 0]
    rest = [j for j, c in enumerate(cols) if c > 0]
    assert item_bands(batch, [left, rest], 0) == [None, None]  # both span every row band

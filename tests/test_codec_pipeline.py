"""The CPU half of the reference's tests/test_codec_pipeline.py, restated
against HipCodecPipeline (zarr itself cannot be imported here):

* the codec-order property (tests/test_codec_pipeline.py:263-323):
  ``from_codecs`` must raise exactly what ``codecs_from_list``
  (src/zarr/core/codec_pipeline.py:886-944) raises -- its adjacent-pair scan
  decides TypeError vs ValueError -- with this package's codecs and with
  zarr-shaped codec instances classified by their base class;
* ``test_evolve_threads_spec_preserving_serializer_endian`` (:189-261): a
  dtype-widening array->array codec in front of ``bytes`` must be threaded
  into the serializer's evolve, so it keeps its endian.

The GPU half (GetResult statuses, write_empty_chunks) is
tests/test_gpu_codec_pipeline.py."""

from dataclasses import dataclass, replace

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from tests import zarr_fakes as Z

_AA, _AB, _BB = "AA", "AB", "BB"


def _expected_codec_order_outcome(labels: list) -> str:
    """Independent prediction of codecs_from_list's outcome (the reference
    test's own oracle, tests/test_codec_pipeline.py:283-306, restated)."""
    prev = None
    seen_ab = False
    for cur in labels:
        if cur == _AA:
            if prev in (_AB, _BB):
                return "TypeError"
        elif cur == _AB:
            if prev == _BB:
                return "TypeError"
            if seen_ab:
                return "ValueError"
            seen_ab = True
        elif prev == _AA:
            return "TypeError"
        prev = cur
    return "ok" if seen_ab else "ValueError"


def _own_factory():
    from zarr_hip.codecs import BytesCodec, GzipCodec, TransposeCodec

    return {_AA: lambda: TransposeCodec(order=(0, 1)), _AB: BytesCodec, _BB: GzipCodec}


# zarr-shaped codec instances: the pipeline sees zarr's own TransposeCodec /
# BytesCodec / GzipCodec objects, whose kind is their base class
# (src/zarr/abc/codec.py:228-262)
class ArrayArrayCodec:
    pass


class ArrayBytesCodec:
    pass


class BytesBytesCodec:
    pass


class _ZTranspose(ArrayArrayCodec):
    def to_dict(self):
        return {"name": "transpose", "configuration": {"order": (0, 1)}}


class _ZBytes(ArrayBytesCodec):
    def to_dict(self):
        return {"name": "bytes", "configuration": {"endian": "little"}}


class _ZGzip(Z.GzipCodec, BytesBytesCodec):
    pass


_ZARR_FACTORY = {_AA: _ZTranspose, _AB: _ZBytes, _BB: _ZGzip}


def _check(labels, factory):
    from zarr_hip import HipCodecPipeline

    codecs = [factory[lab]() for lab in labels]
    expected = _expected_codec_order_outcome(labels)
    if expected == "TypeError":
        with pytest.raises(TypeError):
            HipCodecPipeline.from_codecs(codecs)
    elif expected == "ValueError":
        with pytest.raises(ValueError):
            HipCodecPipeline.from_codecs(codecs)
    else:
        p = HipCodecPipeline.from_codecs(codecs)
        assert len(p.array_array_codecs) == labels.count(_AA)
        assert len(p.bytes_bytes_codecs) == labels.count(_BB)


@settings(max_examples=300, deadline=None)
@given(labels=st.lists(st.sampled_from([_AA, _AB, _BB]), min_size=1, max_size=5))
def test_codecs_from_list_outcome_matches_order_rules(labels):
    _check(labels, _own_factory())


@settings(max_examples=200, deadline=None)
@given(labels=st.lists(st.sampled_from([_AA, _AB, _BB]), min_size=1, max_size=5))
def test_codecs_from_list_order_rules_zarr_instances(labels):
    _check(labels, _ZARR_FACTORY)


@pytest.mark.parametrize("labels,err", [
    ([_BB], ValueError),                 # no array->bytes codec (the scan finds no pair violation)
    ([_AB, _BB, _AB], TypeError),        # AB right after BB is an order violation first
    ([_AA, _BB, _AB], TypeError),        # BB right after AA
    ([_AB, _AB], ValueError),            # two array->bytes codecs
    ([_AB, _AA], TypeError),
    ([_AA, _AA, _AB, _BB, _BB], None),
])
def test_codecs_from_list_named_cases(labels, err):
    """The cases round 3 classified differently from the reference."""
    from zarr_hip import HipCodecPipeline

    codecs = [_own_factory()[lab]() for lab in labels]
    if err is None:
        HipCodecPipeline.from_codecs(codecs)
    else:
        with pytest.raises(err):
            HipCodecPipeline.from_codecs(codecs)


def test_sharding_combination_warns():
    """codecs_from_list's advisory when sharding is combined with other codecs
    (codec_pipeline.py:876-882)."""
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import Crc32cCodec, ShardingCodec

    with pytest.warns(UserWarning, match="sharding_indexed"):
        HipCodecPipeline.from_codecs([ShardingCodec(chunk_shape=(2,)), Crc32cCodec()])


@dataclass(frozen=True)
class _WidenToInt16(ArrayArrayCodec):
    """Test-only array->array codec: reports the encoded dtype as int16 (the
    reference test's stub, tests/test_codec_pipeline.py:213-240)."""

    is_fixed_size = True

    def to_dict(self):
        return {"name": "_widen_to_int16"}

    def resolve_metadata(self, chunk_spec):
        return replace(chunk_spec, dtype=Z.ZDType("int16"))

    def compute_encoded_size(self, input_byte_length, _spec):
        return input_byte_length


def test_evolve_threads_spec_preserving_serializer_endian():
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import BytesCodec

    spec = Z.ArraySpec((4,), Z.ZDType("int8"), np.int8(0), Z.ArrayConfig(order="C", write_empty_chunks=False),
                       Z.cpu_prototype)
    pipe = HipCodecPipeline.from_codecs((_WidenToInt16(), BytesCodec(endian="little")))
    evolved = pipe.evolve_from_array_spec(spec)
    ser = evolved.array_bytes_codec
    assert isinstance(ser, BytesCodec)
    assert ser.endian is not None, "the serializer was evolved against the int8 source, not the widened int16"
    # the same chain with zarr-shaped codec objects
    evolved2 = HipCodecPipeline.from_codecs((_WidenToInt16(), _ZBytes())).evolve_from_array_spec(spec)
    assert evolved2.array_bytes_codec.endian == "little"
    # and without the widening codec, bytes on int8 drops its endian (bytes.py:74-95)
    plain = HipCodecPipeline.from_codecs((BytesCodec(endian="little"),)).evolve_from_array_spec(spec)
    assert plain.array_bytes_codec.endian is None


def test_foreign_array_codec_is_not_run():
    """An array->array codec other than transpose is accepted for spec
    threading but a read through it fails loudly (no CPU fallback)."""
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import BytesCodec
    from zarr_hip.planner import analyze_chain
    from zarr_hip.spec import coerce_spec

    spec = Z.ArraySpec((4,), Z.ZDType("int8"), np.int8(0), Z.ArrayConfig(), Z.cpu_prototype)
    ev = HipCodecPipeline.from_codecs((_WidenToInt16(), BytesCodec(endian="little"))).evolve_from_array_spec(spec)
    with pytest.raises(NotImplementedError, match="_widen_to_int16"):
        analyze_chain(ev.codecs, coerce_spec(spec))

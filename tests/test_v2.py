"""zarr v2's codec wrapper (V2Codec, src/zarr/codecs/_v2.py:19-96) on the CPU:
the mapping to the GPU's fixed-size chain plus the host stage, the host
stage's decode / encode order, the F-order transpose added at evolve time, and
what is refused (the GPU half runs in tests/test_gpu_pipeline_suite.py's v2
scenarios).  The numcodecs objects are restated fakes (tests/zarr_fakes.py)."""

import numpy as np
import pytest

from zarr_fakes import NumDelta, NumGZip, V2Codec


def _spec(shape, dtype="float64", order="C"):
    from zarr_hip.spec import ArrayConfig, ArraySpec

    return ArraySpec(shape, np.dtype(dtype), 0, ArrayConfig(order=order))


def test_v2_chain_mapping():
    from zarr_hip import HipCodecPipeline
    from zarr_hip.codecs import BytesCodec, TransposeCodec, V2Stage

    p = HipCodecPipeline.from_codecs([V2Codec()]).evolve_from_array_spec(_spec((10,)))
    assert [type(c) for c in p.codecs] == [BytesCodec]  # raw chunks: nothing on the host
    p = HipCodecPipeline.from_codecs([V2Codec([NumDelta("f8")], NumGZip(1))]).evolve_from_array_spec(_spec((10,)))
    assert [type(c) for c in p.codecs] == [BytesCodec, V2Stage]
    assert p._host_split() is not None
    # order="F": the raw chunk is the array in Fortran order = a reversing transpose
    pf = HipCodecPipeline.from_codecs([V2Codec(None, NumGZip(1))]).evolve_from_array_spec(_spec((4, 6, 2), order="F"))
    assert isinstance(pf.codecs[0], TransposeCodec) and pf.codecs[0].order == (2, 1, 0)
    with pytest.raises(NotImplementedError):
        HipCodecPipeline.from_codecs([V2Codec()]).evolve_from_array_spec(_spec((10,), dtype=">f8"))


@pytest.mark.parametrize("order", ["C", "F"])
def test_v2_stage_matches_wrapper_order(order):
    """_v2.py:25-93: encode = astype(order) -> filters -> compressor; decode the
    reverse, then the bytes in memory order."""
    from zarr_hip.codecs import V2Stage

    spec = _spec((5, 4), order=order)
    a = np.arange(20, dtype="f8").reshape(5, 4) * 1.5 + 1
    raw = np.asarray(a, order=order).reshape(-1, order="A").view(np.uint8).tobytes()
    st = V2Stage((NumDelta("f8"),), NumGZip(1))
    enc = st.encode_bytes(raw, spec)
    ref = NumGZip(1).encode(NumDelta("f8").encode(np.asarray(a, order=order)))
    assert enc == ref
    assert st.decode_bytes(enc, spec) == raw
    # compressor only / filters only
    assert V2Stage((), NumGZip(1)).decode_bytes(V2Stage((), NumGZip(1)).encode_bytes(raw, spec), spec) == raw
    assert V2Stage((NumDelta("f8"),), None).decode_bytes(
        V2Stage((NumDelta("f8"),), None).encode_bytes(raw, spec), spec) == raw

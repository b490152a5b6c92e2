"""zarr_hip — MI355X-native zarr v3 codec pipeline (fixed-size chain on the GPU).

Drop-in for zarr-python's CodecPipeline (src/zarr/abc/codec.py:315-508): see
``HipCodecPipeline``.  Select it in a zarr >= 3.3 environment with
``zarr.config.set({"codec_pipeline.path": "zarr_hip.HipCodecPipeline"})``
(INTEGRATION.md).  Kernels live in ``csrc/`` behind the C ABI in
``include/zarrhip.h``; there is no CPU fallback.
"""

from .array import Array, ArrayMetadata, ChunkNotFoundError
from .buffer import Buffer, BufferPrototype, NDBuffer, buffer_prototype
from .codecs import BytesCodec, Crc32cCodec, ShardingCodec, TransposeCodec
from .pipeline import DecodeProgram, HipCodecPipeline, ReadGraph
from .spec import ArrayConfig, ArraySpec, GetResult
from .store import DeviceStore, LocalStore, MemoryStore, PinnedMemoryStore, StorePath

__all__ = [
    "Array", "ArrayMetadata", "ArrayConfig", "ArraySpec", "Buffer", "BufferPrototype", "BytesCodec",
    "ChunkNotFoundError", "NDBuffer", "buffer_prototype",
    "Crc32cCodec", "DecodeProgram", "DeviceStore", "GetResult", "HipCodecPipeline", "LocalStore",
    "MemoryStore", "PinnedMemoryStore", "ReadGraph", "ShardingCodec", "StorePath", "TransposeCodec",
]

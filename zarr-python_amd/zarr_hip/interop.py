"""Duck-typed conversions at the CodecPipeline boundary.

zarr-python hands a pipeline its own objects (src/zarr/abc/codec.py:315-508):
``Codec`` instances (``to_dict()``), ``ArraySpec`` with a ``ZDType`` dtype
(``to_native_dtype()``, src/zarr/core/array_spec.py:137-186), ``NDBuffer`` /
``Buffer`` values (``as_ndarray_like()`` / ``as_array_like()`` /
``as_numpy_array()``, src/zarr/core/buffer/core.py:130-567), ByteGetters whose
``get_sync`` returns such Buffers and ByteSetters whose ``set_sync`` only takes
them (src/zarr/storage/_memory.py:110-138), and byte-range request objects
(src/zarr/abc/store.py).  This module turns those into what the planner and
the kernels take -- torch tensors, numpy bytes, numpy dtypes -- without
importing zarr (which needs Python >= 3.12): every check is on the interface.
"""

from __future__ import annotations

from typing import Any

import numpy as np

from .store import DeviceRef, DeviceStore, MemoryStore

KDL_ROCM = 10  # DLPack device type of ROCm/HIP memory


def _torch():
    import torch

    return torch


def native_dtype(dtype) -> np.dtype:
    """np.dtype of a numpy dtype, a dtype-like or a zarr ZDType (to_native_dtype)."""
    if hasattr(dtype, "to_native_dtype"):
        return np.dtype(dtype.to_native_dtype())
    return np.dtype(dtype)


def ndarray_like(x) -> Any:
    """Unwrap an NDBuffer / Buffer to the array it holds (torch, numpy or other)."""
    seen = 0
    while seen < 4:
        seen += 1
        if hasattr(x, "as_ndarray_like"):
            x = x.as_ndarray_like()
        elif hasattr(x, "as_array_like") and not isinstance(x, np.ndarray):
            x = x.as_array_like()
        else:
            break
    return x


def _is_device_dlpack(x) -> bool:
    dev = getattr(x, "__dlpack_device__", None)
    if dev is None:
        return False
    try:
        return int(dev()[0]) == KDL_ROCM
    except Exception:
        return False


def device_tensor(x):
    """The torch CUDA (ROCm) tensor behind x (zero-copy), or None when x lives in
    host memory."""
    torch = _torch()
    a = ndarray_like(x)
    if isinstance(a, torch.Tensor):
        return a if a.is_cuda else None
    if _is_device_dlpack(a):
        return torch.from_dlpack(a)
    return None


def host_array(x) -> np.ndarray | None:
    """The numpy array behind a host-resident NDBuffer / Buffer / array-like, or None."""
    torch = _torch()
    a = ndarray_like(x)
    if isinstance(a, np.ndarray):
        return a
    if isinstance(a, torch.Tensor):
        return a.numpy() if not a.is_cuda else None
    if hasattr(x, "as_numpy_array") and device_tensor(x) is None:
        return np.asarray(x.as_numpy_array())
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(a, dtype=np.uint8)
    if hasattr(a, "__array__") and device_tensor(a) is None:
        return np.asarray(a)
    return None


def byte_payload(value, host: bool = False):
    """A stored value's bytes: a 1-D uint8 torch CUDA tensor when device-resident
    (and host=False), else a 1-D uint8 numpy array.  Accepts bytes-likes, numpy,
    torch, zarr Buffers and this package's buffers."""
    torch = _torch()
    if isinstance(value, (bytes, bytearray, memoryview)):
        return np.frombuffer(value, dtype=np.uint8)
    if isinstance(value, DeviceRef):
        value = value.arena.view(value.offset, value.length)
    t = device_tensor(value)
    if t is not None:
        t = t.reshape(-1).view(torch.uint8) if t.is_contiguous() else t.contiguous().reshape(-1).view(torch.uint8)
        return t.cpu().numpy() if host else t
    a = host_array(value)
    if a is None:
        raise TypeError(f"cannot take the bytes of a {type(value).__name__}")
    return np.ascontiguousarray(a).reshape(-1).view(np.uint8)


def staged_bytes(raw):
    """What a ByteGetter returned, as something staging can pack: a DeviceRef /
    device tensor stays on the device; host buffers become uint8 numpy views."""
    if raw is None or isinstance(raw, (DeviceRef, bytes, bytearray, memoryview)):
        return raw
    if type(raw) is np.ndarray and raw.dtype == np.uint8 and raw.ndim == 1 and raw.flags.c_contiguous:
        return raw  # a pinned store's arena view, already host bytes
    t = device_tensor(raw)
    if t is not None:
        return t.reshape(-1).view(_torch().uint8)
    return byte_payload(raw)


def wrap_for_setter(data: bytes, prototype):
    """Bytes in the form a ByteSetter accepts: zarr stores require a Buffer of the
    spec's prototype (MemoryStore.set_sync, src/zarr/storage/_memory.py:129-138);
    this package's stores take raw bytes."""
    buf_cls = getattr(prototype, "buffer", None)
    if buf_cls is not None and hasattr(buf_cls, "from_bytes"):
        return buf_cls.from_bytes(data)
    return data


def is_own_store(obj) -> bool:
    return isinstance(obj, (DeviceStore, MemoryStore))


def request_classes(store=None):
    """(RangeByteRequest, SuffixByteRequest) to hand to `store`: this package's for
    its own stores, zarr's (src/zarr/abc/store.py) for zarr stores when zarr is
    importable, else this package's (duck-typed stores read them by attribute)."""
    from . import store as S

    if store is None or not is_own_store(store):
        try:  # pragma: no cover - needs zarr >= 3 (Python >= 3.12)
            from zarr.abc.store import RangeByteRequest, SuffixByteRequest

            return RangeByteRequest, SuffixByteRequest
        except Exception:
            pass
    return S.RangeByteRequest, S.SuffixByteRequest


def is_missing_key_error(exc: BaseException) -> bool:
    """FileNotFoundError, or zarr's BaseExceptionGroup of them (get_ranges_sync,
    src/zarr/abc/store.py:474-539; handled as a missing shard like
    src/zarr/codecs/sharding.py:1662-1672)."""
    if isinstance(exc, FileNotFoundError):
        return True
    subs = getattr(exc, "exceptions", None)
    return bool(subs) and all(is_missing_key_error(e) for e in subs)

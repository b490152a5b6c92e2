"""Device buffers on ROCm: torch tensors stand in for the reference's CuPy-backed
gpu.Buffer / gpu.NDBuffer (src/zarr/core/buffer/gpu.py:34-237), which cannot
run on ROCm.  torch is used for device memory and streams only; every codec
operation on these buffers is a HIP kernel of this package."""

from __future__ import annotations

import numpy as np

_MAP = None


def torch_dtype(dtype) -> "torch.dtype":
    import torch

    global _MAP
    if _MAP is None:
        _MAP = {
            np.dtype("bool"): torch.bool, np.dtype("uint8"): torch.uint8,
            np.dtype("int8"): torch.int8, np.dtype("int16"): torch.int16,
            np.dtype("uint16"): torch.uint16, np.dtype("int32"): torch.int32,
            np.dtype("uint32"): torch.uint32, np.dtype("int64"): torch.int64,
            np.dtype("uint64"): torch.uint64, np.dtype("float16"): torch.float16,
            np.dtype("float32"): torch.float32, np.dtype("float64"): torch.float64,
            np.dtype("complex64"): torch.complex64,
        }
    dt = np.dtype(dtype).newbyteorder("=")
    if dt not in _MAP:
        raise TypeError(f"dtype {dt} has no device representation")
    return _MAP[dt]


def empty(shape, dtype, device, order: str = "C"):
    """prototype.nd_buffer.empty (array.py:5456-5460): C or F ordered device array."""
    import torch

    td = torch_dtype(dtype)
    if order == "F" and len(shape) > 1:
        return torch.empty(tuple(reversed(shape)), dtype=td, device=device).permute(
            *reversed(range(len(shape))))
    return torch.empty(tuple(shape), dtype=td, device=device)


def to_numpy(t, dtype) -> np.ndarray:
    """Device tensor -> numpy with the array's dtype (bit-exact: via raw bytes).

    One hipMemcpyAsync into pinned host memory (DMA at full PCIe rate, no
    pageable bounce); the returned array keeps the pinned block alive."""
    import torch

    dt = np.dtype(dtype).newbyteorder("=")
    c = t.contiguous() if not t.is_contiguous() else t
    flat = c.reshape(-1).view(torch.uint8)
    if not flat.is_cuda:
        return flat.numpy().view(dt).reshape(tuple(t.shape))
    host = torch.empty(flat.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(flat, non_blocking=True)
    torch.cuda.current_stream(flat.device).synchronize()
    return host.numpy().view(dt).reshape(tuple(t.shape))

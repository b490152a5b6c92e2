"""ArraySpec / ArrayConfig / GetResult restated (src/zarr/core/array_spec.py:40-186,
src/zarr/abc/codec.py:40-43)."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Literal, TypedDict

import numpy as np


class GetResult(TypedDict):
    status: Literal["present", "missing"]


@dataclass(frozen=True)
class ArrayConfig:
    """array_spec.py:40-105 (the fields this path reads)."""

    order: Literal["C", "F"] = "C"
    write_empty_chunks: bool = False
    read_missing_chunks: bool = True
    sharding_coalesce_max_gap_bytes: int = 1 << 20
    sharding_coalesce_max_bytes: int = 16 << 20


@dataclass(frozen=True)
class ArraySpec:
    shape: tuple[int, ...]
    dtype: np.dtype
    fill_value: Any
    config: ArrayConfig = ArrayConfig()
    prototype: Any = None
    # the caller's own spec object (zarr's ArraySpec) this one was made from:
    # host-stage codec instances are handed that one (HostCodec)
    source: Any = field(default=None, compare=False, hash=False, repr=False)

    def __post_init__(self):
        object.__setattr__(self, "shape", tuple(int(s) for s in self.shape))
        dt = self.dtype
        object.__setattr__(self, "dtype", np.dtype(dt.to_native_dtype() if hasattr(dt, "to_native_dtype")
                                                   else dt))
        object.__setattr__(self, "config", coerce_config(self.config))

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def order(self) -> str:
        return self.config.order

    def fill_bytes(self) -> bytes:
        """The fill value as native-order item bytes (fill_value_or_default,
        chunk_utils.py:61-71)."""
        b = self.__dict__.get("_fill_b")
        if b is None:  # memoised: the spec is frozen
            fv = self.fill_value
            if fv is None:
                fv = 0
            b = np.asarray(fv, dtype=self.dtype).astype(self.dtype.newbyteorder("=")).tobytes()
            object.__setattr__(self, "_fill_b", b)
        return b


def coerce_config(config) -> ArrayConfig:
    """This package's ArrayConfig from zarr's (array_spec.py:39-119) or a dict."""
    if isinstance(config, ArrayConfig):
        return config
    if config is None:
        return ArrayConfig()
    get = config.get if isinstance(config, dict) else (lambda k, d: getattr(config, k, d))
    base = ArrayConfig()
    return ArrayConfig(
        order=get("order", base.order),
        write_empty_chunks=bool(get("write_empty_chunks", base.write_empty_chunks)),
        read_missing_chunks=bool(get("read_missing_chunks", base.read_missing_chunks)),
        sharding_coalesce_max_gap_bytes=int(get("sharding_coalesce_max_gap_bytes",
                                                base.sharding_coalesce_max_gap_bytes)),
        sharding_coalesce_max_bytes=int(get("sharding_coalesce_max_bytes",
                                            base.sharding_coalesce_max_bytes)))


def coerce_spec(spec) -> ArraySpec:
    """This package's ArraySpec from zarr's (array_spec.py:137-186): the dtype is
    a ZDType there (``to_native_dtype()``), the fill value a numpy scalar, the
    prototype a BufferPrototype (kept: writes hand it back to the store)."""
    if isinstance(spec, ArraySpec):
        return spec
    from .interop import native_dtype

    fv = spec.fill_value
    if hasattr(fv, "item") and not isinstance(fv, np.generic):
        fv = fv.item()
    return ArraySpec(tuple(int(s) for s in spec.shape), native_dtype(spec.dtype), fv,
                     coerce_config(getattr(spec, "config", None)), getattr(spec, "prototype", None),
                     source=spec)

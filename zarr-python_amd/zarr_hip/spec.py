"""ArraySpec / ArrayConfig / GetResult restated (src/zarr/core/array_spec.py:40-186,
src/zarr/abc/codec.py:40-43)."""

from __future__ import annotations

from dataclasses import dataclass
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

    def __post_init__(self):
        object.__setattr__(self, "shape", tuple(int(s) for s in self.shape))
        object.__setattr__(self, "dtype", np.dtype(self.dtype))

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def order(self) -> str:
        return self.config.order

    def fill_bytes(self) -> bytes:
        """The fill value as native-order item bytes (fill_value_or_default,
        chunk_utils.py:61-71)."""
        fv = self.fill_value
        if fv is None:
            fv = 0
        return np.asarray(fv, dtype=self.dtype).astype(self.dtype.newbyteorder("=")).tobytes()

"""Multi-GPU partitioning: one process per GPU, chunks split across ranks.

Chunks (or shards) are independent — the reference's read_sync already maps
them over a pool with disjoint out selections (src/zarr/core/codec_pipeline.py:
1104-1109, 1169-1171) — so a batch is partitioned into per-rank sub-batches
with no collective on the data path.  RCCL (torch.distributed "nccl") is only
used by callers for barriers / timing reductions, and by `gather_to` for an
optional post-step gather of results onto one rank.
"""

from __future__ import annotations

import numpy as np


def partition(n_items: int, world: int, rank: int, mode: str = "round_robin") -> np.ndarray:
    """Indices of the batch items owned by `rank` (disjoint, covering)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    idx = np.arange(int(n_items))
    if mode == "round_robin":
        return idx[rank::world]
    if mode == "contiguous":
        per, rem = divmod(int(n_items), world)
        start = rank * per + min(rank, rem)
        return idx[start: start + per + (1 if rank < rem else 0)]
    raise ValueError(f"unknown partition mode {mode!r}")


def rank_batch(batch: list, world: int, rank: int, mode: str = "round_robin") -> list:
    """The rank's sub-batch of a CodecPipeline batch_info list."""
    return [batch[i] for i in partition(len(batch), world, rank, mode)]


def read_partitioned(array, selection, world: int, rank: int, out=None, mode: str = "round_robin"):
    """Each rank decodes only its chunks of `selection` into its own device
    `out` (full selection shape; the other ranks' regions are left untouched).
    Returns (out, results)."""
    import torch

    from . import buffer

    batch, out_shape = array.batch_info(selection)
    mine = rank_batch(batch, world, rank, mode)
    if out is None:
        dev = torch.device("cuda", torch.cuda.current_device())
        out = buffer.empty(out_shape, array.metadata.dtype, dev, array.config.order)
    if not mine:
        return out, ()
    return out, array.codec_pipeline.read_sync(mine, out)


def owned_regions(array, selection, world: int, rank: int, mode: str = "round_robin"):
    """Out selections owned by `rank` (for assembling / checking partitioned reads)."""
    batch, _ = array.batch_info(selection)
    return [batch[i][3] for i in partition(len(batch), world, rank, mode)]

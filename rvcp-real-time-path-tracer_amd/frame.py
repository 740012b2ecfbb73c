"""Multi-GPU frame assembly.

A frame is cut into 8-row stripes (the reference's 8x8 workgroup rows,
src/ray_tracer/vulkan.rs:266); stripe s belongs to rank s % world.  Each rank renders its
stripes packed into a [slot_rows, W] int32 buffer (one RGBA8 texel per int32), the buffers
are gathered to rank 0 with ONE collective (RCCL over xGMI with the 'nccl' backend; gloo on
CPU tests), and rank 0 un-permutes them with rvcp_assemble_frame_async (device) -- or
`assemble_host` below, the same index map on the host.  Pixel values do not depend on the
sharding: the RNG seed depends only on the global (x, y) (ray_tracer_games101_branch.comp:
487-489), so an N-rank frame is bit-identical to a 1-rank frame.
"""
from __future__ import annotations

import numpy as np

from .ray_tracer import shard_row_ids, shard_rows


def slot_rows(height: int, world: int) -> int:
    return max(shard_rows(height, k, world) for k in range(world))


def gather_shards(shard_buf, rank: int, world: int, dst: int = 0, out=None):
    """Gather every rank's [slot, W] shard buffer to `dst` with one torch.distributed gather.
    `out` (dst only, optional): a contiguous [world, slot, W] tensor the shards land in
    without a copy.  Returns the list of per-rank tensors on dst, None elsewhere."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [shard_buf]
    parts = None
    if rank == dst:
        parts = list(out.unbind(0)) if out is not None else \
            [torch.empty_like(shard_buf) for _ in range(world)]
    dist.gather(shard_buf, parts, dst=dst)
    return parts


def assemble_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """Host twin of assemble_kernel: gathered [world, slot, W] -> frame [H, W]."""
    frame = np.empty((height, width) + gathered.shape[3:], dtype=gathered.dtype)
    for k in range(world):
        rows = shard_row_ids(height, k, world)
        frame[rows] = gathered[k, :len(rows)]
    return frame

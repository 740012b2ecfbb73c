"""Sharding invariance and the N>1 gather path on CPU (no GPU).

The oracle plays the part of each rank's kernel; the gather runs over torch.distributed
'gloo' with world_size 2 (the product uses the same rvcp_amd.frame.gather_shards over
RCCL); rank 0 assembles with the host twin of the device assemble kernel."""
import os
import socket

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from rvcp_amd import frame as FR
from conftest import scene_arrays

TIME = 123.0


def _render_shard(sc, cfg, W, H, rank, world):
    """This rank's stripes, packed in increasing stripe order: [rows, W, 4] u8."""
    arrays = scene_arrays(sc)
    parts = []
    stripes = (H + 7) // 8
    for s in range(rank, stripes, world):
        h = min(8, H - 8 * s)
        _, rgba, _ = O.render(arrays, sc.push_constant(TIME), cfg, W, H, rect=(0, 8 * s, W, h),
                              threads=2, want_linear=False)
        parts.append(rgba)
    return np.concatenate(parts, axis=0) if parts else np.zeros((0, W, 4), np.uint8)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_union_is_full_frame(cornell, world):
    W, H = 40, 37
    cfg = rvcp_amd.abi.make_config(spp=2)
    _, full, _ = O.render(scene_arrays(cornell), cornell.push_constant(TIME), cfg, W, H,
                          want_linear=False)
    slot = FR.slot_rows(H, world)
    gathered = np.zeros((world, slot, W, 4), np.uint8)
    for k in range(world):
        part = _render_shard(cornell, cfg, W, H, k, world)
        assert len(part) == rvcp_amd.shard_rows(H, k, world)
        gathered[k, :len(part)] = part
    assert np.array_equal(FR.assemble_host(gathered, W, H, world), full)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = rvcp_amd.Scene.default()
        cfg = rvcp_amd.abi.make_config(spp=2)
        W, H = 48, 44
        part = _render_shard(sc, cfg, W, H, rank, world)
        slot = FR.slot_rows(H, world)
        buf = torch.zeros((slot, W), dtype=torch.int32)
        buf[:len(part)] = torch.from_numpy(part.view(np.int32).reshape(len(part), W))
        got = FR.gather_shards(buf, rank, world)
        if rank == 0:
            g = torch.stack(got).numpy().view(np.uint8).reshape(world, slot, W, 4)
            frame = FR.assemble_host(g, W, H, world)
            _, full, _ = O.render(scene_arrays(sc), sc.push_constant(TIME), cfg, W, H,
                                  want_linear=False)
            np.save(os.path.join(outdir, "ok.npy"), np.array([np.array_equal(frame, full)]))
    finally:
        dist.destroy_process_group()


def test_gloo_two_rank_gather(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert bool(np.load(tmp_path / "ok.npy")[0])


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("H", [2048, 1024, 37, 8, 1])
def test_gather_entry_point_geometry(world, H):
    """The buffer geometry rvcp_gather_frame_async relies on (include/rvcp.h), from the C-ABI's
    rvcp_shard_rows: every rank sends rvcp_shard_rows(H, 0, world) rows (shard 0 has the most;
    shorter shards send padding), the N slots cover the frame exactly once, and the device
    assembly (assemble_kernel, stripe s -> slot s % N, row (s / N) * 8 + y % 8) puts every row
    where a 1-GPU render has it."""
    L = rvcp_amd.abi.load()
    rows = [int(L.rvcp_shard_rows(H, k, world)) for k in range(world)]
    slot = int(L.rvcp_shard_rows(H, 0, world))
    assert sum(rows) == H and max(rows) == slot == FR.slot_rows(H, world)
    # the gathered buffer carries each row's global index; the kernel's index arithmetic
    gathered = np.full((world, slot), -1, np.int64)
    for k in range(world):
        ids = FR.shard_row_ids(H, k, world)
        assert len(ids) == rows[k]
        gathered[k, :rows[k]] = ids
    frame_rows = np.empty(H, np.int64)
    for y in range(H):
        stripe = y >> 3
        shard = stripe % world
        lrow = (stripe // world) * 8 + (y & 7)
        frame_rows[y] = gathered[shard, lrow]
    assert np.array_equal(frame_rows, np.arange(H))

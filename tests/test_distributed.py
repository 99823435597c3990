"""Multi-rank screen-tile sharding on CPU (gloo, world_size 2 and 3).

Each rank renders ONLY its interleaved tiles' rows with the CPU oracle
(standing in for the GPU render), packs them tile-major, the packed buffers
are gathered to rank 0 over torch.distributed, and rank 0 untiles them.  The
assembled frame must equal a single-rank full-frame render bit for bit --
including pre-pass pixels, whose half-res footprint each rank recomputes.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world_size, port, flags, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    from oracle import oracle as O
    from rvgrt_amd import tiles
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import TEST_POSES_128

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    O.set_threads(2)
    W, H, T = 160, 96, 32
    w = O.OracleWorld(6, 6, 6, atlas=load_atlas()).build(gi_sweeps=1)
    pos, yaw, pitch = TEST_POSES_128["P0"]
    pos = (pos[0] / 2, pos[1] / 2, pos[2] / 2)
    cam = O.camera_from_pose(pos, yaw, pitch, W, H)
    fr = O.make_frame(W, H, flags, cam)
    tx_n, ty_n = tiles.tile_grid(W, H, T)
    ntiles = tx_n * ty_n
    mine = tiles.rank_tiles(ntiles, rank, world_size)
    # render only the rows my tiles cover (the oracle renders whole rows)
    img = np.zeros((H, W, 4), np.uint8)
    for ty in sorted({int(t) // tx_n for t in mine}):
        r = O.render(w, fr, ty * T, min(H, ty * T + T))
        img[ty * T:ty * T + T] = r["rgba"][ty * T:ty * T + T]
    packed = tiles.pack_tiles(img, mine, T, pad_to=tiles.max_tiles_per_rank(ntiles, world_size))
    bufs = tiles.gather_frame(dist, torch.from_numpy(packed), rank, world_size)
    if rank == 0:
        frame = np.zeros((H, W, 4), np.uint8)
        for q in range(world_size):
            ids = tiles.rank_tiles(ntiles, q, world_size)
            tiles.untile(bufs[q].numpy(), ids, T, frame)
        full = O.render(w, fr)["rgba"]
        np.save(out_path, np.stack([frame, full]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,flags", [(2, 8), (3, 7)])
def test_tile_gather_reassembles_frame(tmp_path, world_size, flags):
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_worker, args=(world_size, _free_port(), flags, out), nprocs=world_size,
                       join=True, start_method="spawn")
    frame, full = np.load(out)
    assert np.array_equal(frame, full)
    assert len(np.unique(full.reshape(-1, 4), axis=0)) > 20


def test_tile_assignment_covers_frame_once():
    from rvgrt_amd import tiles
    for (W, H, T, N) in [(1920, 1080, 64, 8), (3840, 2160, 64, 3), (640, 360, 32, 4)]:
        tx, ty = tiles.tile_grid(W, H, T)
        seen = np.concatenate([tiles.rank_tiles(tx * ty, r, N) for r in range(N)])
        assert np.array_equal(np.sort(seen), np.arange(tx * ty))
        counts = [len(tiles.rank_tiles(tx * ty, r, N)) for r in range(N)]
        assert max(counts) - min(counts) <= 1
        assert max(counts) == tiles.max_tiles_per_rank(tx * ty, N)


def test_pack_untile_roundtrip():
    from rvgrt_amd import tiles
    rng = np.random.default_rng(0)
    img = rng.integers(0, 255, (100, 150, 4), np.uint8)
    tx, ty = tiles.tile_grid(150, 100, 32)
    out = np.zeros_like(img)
    for r in range(3):
        ids = tiles.rank_tiles(tx * ty, r, 3)
        tiles.untile(tiles.pack_tiles(img, ids, 32), ids, 32, out)
    assert np.array_equal(out, img)


@pytest.mark.parametrize("world_size", [2, 4, 8])
def test_weighted_shard_assignment(world_size):
    """rv_tile_shard_assign (host-only C ABI, the native loop's deal): equal
    weights reproduce the plain interleave; a lighter rank 0 gets about
    root_weight times the others' tiles, still spread over the whole frame;
    every tile has exactly one owner."""
    from rvgrt_amd.tiles import rank_tiles, shard_owners
    W, H, T = 1920, 1080, 16
    own = shard_owners(W, H, T, world_size, 1.0)
    nt = own.size
    for r in range(world_size):
        assert np.array_equal(np.flatnonzero(own == r), rank_tiles(nt, r, world_size))
    w0 = 1.0 - 0.019 * (world_size - 1)
    own = shard_owners(W, H, T, world_size, w0)
    counts = np.bincount(own, minlength=world_size)
    assert counts.sum() == nt and counts.min() > 0
    others = counts[1:].mean()
    assert abs(counts[0] / others - w0) < 0.01
    assert counts[1:].max() - counts[1:].min() <= 1
    gaps = np.diff(np.flatnonzero(own == 0))
    assert gaps.max() <= 2 * world_size   # rank 0's tiles stay interleaved over the frame

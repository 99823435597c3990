"""Screen-tile sharding of a frame across GPUs.

Every pixel of the reference frame depends only on read-only world data plus
a 2x2 half-res neighbourhood, so a frame splits into independent tiles.
Tiles of T x T pixels are dealt round-robin over ranks (interleaving keeps
sky and terrain tiles mixed on every rank), each rank renders its tiles
against its own replica of the world and packs them tile-major; rank 0
gathers the packed buffers (RCCL over xGMI when the backend is "nccl") and
scatters them into the frame.  The numpy pack/untile functions are the host
restatement of k_render_tiles' packing and k_untile (rv_kernels.hip).
"""
from __future__ import annotations

import numpy as np


def tile_grid(width: int, height: int, tile_px: int):
    """(tiles_x, tiles_y); tile id = ty * tiles_x + tx."""
    return (width + tile_px - 1) // tile_px, (height + tile_px - 1) // tile_px


def rank_tiles(ntiles: int, rank: int, world_size: int) -> np.ndarray:
    """Interleaved assignment: rank r owns tiles r, r+N, r+2N, ..."""
    return np.arange(rank, ntiles, world_size, dtype=np.int32)


def shard_owners(width: int, height: int, tile_px: int, world_size: int, root_weight: float = 1.0) -> np.ndarray:
    """Owner rank of every tile as the native loop deals them (rv_tile_shard_assign,
    host-only C ABI): interleaved, rank 0 weighing root_weight.  Equal weights give
    rank_tiles' assignment."""
    from . import _lib
    import ctypes as C
    nt = len(np.arange(0, ((width + tile_px - 1) // tile_px) * ((height + tile_px - 1) // tile_px)))
    out = np.empty(nt, np.int32)
    st = _lib.load().rv_tile_shard_assign(int(width), int(height), int(tile_px), int(world_size),
                                          float(root_weight), out.ctypes.data_as(C.c_void_p))
    if st != 0:
        raise ValueError(f"rv_tile_shard_assign: status {st}")
    return out


def max_tiles_per_rank(ntiles: int, world_size: int) -> int:
    return (ntiles + world_size - 1) // world_size


def pack_tiles(img: np.ndarray, ids, tile_px: int, pad_to: int | None = None) -> np.ndarray:
    """Tile-major packing of an (H, W, C) image; pixels outside the image are 0."""
    H, W = img.shape[:2]
    tx_n, _ = tile_grid(W, H, tile_px)
    n = len(ids) if pad_to is None else pad_to
    out = np.zeros((n, tile_px, tile_px) + img.shape[2:], img.dtype)
    for slot, t in enumerate(ids):
        tx, ty = t % tx_n, t // tx_n
        y0, x0 = ty * tile_px, tx * tile_px
        blk = img[y0:y0 + tile_px, x0:x0 + tile_px]
        out[slot, :blk.shape[0], :blk.shape[1]] = blk
    return out


def untile(tiles: np.ndarray, ids, tile_px: int, img: np.ndarray) -> None:
    """Scatter packed tiles into img in place (rank-0 side of the gather)."""
    H, W = img.shape[:2]
    tx_n, _ = tile_grid(W, H, tile_px)
    for slot, t in enumerate(ids):
        tx, ty = t % tx_n, t // tx_n
        y0, x0 = ty * tile_px, tx * tile_px
        h, w = min(tile_px, H - y0), min(tile_px, W - x0)
        img[y0:y0 + h, x0:x0 + w] = tiles[slot, :h, :w]


def gather_frame(dist, packed, rank: int, world_size: int, dst: int = 0):
    """Gather every rank's packed tile buffer (same padded size on all ranks)
    to rank `dst`; returns the list of buffers there, None elsewhere."""
    if world_size == 1:
        return [packed]
    lst = [packed.new_empty(packed.shape) for _ in range(world_size)] if rank == dst else None
    dist.gather(packed, lst, dst=dst)
    return lst

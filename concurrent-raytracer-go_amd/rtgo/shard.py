"""Tile sharding across ranks: layout and gather protocol.

Tiles are the reference's 32x32 row-major tiles (createRenderTasks,
internal/renderer/renderer.go:398-436); tile t belongs to rank t % world.
Each rank renders its tiles into one PACKED SHARE (rt_context_render_async
with RT_LAYOUT_PACKED_TILES):

    [max_local * 1024 float3 linear][max_local * 1024 RGBA8]   (16 B / pixel)

local tile lt = t // world occupies slots [lt*1024, lt*1024+1024), pixel
(x, y) of the tile at slot lt*1024 + y*32 + x.  Every share is sized for
max_local = tiles_for_rank(w, h, 0, world) tiles (rank 0 owns the most), so
ONE equal-size gather collects them all (rt_comm_gather_tiles_async: RCCL
send/recv over xGMI; rank 0 renders its own share in place).  Rank 0 then
scatters the slots into the image (rt_unpack_tiles_async on the GPU;
`unpack_shares_host` is the same mapping for host buffers and tests).  The
RGBA8 bytes travel with the linear values because the kernel tone-maps the
binary64 mean: re-deriving them from the float32 copy would change a few
bytes (a truncation boundary crossed by the float rounding).
No other data-path collective: the ranks' work is independent, and the
random stream is keyed by global pixel and sample, so the assembled image is
bit-identical to a 1-rank render.
"""
from __future__ import annotations

import numpy as np

from . import max_local_tiles, num_tiles, packed_bytes, packed_rgba_offset


def rank_tiles(width: int, height: int, rank: int, world: int, owner=None) -> list:
    """The tiles of `rank` in local-tile order: t % world == rank, or, with a
    partition's owner array (owner[t] = rank of tile t), its tiles ascending."""
    if owner is None:
        return list(range(rank, num_tiles(width, height), world))
    return [t for t in range(num_tiles(width, height)) if owner[t] == rank]


def packed_index(width: int, height: int, rank: int, world: int, owner=None) -> np.ndarray:
    """Image pixel index (y*W + x) of every packed slot of `rank`, -1 where
    the slot is padding (a missing tile or a clipped edge pixel)."""
    if owner is None:
        ml = max_local_tiles(width, height, world)
    else:
        ml = max(len(rank_tiles(width, height, r, world, owner)) for r in range(world))
    idx = np.full(ml * 1024, -1, np.int64)
    tiles_x = (width + 31) // 32
    p = np.arange(1024)
    px, py = p % 32, p // 32
    for lt, t in enumerate(rank_tiles(width, height, rank, world, owner)):
        x = (t % tiles_x) * 32 + px
        y = (t // tiles_x) * 32 + py
        ok = (x < width) & (y < height)
        idx[lt * 1024 + p[ok]] = y[ok] * width + x[ok]
    return idx


def pack_share_host(lin: np.ndarray, rgba: np.ndarray, rank: int, world: int) -> np.ndarray:
    """The packed share of `rank` (uint8, packed_bytes long) from an (H, W, 3)
    float32 image and its (H, W, 4) RGBA8 image; padding slots are 0."""
    h, w, _ = lin.shape
    idx = packed_index(w, h, rank, world)
    ok = idx >= 0
    out = np.zeros(packed_bytes(w, h, world), np.uint8)
    off = packed_rgba_offset(w, h, world)
    pl = out[:off].view(np.float32).reshape(-1, 3)
    pr = out[off:].reshape(-1, 4)
    pl[ok] = lin.reshape(h * w, 3)[idx[ok]]
    pr[ok] = rgba.reshape(h * w, 4)[idx[ok]]
    return out


def unpack_shares_host(gathered: np.ndarray, width: int, height: int, world: int, owner=None):
    """(world * packed_bytes,) uint8 gathered shares -> ((H, W, 3) f32, (H, W, 4) u8)."""
    if owner is None:
        share = packed_bytes(width, height, world)
        off = packed_rgba_offset(width, height, world)
    else:
        ml = max(len(rank_tiles(width, height, r, world, owner)) for r in range(world))
        share, off = ml * 1024 * 16, ml * 1024 * 12
    lin = np.zeros((height * width, 3), np.float32)
    rgba = np.zeros((height * width, 4), np.uint8)
    for r in range(world):
        part = gathered[r * share:(r + 1) * share]
        idx = packed_index(width, height, r, world, owner)
        ok = idx >= 0
        lin[idx[ok]] = part[:off].view(np.float32).reshape(-1, 3)[ok]
        rgba[idx[ok]] = part[off:].reshape(-1, 4)[ok]
    return lin.reshape(height, width, 3), rgba.reshape(height, width, 4)


def gather_packed(dist, local, world: int, rank: int, out=None):
    """Equal-size gather of every rank's share into `out` (a (world * n,)
    tensor on rank 0; None elsewhere) through torch.distributed.  The GPU
    path uses rt_comm_gather_tiles_async instead; this is the same protocol
    for the gloo (CPU) tests of the multi-process orchestration."""
    if world == 1:
        return local
    if rank == 0:
        parts = list(out.chunk(world))
        dist.gather(local, parts, dst=0)
        return out
    dist.gather(local, None, dst=0)
    return None

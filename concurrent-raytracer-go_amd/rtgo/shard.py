"""Tile sharding across ranks: layout and gather protocol.

Tiles are the reference's 32x32 row-major tiles (createRenderTasks,
internal/renderer/renderer.go:398-436); tile t belongs to rank t % world.
Each rank renders its tiles into a PACKED buffer (rt_context_render_async
with RT_LAYOUT_PACKED_TILES): local tile lt = t // world occupies slots
[lt*1024, lt*1024+1024), pixel (x, y) of the tile at slot lt*1024 + y*32 + x.
Every rank's buffer is sized for max_local = tiles_for_rank(w, h, 0, world)
tiles (rank 0 owns the most), so one equal-count gather collects them all;
rank 0 then scatters the slots into the image (rt_unpack_tiles_async on the
GPU; `unpack_host` is the same mapping for host buffers and tests).
No data-path collective other than that single gather: the ranks' work is
independent, and the stream is keyed by global pixel and sample, so the
assembled image is bit-identical to a 1-rank render.
"""
from __future__ import annotations

import numpy as np

from . import num_tiles, tiles_for_rank


def max_local_tiles(width: int, height: int, world: int) -> int:
    return tiles_for_rank(width, height, 0, world)


def packed_index(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Image pixel index (y*W + x) of every packed slot of `rank`, -1 where
    the slot is padding (a missing tile or a clipped edge pixel)."""
    ml = max_local_tiles(width, height, world)
    idx = np.full(ml * 1024, -1, np.int64)
    tiles_x = (width + 31) // 32
    p = np.arange(1024)
    px, py = p % 32, p // 32
    for lt, t in enumerate(range(rank, num_tiles(width, height), world)):
        x = (t % tiles_x) * 32 + px
        y = (t // tiles_x) * 32 + py
        ok = (x < width) & (y < height)
        idx[lt * 1024 + p[ok]] = y[ok] * width + x[ok]
    return idx


def pack_host(image: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Packed slots of `rank` from an (H, W, C) image (padding = 0)."""
    h, w, c = image.shape
    idx = packed_index(w, h, rank, world)
    flat = image.reshape(h * w, c)
    out = np.zeros((len(idx), c), image.dtype)
    out[idx >= 0] = flat[idx[idx >= 0]]
    return out


def unpack_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """(world * max_local * 1024, C) gathered slots -> (H, W, C) image."""
    c = gathered.shape[-1]
    ml = max_local_tiles(width, height, world)
    img = np.zeros((height * width, c), gathered.dtype)
    for r in range(world):
        idx = packed_index(width, height, r, world)
        part = gathered[r * ml * 1024:(r + 1) * ml * 1024]
        img[idx[idx >= 0]] = part[idx >= 0]
    return img.reshape(height, width, c)


def gather_packed(dist, local, world: int, rank: int, out=None):
    """The one collective: equal-size gather of every rank's packed buffer
    into `out` (a (world * n,) tensor on rank 0; None elsewhere).  Works
    on any backend (RCCL on the GPU, gloo on the CPU tests)."""
    if world == 1:
        return local
    if rank == 0:
        parts = list(out.chunk(world))
        dist.gather(local, parts, dst=0)
        return out
    dist.gather(local, None, dst=0)
    return None

"""Helpers of the GPU tests: render through one rt_context (the C ABI), as an
image or as one rank's packed share, and reassemble shares on the GPU."""
import numpy as np

import rtgo


def render_dev(scene, w, h, st, rank=0, world=1, tuning=None, force_bvh=0, count=False, partition=None):
    """Render on device 0 through a fresh rt_context.

    world == 1: the W*H image.  world > 1: the packed share of `rank`
    (rt_packed_bytes: float3 slots, then RGBA8 slots; unused slots NaN / 0).
    Returns (linear (N, 3) float32, rgba (N, 4) uint8, share bytes or None,
    counts or None); N = W*H or max_local_tiles * 1024.  partition: an
    rtgo.Partition (world > 1): the share holds its tiles of `rank`.
    count == "full": the counts as an rtgo.Counts (culled / soft parts too).
    """
    import torch

    ctx = rtgo.Context(0)
    if tuning is not None:
        ctx.set_tuning(tuning)
    ctx.set_scene(scene, force_bvh=force_bvh)
    if partition is not None:
        ctx.set_partition(partition)
    if world > 1:
        nb = partition.packed_bytes if partition is not None else rtgo.packed_bytes(w, h, world)
        off = partition.rgba_offset if partition is not None else rtgo.packed_rgba_offset(w, h, world)
        share = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        share[:off].view(torch.float32).fill_(float("nan"))
        p_lin, p_rgba = share.data_ptr(), share.data_ptr() + off
        layout = rtgo.RT_LAYOUT_PACKED_TILES
    else:
        lin = torch.full((w * h * 3,), float("nan"), dtype=torch.float32, device="cuda")
        rgba = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
        p_lin, p_rgba = lin.data_ptr(), rgba.data_ptr()
        layout = rtgo.RT_LAYOUT_IMAGE
    counts = None
    if count:
        counts = ctx.count(w, h, st, p_lin, p_rgba, 0, rank, world, layout, full=(count == "full"))
    else:
        ctx.render_async(w, h, st, p_lin, p_rgba, 0, rank, world, layout)
    torch.cuda.synchronize()
    ctx.close()
    if world > 1:
        b = share.cpu().numpy()
        return b[:off].view(np.float32).reshape(-1, 3), b[off:].reshape(-1, 4), b, counts
    return lin.cpu().numpy().reshape(-1, 3), rgba.cpu().numpy().reshape(-1, 4), None, counts


def unpack_dev(w, h, world, shares, partition=None):
    """Gathered shares (list of uint8 arrays, rank order) -> (H,W,3) f32, (H,W,4) u8
    through rt_unpack_tiles_async (rt_unpack_partition_async with a partition)."""
    import torch

    g = torch.from_numpy(np.concatenate(shares)).cuda()
    lin = torch.full((h * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
    rgba = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda")
    if partition is not None:
        partition.unpack_async(g.data_ptr(), lin.data_ptr(), rgba.data_ptr(), 0)
    else:
        rtgo.unpack_tiles_async(w, h, world, g.data_ptr(), lin.data_ptr(), rgba.data_ptr(), 0)
    torch.cuda.synchronize()
    return lin.cpu().numpy().reshape(h, w, 3), rgba.cpu().numpy().reshape(h, w, 4)

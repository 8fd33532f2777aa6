"""librtgo in a multi-process run on the one GPU of the box (world_size 2).

The bench's N>1 model is one process per GPU (torch.distributed.run): each
process renders only its tiles (t % world == rank) through
its own rt_context into a packed share, and the shares meet on rank 0.  On
a one-GPU box both processes share device 0, where RCCL refuses two ranks
of one communicator, so the shares travel over gloo (host copies) with the
same packed layout and the same unpack kernel on rank 0.  Rank 0 must
obtain exactly the 1-rank image of librtgo, and the oracle's."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

W, H, SPP = 150, 100, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import sys

    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rtgo
        from rtgo import shard
        from scene_cases import load_case, make_settings

        torch.cuda.set_device(0)
        scene = load_case(rtgo, ("json", None))
        st = make_settings(rtgo, {"samples": SPP}, seed=4)
        nb = rtgo.packed_bytes(W, H, world)
        share = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        ctx = rtgo.Context(0)
        ctx.set_scene(scene)
        ctx.render_async(W, H, st, share.data_ptr(), share.data_ptr() + rtgo.packed_rgba_offset(W, H, world), 0,
                         rank, world, rtgo.RT_LAYOUT_PACKED_TILES)
        torch.cuda.synchronize()
        ctx.close()
        g = torch.empty(world * nb, dtype=torch.uint8) if rank == 0 else None
        g = shard.gather_packed(dist, share.cpu(), world, rank, g)
        if rank == 0:
            gd = g.to("cuda")
            lin = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
            rgba = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
            rtgo.unpack_tiles_async(W, H, world, gd.data_ptr(), lin.data_ptr(), rgba.data_ptr(), 0)
            torch.cuda.synchronize()
            np.savez(os.path.join(outdir, "r0.npz"), lin=lin.cpu().numpy(), rgba=rgba.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_two_processes_render_their_shares_like_one():
    import tempfile

    import oracle
    import rtgo
    from gpu_util import render_dev
    from scene_cases import load_case, make_settings

    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        got = dict(np.load(os.path.join(tmp, "r0.npz")))
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": SPP}, seed=4)
    one_lin, one_rgba, _, _ = render_dev(scene, W, H, st)
    assert got["lin"].tobytes() == one_lin.tobytes()
    assert got["rgba"].tobytes() == one_rgba.tobytes()
    ref_lin, ref_rgba, _ = oracle.render(scene, W, H, st)
    assert got["lin"].tobytes() == ref_lin.astype(np.float32).tobytes()
    assert got["rgba"].tobytes() == ref_rgba.tobytes()

"""N>1 path on the CPU: world_size 2 (and 3) over gloo.

Each rank renders only its tiles (t % world == rank) with the
oracle, packs them in the packed-tile layout, and the ranks run the same
single gather bench.py uses on RCCL (rtgo.shard.gather_packed).  Rank 0
unpacks and must obtain exactly the 1-rank image: the stream is keyed by
global pixel and sample, never by rank or tile."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

W, H, SPP = 75, 41, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import sys

    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        import rtgo
        from rtgo import shard
        from scene_cases import load_case, make_settings

        scene = load_case(rtgo, ("json", None))
        st = make_settings(rtgo, {"samples": SPP}, seed=5)
        lin, rgba, counts = oracle.render(scene, W, H, st, rank=rank, world=world, nthreads=2, counts=True)
        lin32 = lin.astype(np.float32)
        p_lin = torch.from_numpy(np.ascontiguousarray(shard.pack_host(np.nan_to_num(lin32, nan=0.0), rank,
                                                                      world)).ravel())
        p_rgba = torch.from_numpy(np.ascontiguousarray(shard.pack_host(rgba, rank, world)).ravel())
        n = shard.max_local_tiles(W, H, world) * 1024
        g_lin = torch.empty(world * n * 3, dtype=torch.float32) if rank == 0 else None
        g_rgba = torch.empty(world * n * 4, dtype=torch.uint8) if rank == 0 else None
        g_lin = shard.gather_packed(dist, p_lin, world, rank, g_lin)
        g_rgba = shard.gather_packed(dist, p_rgba, world, rank, g_rgba)
        # per-rank work sums to the whole frame (weak-scaling accounting in bench.py)
        cam = torch.tensor([counts["camera_rays"]], dtype=torch.int64)
        dist.all_reduce(cam)
        if rank == 0:
            img = shard.unpack_host(g_lin.numpy().reshape(-1, 3), W, H, world)
            img_rgba = shard.unpack_host(g_rgba.numpy().reshape(-1, 4), W, H, world)
            np.savez(os.path.join(outdir, "r0.npz"), lin=img, rgba=img_rgba, cam=cam.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_reassembles_the_1_rank_image(world, tmp_path):
    import oracle
    import rtgo
    from scene_cases import load_case, make_settings

    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(os.path.join(tmp_path, "r0.npz"))
    scene = load_case(rtgo, ("json", None))
    lin, rgba, _ = oracle.render(scene, W, H, make_settings(rtgo, {"samples": SPP}, seed=5))
    assert got["lin"].tobytes() == lin.astype(np.float32).tobytes()
    assert got["rgba"].tobytes() == rgba.tobytes()
    assert int(got["cam"][0]) == W * H * SPP


def test_packed_index_covers_every_pixel_once():
    from rtgo import shard

    for w, h in ((75, 41), (800, 600), (33, 1)):
        for world in (1, 2, 3, 8):
            seen = np.concatenate([shard.packed_index(w, h, r, world) for r in range(world)])
            seen = seen[seen >= 0]
            assert len(seen) == w * h and np.array_equal(np.sort(seen), np.arange(w * h))


def test_pack_unpack_roundtrip():
    from rtgo import shard

    img = np.random.default_rng(0).random((41, 75, 3)).astype(np.float32)
    for world in (1, 2, 5):
        g = np.concatenate([shard.pack_host(img, r, world) for r in range(world)])
        assert np.array_equal(shard.unpack_host(g, 75, 41, world), img)

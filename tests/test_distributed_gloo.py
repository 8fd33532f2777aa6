"""N>1 path on the CPU: world_size 2 (and 3) over gloo.

Each rank renders only its tiles (t % world == rank) with the
oracle, packs them in the packed-tile layout, and the ranks run the same
single equal-size gather of packed shares that bench.py runs on RCCL
(rt_comm_gather_tiles_async; here rtgo.shard.gather_packed over gloo).  Rank 0
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
        lin32 = np.nan_to_num(lin.astype(np.float32), nan=0.0)
        share = torch.from_numpy(shard.pack_share_host(lin32, rgba, rank, world))
        nb = rtgo.packed_bytes(W, H, world)
        g = torch.empty(world * nb, dtype=torch.uint8) if rank == 0 else None
        g = shard.gather_packed(dist, share, world, rank, g)
        # per-rank work sums to the whole frame (bench.py's value: all ranks' rays / the slowest rank's time)
        cam = torch.tensor([counts["camera_rays"]], dtype=torch.int64)
        dist.all_reduce(cam)
        if rank == 0:
            img, img_rgba = shard.unpack_shares_host(g.numpy(), W, H, world)
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

    rng = np.random.default_rng(0)
    img = rng.random((41, 75, 3)).astype(np.float32)
    rgba = rng.integers(0, 256, (41, 75, 4), dtype=np.uint8)
    for world in (1, 2, 5):
        g = np.concatenate([shard.pack_share_host(img, rgba, r, world) for r in range(world)])
        lin2, rgba2 = shard.unpack_shares_host(g, 75, 41, world)
        assert np.array_equal(lin2, img) and np.array_equal(rgba2, rgba)

"""GPU: tail helpers do not change a single bit.

A block whose entries have all started hands its last few long paths to
helper workgroups at the end of the launch (rt_tuning.tail_*); each path's
radiance then reaches its pixel through a per-sample row (or the split row of
a split pixel) that the pixel's last contributor sums in sample order.  The
images must equal the oracle's (and the renders without helpers) bit for bit,
with the export forced to happen often (every path of a draining block, from
its first bounce on), on blocks of several pixels, split pixels, triangles,
frames of one launch and packed tiles; and the paths must really have been
exported (rt_context_stats.tail_exported > 0, no helper error)."""
import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import load_case, make_settings

pytestmark = pytest.mark.gpu

# every path of a draining block, from its first bounce, checked every iteration
FORCED = {"tail_helpers": 256, "tail_paths": 64, "tail_depth": 1, "tail_every": 1}
ON = {"tail_helpers": 256}


def _render(scene, w, h, st, tun, frames=None, world=1, rank=0):
    """(linear, rgba, stats) of one context; frames: seeds of one batched launch."""
    import torch

    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning(**tun))
    ctx.set_scene(scene)
    if world > 1:
        nb, off = rtgo.packed_bytes(w, h, world), rtgo.packed_rgba_offset(w, h, world)
        share = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        ctx.render_async(w, h, st, share.data_ptr(), share.data_ptr() + off, 0, rank, world,
                         rtgo.RT_LAYOUT_PACKED_TILES)
        torch.cuda.synchronize()
        stats = ctx.stats()
        ctx.close()
        b = share.cpu().numpy()
        return b[:off].view(np.float32).reshape(-1, 3), b[off:].reshape(-1, 4), stats
    n = len(frames) if frames else 1
    lin = torch.full((n, w * h * 3), float("nan"), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((n, w * h * 4), dtype=torch.uint8, device="cuda")
    if frames:
        ctx.render_frames_async(w, h, st, list(frames), [lin[f].data_ptr() for f in range(n)],
                                [rgba[f].data_ptr() for f in range(n)], 0, 0, 1, rtgo.RT_LAYOUT_IMAGE)
    else:
        ctx.render_async(w, h, st, lin[0].data_ptr(), rgba[0].data_ptr(), 0)
    torch.cuda.synchronize()
    stats = ctx.stats()
    ctx.close()
    return lin.cpu().numpy().reshape(n, h, w, 3), rgba.cpu().numpy().reshape(n, h, w, 4), stats


def _same_as_oracle(scene, w, h, st, lin, rgba):
    ref, ref_rgba, _ = oracle.render(scene, w, h, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()


CASES = [
    ("spheres_facing", ("file", "sphere_reflections_light_facing.json"), 160, 120, {"samples": 40}),
    ("silver_facing", ("file", "final_silver_prism_purple_cube_facing.json"), 96, 72, {"samples": 24}),
    ("all_materials", ("json", None), 64, 48, {"samples": 30, "max_depth": 20}),
]


@pytest.mark.parametrize("name,loader,w,h,over", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("tun", [FORCED, ON, {"tail_helpers": -1}], ids=["forced", "on", "off"])
def test_tail_helpers_keep_the_oracle_image(name, loader, w, h, over, tun):
    scene = load_case(rtgo, loader)
    for seed in (1, 2):
        st = make_settings(rtgo, over, seed=seed)
        lin, rgba, stats = _render(scene, w, h, st, tun)
        _same_as_oracle(scene, w, h, st, lin[0], rgba[0])
        assert stats["tail_errors"] == 0
        if tun is FORCED:
            assert stats["tail_exported"] > 0, stats
        if tun.get("tail_helpers") == -1:
            assert stats["tail_exported"] == 0


@pytest.mark.parametrize("tun", [{"block_work": 1}, {"block_work": 64, "split_samples": 8}],
                         ids=["every_pixel_split", "split_by_8"])
def test_exports_from_split_pixels(tun):
    """Split pixels: an exported path's radiance goes to the split row and the
    sub-block counter owes one more finisher; the last one sums the row."""
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 130, "max_depth": 12}, seed=4)
    lin, rgba, stats = _render(scene, 40, 24, st, dict(tun, **FORCED))
    _same_as_oracle(scene, 40, 24, st, lin[0], rgba[0])
    assert stats["tail_exported"] > 0 and stats["tail_errors"] == 0


def test_exports_in_a_batched_launch_and_across_launches():
    """Several frames of one launch, then the same context again (its control
    block zeroed by the previous launch's last helper, its rows reused)."""
    scene = load_case(rtgo, ("file", "sphere_reflections_light_facing.json"))
    w, h = 128, 96
    st = make_settings(rtgo, {"samples": 24}, seed=1)
    seeds = [3, 4, 5, 6]
    lin, rgba, stats = _render(scene, w, h, st, FORCED, frames=seeds)
    assert stats["tail_exported"] > 0 and stats["tail_errors"] == 0
    for f, seed in enumerate(seeds):
        sf = make_settings(rtgo, {"samples": 24}, seed=seed)
        _same_as_oracle(scene, w, h, sf, lin[f], rgba[f])


def test_exports_into_packed_tiles():
    """A rank's packed share (RT_LAYOUT_PACKED_TILES): the row's output index
    is the packed slot."""
    scene = load_case(rtgo, ("file", "sphere_reflections_light_facing.json"))
    w, h, world = 96, 64, 3
    st = make_settings(rtgo, {"samples": 30}, seed=2)
    shares = []
    for rank in range(world):
        lin, rgba, stats = _render(scene, w, h, st, FORCED, world=world, rank=rank)
        assert stats["tail_errors"] == 0
        ref_lin, ref_rgba, _ = _render(scene, w, h, st, {"tail_helpers": -1}, world=world, rank=rank)
        assert lin.tobytes() == ref_lin.tobytes() and rgba.tobytes() == ref_rgba.tobytes(), rank
        shares.append(stats["tail_exported"])
    assert sum(shares) > 0


def test_headline_frame_with_helpers():
    """BASELINE configs[1] (800x600x100, depth 50) with 256 helpers:
    the oracle's frame, and paths were exported."""
    scene = load_case(rtgo, ("file", "sphere_reflections_light_facing.json"))
    st = make_settings(rtgo, {}, seed=7)
    lin, rgba, stats = _render(scene, 800, 600, st, ON)
    _same_as_oracle(scene, 800, 600, st, lin[0], rgba[0])
    assert stats["tail_exported"] > 0 and stats["tail_errors"] == 0

"""GPU: tile partitions across ranks, the counting variant's culled share,
per-kernel timing, and the advisor's round-2 edge cases.

* A work-balanced partition (rt_partition_balanced: every tile's work
  measured by one whole-frame render, tiles dealt heaviest first to the
  least loaded rank) of the headline frame
  (BASELINE configs[1]: sphere_reflections_light facing, 800x600x100, depth 50)
  over 8 ranks, rendered rank by rank on device 0 and unpacked, equals the
  1-rank image bit for bit; so does rt_renderer with 8 ranks on device 0
  (whose default partition for a linear-scan scene is the balanced one).
  The reference deals tiles through one channel to NumCPU goroutines
  (renderer.go:398-436); every pixel stays on one rank here, and the random
  stream is keyed by global pixel and sample, so the partition cannot change
  a bit.
* The partition is a pure function of the frame: two contexts plan the same.
* More ranks than tiles, after a larger frame on the same context / renderer.
* Counts with an opted-in sky leave the image unchanged.
* rt_counts.culled: the camera samples the product skips.
* rt_context_profile: per-kernel HIP-event times of the wavefront loop.
"""
import numpy as np
import pytest

import rtgo
from gpu_util import render_dev, unpack_dev
from rtgo import shard
from scene_cases import load_case, make_settings, spheres10k_scene

pytestmark = pytest.mark.gpu

FACING = ("file", "sphere_reflections_light_facing.json")


def _gpu(scene, w, h, st, devices=None):
    r = rtgo.ParallelRenderer(devices=devices)
    if devices:
        st.num_devices = len(devices)
    r.settings = st
    rgba = r.render(scene, w, h)
    lin = r.last_linear.copy()
    secs = r.rank_seconds()
    r.close()
    return lin, rgba, secs


def test_balanced_partition_of_the_headline_frame_over_8_ranks():
    scene = load_case(rtgo, FACING)
    st = make_settings(rtgo, {"samples": 100, "max_depth": 50}, seed=5)
    w, h, world = 800, 600, 8
    ref_lin, ref_rgba, _ = _gpu(scene, w, h, st)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    part = ctx.balanced_partition(w, h, st, world)
    ctx2 = rtgo.Context(0)
    ctx2.set_scene(scene)
    again = ctx2.balanced_partition(w, h, st, world)
    ctx.close()
    ctx2.close()
    owners = part.owners(w, h)
    # deterministic: every rank plans the same partition from the same frame
    assert np.array_equal(owners, again.owners(w, h))
    assert sorted(set(owners.tolist())) == list(range(world))
    work = [part.work(r) for r in range(world)]
    spread = max(work) / (sum(work) / world)
    print(f"estimated work per rank {[round(x) for x in work]}; max/mean {spread:.3f}")
    assert spread < 1.25  # the strided deal t % 8 gives ~1.7 on this frame
    shares = [render_dev(scene, w, h, st, rank=r, world=world, partition=part)[2] for r in range(world)]
    img_lin, img_rgba = unpack_dev(w, h, world, shares, partition=part)
    assert img_lin.tobytes() == ref_lin.tobytes()
    assert img_rgba.tobytes() == ref_rgba.tobytes()
    # the packed layout is rtgo.shard's with the partition's owner array
    lin_h, rgba_h = shard.unpack_shares_host(np.concatenate(shares), w, h, world, owner=owners)
    assert rgba_h.tobytes() == ref_rgba.tobytes()
    # the C ABI's renderer: 8 ranks on device 0, balanced by default
    r_lin, r_rgba, secs = _gpu(scene, w, h, make_settings(rtgo, {"samples": 100, "max_depth": 50}, seed=5),
                               devices=[0] * world)
    assert r_lin.tobytes() == ref_lin.tobytes()
    assert r_rgba.tobytes() == ref_rgba.tobytes()
    assert len(secs) == world and all(s > 0 for s in secs)
    print("rank kernel seconds", [round(s * 1e3, 3) for s in secs])


@pytest.mark.parametrize("mode", [rtgo.RT_PARTITION_STRIDED, rtgo.RT_PARTITION_BALANCED])
def test_renderer_partition_modes_on_a_bvh_scene(mode):
    """The 10k-sphere scene (wavefront path) with 3 ranks on device 0, dealt
    strided (the default for BVH scenes) or balanced: the 1-rank image."""
    scene = spheres10k_scene(rtgo)
    w, h = 96, 64
    st = make_settings(rtgo, {"samples": 2, "max_depth": 6}, seed=7)
    ref_lin, ref_rgba, _ = _gpu(scene, w, h, st)
    r = rtgo.ParallelRenderer(devices=[0, 0, 0])
    r.set_tuning(rtgo.default_tuning(partition=mode))
    st.num_devices = 3
    r.settings = st
    rgba = r.render(scene, w, h)
    assert r.last_linear.tobytes() == ref_lin.tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()
    r.close()


def test_explicit_partition_of_every_tile_to_one_rank():
    """rt_partition_create with an owner array: ranks with no tiles render
    nothing, and the shares still reassemble the image."""
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3})
    w, h, world = 75, 50, 4
    ref_lin, ref_rgba, _ = _gpu(scene, w, h, st)
    nt = rtgo.num_tiles(w, h)
    owner = [2 if t % 3 else 0 for t in range(nt)]  # ranks 1 and 3 own nothing
    part = rtgo.Partition(w, h, world, owner)
    assert part.local_tiles(1) == 0 and part.local_tiles(3) == 0
    assert part.tiles(0) == [t for t in range(nt) if owner[t] == 0]
    shares = [render_dev(scene, w, h, st, rank=r, world=world, partition=part)[2] for r in range(world)]
    img_lin, img_rgba = unpack_dev(w, h, world, shares, partition=part)
    assert img_lin.tobytes() == ref_lin.tobytes()
    assert img_rgba.tobytes() == ref_rgba.tobytes()


def test_more_ranks_than_tiles_after_a_larger_frame():
    """a rank with no tiles must render nothing, also when
    its context built a larger schedule before (stale scheduler scratch)."""
    import torch

    scene = load_case(rtgo, FACING)
    st = make_settings(rtgo, {"samples": 4}, seed=2)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    big = torch.zeros(800 * 600 * 4, dtype=torch.float32, device="cuda")
    ctx.render_async(800, 600, st, big.data_ptr(), 0)  # a large schedule first
    torch.cuda.synchronize()
    w, h, world = 40, 30, 8  # one tile, eight ranks
    nb = rtgo.packed_bytes(w, h, world)
    share = torch.full((nb,), 7, dtype=torch.uint8, device="cuda")
    ctx.render_async(w, h, st, share.data_ptr(), share.data_ptr() + rtgo.packed_rgba_offset(w, h, world), 0,
                     rank=5, world=world, layout=rtgo.RT_LAYOUT_PACKED_TILES)
    torch.cuda.synchronize()
    assert rtgo.tiles_for_rank(w, h, 5, world) == 0
    assert bool((share == 7).all())  # nothing written
    ctx.close()
    ref_lin, ref_rgba, _ = _gpu(scene, w, h, make_settings(rtgo, {"samples": 4}, seed=2))
    r = rtgo.ParallelRenderer(devices=[0] * world)
    for ww, hh in ((320, 240), (w, h)):
        s2 = make_settings(rtgo, {"samples": 4}, seed=2)
        s2.num_devices = world
        r.settings = s2
        rgba = r.render(scene, ww, hh)
    assert r.last_linear.tobytes() == ref_lin.tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()
    r.close()


def test_counts_with_an_opted_in_sky_keep_the_image():
    """the counting render with a sky returns the sky
    image, not black misses."""
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3})
    st.sky = rtgo.SKIES["sunset"]
    plain = render_dev(scene, 64, 48, st)
    counted = render_dev(scene, 64, 48, st, count="full")
    assert counted[0].tobytes() == plain[0].tobytes()
    assert counted[1].tobytes() == plain[1].tobytes()
    c = counted[3]
    assert c.camera_rays == 64 * 48 * 3
    # a sky culls no camera sample; the culled work is the shadow rays the
    # product does not trace (empty shadow cones, inert lights), their sphere
    # tests and their soft-shadow draws (spec v4: not drawn by the product)
    cull = c.culled_dict()
    assert cull["camera_rays"] == cull["bounce_rays"] == cull["shade_events"] == cull["light_evals"] == 0
    assert cull["rng_draws"] % 3 == 0 and cull["shadow_rays"] <= c.shadow_rays


def test_culled_counts_are_the_skipped_camera_samples():
    scene = load_case(rtgo, FACING)
    st = make_settings(rtgo, {"samples": 10})
    c = render_dev(scene, 160, 120, st, count="full")[3]
    cull, ex = c.culled_dict(), c.executed_dict()
    assert c.camera_rays == 160 * 120 * 10
    assert 0 < cull["camera_rays"] < c.camera_rays
    # a culled sample draws its jitter only; the rest of the culled draws are
    # the rejection tries (3 draws each) of soft rays that cannot be blocked,
    # which the product does not draw (spec v4, include/rt_rng.h)
    extra = cull["rng_draws"] - 2 * cull["camera_rays"]
    assert extra >= 0 and extra % 3 == 0
    assert cull["shade_events"] == cull["light_evals"] == 0  # culled samples miss
    # (shadow rays the product does not trace: empty cones, inert lights)
    assert 0 < cull["shadow_rays"] < c.shadow_rays
    assert ex["shade_events"] == c.shade_events
    # the as-committed scene: every camera ray misses, every sample is culled
    black = render_dev(load_case(rtgo, ("file", "sphere_reflections_light.json")), 64, 48,
                       make_settings(rtgo, {"samples": 4}), count="full")[3]
    assert black.culled_dict()["camera_rays"] == black.camera_rays == 64 * 48 * 4


def test_wavefront_kernel_profile():
    """rt_context_profile: HIP events at every kernel boundary of the bounce
    loop; the soft-shadow traversal's own counts (rt_counts.soft_occlusion)."""
    import torch

    scene = spheres10k_scene(rtgo)
    st = make_settings(rtgo, {"samples": 4, "max_depth": 8})
    w, h = 128, 72
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    lin = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    ctx.profile(True)
    for seed in (1, 2):
        st.seed = seed
        ctx.render_async(w, h, st, lin.data_ptr(), 0)
    ks = ctx.kernel_seconds()
    assert ks["extend"][0] > 0 and ks["occlude_soft"][0] > 0 and ks["resolve"][1] == 2
    assert ks["extend"][1] == ks["occlude_soft"][1] == ks["shade"][1] > 2
    c = ctx.count(w, h, st, lin.data_ptr(), 0, full=True)
    soft = c.soft_occlusion_dict()
    assert 0 < soft["box_tests"] < c.box_tests and 0 < soft["sphere_tests"] < c.sphere_tests
    assert soft["camera_rays"] == 0 and soft["rng_draws"] == 0
    ctx.profile(False)
    ctx.close()


@pytest.mark.parametrize("tuning", [{}, {"split_samples": 16, "block_work": 64.0}], ids=["default", "many_splits"])
def test_frames_of_one_launch_equal_single_renders(tuning):
    """rt_context_render_frames_async: 6 frames (seeds 11..16) of the headline
    frame in one launch, each bit-identical to its own single render (split
    pixels included: a copy of their rows per frame); then the packed shares
    of 3 ranks of a balanced partition, 4 frames per launch, gathered as
    [rank][frame][share] and unpacked in one launch.  With the default tuning
    the launch of 6 frames is cut into larger blocks than a single render's
    (1024 vs 384 bounce-samples, rt_api.cpp default_block_work), so this also
    checks that the image does not depend on the schedule."""
    import torch

    scene = load_case(rtgo, FACING)
    w, h, spp = 800, 600, 100
    tn = rtgo.default_tuning(**tuning)
    st = make_settings(rtgo, {"samples": spp, "max_depth": 50}, seed=1)
    seeds = list(range(11, 17))
    ctx = rtgo.Context(0)
    ctx.set_tuning(tn)
    ctx.set_scene(scene)
    lin = torch.zeros((len(seeds), w * h * 3), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((len(seeds), w * h * 4), dtype=torch.uint8, device="cuda")
    ctx.render_frames_async(w, h, st, seeds, [lin[f].data_ptr() for f in range(len(seeds))],
                            [rgba[f].data_ptr() for f in range(len(seeds))])
    torch.cuda.synchronize()
    for f, sd in enumerate(seeds):
        ref_lin, ref_rgba, _, _ = render_dev(scene, w, h, make_settings(rtgo, {"samples": spp, "max_depth": 50},
                                                                        seed=sd), tuning=tn)
        assert lin[f].cpu().numpy().tobytes() == ref_lin.tobytes(), f
        assert rgba[f].cpu().numpy().tobytes() == ref_rgba.tobytes(), f
    # packed shares of a balanced partition, frames batched per rank
    world, nf = 3, 4
    part = ctx.balanced_partition(w, h, st, world)
    ctx.close()
    nb = part.packed_bytes
    g = torch.zeros(world * nf * nb, dtype=torch.uint8, device="cuda")
    for r in range(world):
        c = rtgo.Context(0)
        c.set_tuning(tn)
        c.set_scene(scene)
        c.set_partition(part)
        base = g.data_ptr() + r * nf * nb
        lp = [base + f * nb for f in range(nf)]
        c.render_frames_async(w, h, st, seeds[:nf], lp, [p + part.rgba_offset for p in lp], 0, r, world,
                              rtgo.RT_LAYOUT_PACKED_TILES)
        torch.cuda.synchronize()
        c.close()
    img_lin = torch.zeros(nf * w * h * 3, dtype=torch.float32, device="cuda")
    img_rgba = torch.zeros(nf * w * h * 4, dtype=torch.uint8, device="cuda")
    part.unpack_frames_async(nf, g.data_ptr(), img_lin.data_ptr(), img_rgba.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(img_lin.view(nf, -1), lin[:nf]) and torch.equal(img_rgba.view(nf, -1), rgba[:nf])


def test_batched_triangle_frames_equal_single_renders():
    """The silver prism / purple cube scene (BASELINE C3: triangles, the
    batched schedule cuts 2048 bounce-samples per block against 256 for one
    frame, rt_api.cpp default_block_work): 3 frames of one launch, each
    bit-identical to its own single render, whose parity with the oracle the
    full-size tests pin."""
    import torch

    scene = load_case(rtgo, ("file", "final_silver_prism_purple_cube_facing.json"))
    w, h, spp = 600, 450, 32
    st = make_settings(rtgo, {"samples": spp, "max_depth": 50}, seed=1)
    seeds = [21, 22, 23]
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    lin = torch.zeros((len(seeds), w * h * 3), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((len(seeds), w * h * 4), dtype=torch.uint8, device="cuda")
    ctx.render_frames_async(w, h, st, seeds, [lin[f].data_ptr() for f in range(len(seeds))],
                            [rgba[f].data_ptr() for f in range(len(seeds))])
    torch.cuda.synchronize()
    ctx.close()
    for f, sd in enumerate(seeds):
        ref_lin, ref_rgba, _, _ = render_dev(scene, w, h, make_settings(rtgo, {"samples": spp, "max_depth": 50},
                                                                        seed=sd))
        assert lin[f].cpu().numpy().tobytes() == ref_lin.tobytes(), f
        assert rgba[f].cpu().numpy().tobytes() == ref_rgba.tobytes(), f

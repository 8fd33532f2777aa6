"""GPU: the image does not depend on how the work is cut and ordered.

The host cuts a rank's tiles into work blocks from a one-sample pilot render
(rt_api.cpp prepare_schedule, schedule.cpp build_blocks): blocks of several
pixels, single pixels, and pixels SPLIT into sample ranges that the last
finishing range resolves.  Every schedule must give the oracle's image bit
for bit.  The rt_tuning settings below force each kind of block.
"""
import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import load_case, make_settings

pytestmark = pytest.mark.gpu

SCHEDULES = [
    ("default", {}),
    ("every_pixel_split", {"block_work": 1}),         # nearly every pixel split into sample ranges
    ("huge_blocks", {"block_work": 1e6}),            # the largest blocks everywhere
    ("small_blocks", {"block_samples": 100}),        # few samples per large block
    ("split_by_8", {"block_work": 64, "split_samples": 8}),  # heavy pixels in sub-blocks of <= 8 samples
    ("no_pilot", {"pilot": 0}),                      # geometric estimate only
    ("no_frustum_no_stage", {"frustum": 0, "stage": 0}),
]


@pytest.mark.parametrize("name,tun", SCHEDULES, ids=[s[0] for s in SCHEDULES])
@pytest.mark.parametrize("spp", [3, 40, 130])
def test_schedule_does_not_change_the_image(name, tun, spp):
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": spp, "max_depth": 12}, seed=4)
    w, h = (40, 24) if spp > 100 else (56, 40)
    r = rtgo.ParallelRenderer()
    r.settings = st
    r.set_tuning(rtgo.default_tuning(**tun))
    rgba = r.render(scene, w, h)
    lin = r.last_linear
    ref, ref_rgba, _ = oracle.render(scene, w, h, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes(), name
    assert rgba.tobytes() == ref_rgba.tobytes(), name


@pytest.mark.parametrize("tun", [{"measure": 1}, {"measure": 1, "split_depth": 4, "split_samples": 16}, {}],
                         ids=["measured", "measured_deep_split", "pilot_only"])
def test_measured_recut_does_not_change_the_image(tun):
    """The first frame of a schedule measures every pixel's paths and the
    second frame's blocks are cut from them (rt_tuning.measure): frames 1, 2
    and 3 of one renderer (pilot schedule, measuring frame, measured
    schedule) all equal the oracle."""
    scene = load_case(rtgo, ("file", "sphere_reflections_light_facing.json"))
    w, h = 96, 72
    r = rtgo.ParallelRenderer()
    r.set_tuning(rtgo.default_tuning(**tun))
    for seed in (5, 6, 5):
        st = make_settings(rtgo, {"samples": 24}, seed=seed)
        r.settings = st
        rgba = r.render(scene, w, h)
        ref, ref_rgba, _ = oracle.render(scene, w, h, st)
        assert r.last_linear.tobytes() == ref.astype(np.float32).tobytes(), seed
        assert rgba.tobytes() == ref_rgba.tobytes(), seed


def test_split_pixels_across_frames_of_one_renderer():
    """Split pixels keep per-launch hit bits and sub-block counters that the
    last sub-block of each pixel zeroes again for the next launch (no memset
    per frame, rt_kernel.hip).  Three frames of one renderer with the same
    schedule (seeds 4, 5, 4; nearly every pixel split) all equal the oracle."""
    scene = load_case(rtgo, ("json", None))
    w, h = 40, 24
    r = rtgo.ParallelRenderer()
    r.set_tuning(rtgo.default_tuning(block_work=1))
    for seed in (4, 5, 4):
        st = make_settings(rtgo, {"samples": 130, "max_depth": 12}, seed=seed)
        r.settings = st
        rgba = r.render(scene, w, h)
        ref, ref_rgba, _ = oracle.render(scene, w, h, st)
        assert r.last_linear.tobytes() == ref.astype(np.float32).tobytes(), seed
        assert rgba.tobytes() == ref_rgba.tobytes(), seed


@pytest.mark.parametrize("measure", [1, 0], ids=["measure", "pilot_only"])
def test_measured_schedule_reaches_batched_launches(measure):
    """rt_tuning.measure with batched frames (rt_context_render_frames_async):
    the first call renders frame by frame (its first frame measures, the next
    re-cuts) under the batched launch's own schedule key, so every later call
    is ONE launch on that schedule with no rebuild (the measuring
    frames used the one-frame key and the two keys rebuilt each other on
    every call, so batched launches never happened).  Every frame is the
    oracle's image."""
    import torch

    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 6, "max_depth": 12}, seed=1)
    w, h, nf = 64, 48, 4
    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning(measure=measure))
    ctx.set_scene(scene)
    lin = torch.zeros((nf, w * h * 3), dtype=torch.float32, device="cuda")
    rgba = torch.zeros((nf, w * h * 4), dtype=torch.uint8, device="cuda")
    seen = []
    for call in range(3):
        seeds = [1 + call * nf + f for f in range(nf)]
        ctx.render_frames_async(w, h, st, seeds, [lin[f].data_ptr() for f in range(nf)],
                                [rgba[f].data_ptr() for f in range(nf)], 0)
        torch.cuda.synchronize()
        seen.append(ctx.stats())
        st_f = make_settings(rtgo, {"samples": 6, "max_depth": 12}, seed=seeds[-1])
        ref, ref_rgba, _ = oracle.render(scene, w, h, st_f)
        assert lin[nf - 1].cpu().numpy().tobytes() == ref.astype(np.float32).tobytes(), (call, seen[-1])
        assert rgba[nf - 1].cpu().numpy().tobytes() == ref_rgba.tobytes(), call
    ctx.close()
    first, second, third = seen
    assert second["batched_launches"] == first["batched_launches"] + 1, seen
    assert third["batched_launches"] == second["batched_launches"] + 1, seen
    assert third["schedules_built"] == second["schedules_built"] == first["schedules_built"], seen
    assert third["frames"] == 3 * nf, seen
    if measure:
        assert first["measuring_frames"] == 1 and third["measuring_frames"] == 1, seen
        assert first["batched_launches"] == 0 and first["schedules_built"] == 2, seen  # pilot cut, measured re-cut
    else:
        assert first["batched_launches"] == 1 and first["schedules_built"] == 1, seen

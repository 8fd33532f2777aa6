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

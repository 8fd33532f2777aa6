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

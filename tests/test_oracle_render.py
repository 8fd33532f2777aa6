"""Whole-image behaviour of the CPU oracle (CPU only).

The oracle mirrors the reference's goroutine tile queue (renderer.go:67-148):
its image must not depend on the worker count or on how tiles are dealt to
ranks (the stream is keyed by global pixel and sample), and
it must reproduce the committed fixtures (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

import oracle
import rtgo
from conftest import GOLDEN
from scene_cases import GOLDEN_CASES, load_case, make_settings, scene_path


def same(a, b):
    return a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("case", GOLDEN_CASES, ids=[c[0] for c in GOLDEN_CASES])
def test_oracle_reproduces_committed_fixture(case):
    name, loader, w, h, over, seed = case
    g = np.load(os.path.join(GOLDEN, f"oracle_{name}.npz"))
    lin, rgba, counts = oracle.render(load_case(rtgo, loader), w, h, make_settings(rtgo, over, seed), counts=True)
    assert same(lin, g["linear"]) and same(rgba, g["rgba"])
    assert [counts[k] for k in rtgo.COUNT_FIELDS] == g["counts"].tolist()


def test_worker_count_does_not_change_the_image():
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3})
    a = oracle.render(scene, 70, 40, st, nthreads=1)
    b = oracle.render(scene, 70, 40, st, nthreads=7)
    assert same(a[0], b[0]) and same(a[1], b[1])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_sharding_reassembles_the_image(world):
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 2})
    w, h = 75, 50  # ragged edge tiles
    full_lin, full_rgba, _ = oracle.render(scene, w, h, st)
    lin = np.full_like(full_lin, np.nan)
    rgba = np.zeros_like(full_rgba)
    tiles_x = (w + 31) // 32
    for r in range(world):
        l_r, c_r, _ = oracle.render(scene, w, h, st, rank=r, world=world)
        for t in range(r, rtgo.num_tiles(w, h), world):
            ys = slice((t // tiles_x) * 32, min((t // tiles_x) * 32 + 32, h))
            xs = slice((t % tiles_x) * 32, min((t % tiles_x) * 32 + 32, w))
            assert np.all(np.isnan(lin[ys, xs]))  # each tile owned by exactly one rank
            lin[ys, xs] = l_r[ys, xs]
            rgba[ys, xs] = c_r[ys, xs]
    assert same(lin, full_lin) and same(rgba, full_rgba)


def test_as_committed_scene_renders_black():
    # every object sits behind the fixed -Z camera (renderer.go:377-390)
    scene = rtgo.Scene.load_from_file(scene_path("sphere_reflections_light.json"))
    lin, rgba, c = oracle.render(scene, 40, 30, make_settings(rtgo, {"samples": 2}), counts=True)
    assert np.all(lin == 0) and np.all(rgba[..., :3] == 0) and np.all(rgba[..., 3] == 255)
    assert c["camera_rays"] == 40 * 30 * 2 and c["shade_events"] == 0 and c["rng_draws"] == 2 * 40 * 30 * 2


def test_depth_zero_is_black_and_depth_one_has_no_bounces():
    scene = load_case(rtgo, ("json", None))
    lin, _, c = oracle.render(scene, 20, 10, make_settings(rtgo, {"samples": 2, "max_depth": 0}), counts=True)
    assert np.all(lin == 0) and c["bounce_rays"] == 0
    _, _, c1 = oracle.render(scene, 20, 10, make_settings(rtgo, {"samples": 2, "max_depth": 1}), counts=True)
    assert c1["bounce_rays"] == 20 * 10 * 2  # one closest-hit query per sample


def test_soft_shadow_switch_changes_draws_only_through_shadows():
    scene = load_case(rtgo, ("json", None))
    st_soft = make_settings(rtgo, {"samples": 2})
    st_hard = make_settings(rtgo, {"samples": 2, "soft_shadows": 0})
    _, _, cs = oracle.render(scene, 24, 16, st_soft, counts=True)
    _, _, ch = oracle.render(scene, 24, 16, st_hard, counts=True)
    assert cs["camera_rays"] == ch["camera_rays"]
    assert ch["shadow_rays"] == ch["light_evals"]  # one hard ray per light evaluation
    assert cs["shadow_rays"] > ch["shadow_rays"]


def test_seed_changes_the_image_but_not_black_pixels():
    scene = load_case(rtgo, ("json", None))
    a, _, _ = oracle.render(scene, 32, 20, make_settings(rtgo, {"samples": 2}, seed=1))
    b, _, _ = oracle.render(scene, 32, 20, make_settings(rtgo, {"samples": 2}, seed=2))
    assert not same(a, b)
    assert np.array_equal(a == 0, b == 0) or np.mean((a == 0) != (b == 0)) < 0.05


def test_max_tiles_bounds_the_work():
    scene = load_case(rtgo, ("json", None))
    lin, _, c = oracle.render(scene, 96, 64, make_settings(rtgo, {"samples": 1}), max_tiles=2, counts=True)
    assert c["camera_rays"] == 2 * 32 * 32
    assert np.isnan(lin).any()  # unrendered tiles stay NaN-filled


def test_bvh_baseline_renders_the_linear_scan_image():
    """The secondary CPU baseline (oracle_render_ex with a sphere BVH and
    any-hit shadow rays, bench.py c4/c5) renders exactly the image of the
    reference's linear scans: a 2,000-sphere field of the C4 generator."""
    from scene_cases import spheres10k_scene

    scene = spheres10k_scene(rtgo, 2000)
    st = make_settings(rtgo, {"samples": 2, "max_depth": 8}, seed=3)
    lin, rgba, _ = oracle.render(scene, 40, 24, st)
    lin_b, rgba_b, _ = oracle.render(scene, 40, 24, st, bvh=True)
    assert (rgba[..., :3] > 0).mean() > 0.3
    assert lin_b.tobytes() == lin.tobytes()
    assert rgba_b.tobytes() == rgba.tobytes()

"""GPU parity: the gfx950 kernel (through the C ABI) against the CPU oracle.

Tolerance (BASELINE.json north_star): per-channel RMSE of the linear
radiance < 1e-4.  Both sides use the same counter-keyed RNG (include/rt_rng.h)
and binary64 arithmetic in the reference's order, and the kernel sums each
pixel's samples in sample order like tracePixel (renderer.go:150-163), so the
images are in fact BIT-IDENTICAL: the tests assert max |diff| == 0, identical
RGBA8 and identical integer path counts, which catch kernel bugs an RMSE bound
alone would let through.
"""
import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import PARITY_CASES, load_case, make_settings

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4


def _render_gpu(scene, w, h, st):
    r = rtgo.ParallelRenderer()
    r.settings = st
    rgba = r.render(scene, w, h)
    return r.last_linear.astype(np.float64), rgba


def _compare(lin_gpu, rgba_gpu, lin_ref, rgba_ref):
    ref32 = lin_ref.astype(np.float32).astype(np.float64)
    both_nan = np.isnan(lin_gpu) & np.isnan(ref32)
    assert np.array_equal(np.isnan(lin_gpu), np.isnan(ref32)), "NaN pattern differs"
    d = np.where(both_nan, 0.0, lin_gpu - ref32)
    rmse = np.sqrt(np.mean(d ** 2, axis=(0, 1)))
    return rmse, np.abs(d).max(), np.mean(np.any(rgba_gpu != rgba_ref, axis=2))


@pytest.mark.parametrize("case", PARITY_CASES, ids=[c[0] for c in PARITY_CASES])
def test_parity_vs_oracle(case):
    name, loader, w, h, over = case
    scene = load_case(rtgo, loader)
    for seed in (1, 2):
        st = make_settings(rtgo, over, seed)
        lin_g, rgba_g = _render_gpu(scene, w, h, st)
        lin_r, rgba_r, _ = oracle.render(scene, w, h, st)
        rmse, maxd, rgba_mis = _compare(lin_g, rgba_g, lin_r, rgba_r)
        print(f"{name} seed={seed} rmse={rmse} max|d|={maxd:.3e} rgba_mismatch={rgba_mis:.2e}")
        assert np.all(rmse < RMSE_TOL), (name, seed, rmse)
        # stricter: identical paths, identical sums
        assert maxd == 0.0, (name, seed, maxd)
        assert rgba_mis == 0.0, (name, seed, rgba_mis)


def test_as_committed_scene_is_black():
    """The reference camera looks down -Z from z=-8 and every object is
    behind it (renderer.go:377-390): the faithful image is
    black with alpha 255."""
    scene = rtgo.Scene.load_from_file(__import__("scene_cases").scene_path("sphere_reflections_light.json"))
    st = make_settings(rtgo, {"samples": 2})
    lin, rgba = _render_gpu(scene, 80, 60, st)
    assert np.all(lin == 0)
    assert np.all(rgba[..., :3] == 0) and np.all(rgba[..., 3] == 255)


@pytest.mark.parametrize("case", [c for c in PARITY_CASES if c[0] in ("spheres_facing", "all_materials",
                                                                       "silver_facing")],
                         ids=lambda c: c[0])
def test_path_counts_match_oracle(case):
    """Integer path structure is identical: camera rays, closest-hit queries,
    shadow rays, shading events, light evaluations and RNG draws."""
    import torch

    name, loader, w, h, over = case
    scene = load_case(rtgo, loader)
    st = make_settings(rtgo, over, 3)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    lin = torch.zeros(h * w * 3, dtype=torch.float32, device="cuda")
    rgba = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda")
    cg = ctx.count(w, h, st, lin.data_ptr(), rgba.data_ptr())
    torch.cuda.synchronize()
    _, _, cr = oracle.render(scene, w, h, st, counts=True)
    for k in ("camera_rays", "bounce_rays", "shadow_rays", "shade_events", "light_evals", "rng_draws"):
        assert cg[k] == cr[k], (name, k, cg[k], cr[k])
    ctx.close()


@pytest.mark.parametrize("name", sorted(__import__("scene_cases").EDGE_SCENES))
def test_culling_edge_scenes_match_oracle(name):
    """Huge radii, far coordinates, tiny spheres and lights almost on a
    surface: the exact-culling margins (relative) must never drop a
    primitive that can be hit (scene_cases._edge_scenes)."""
    import json

    from scene_cases import EDGE_SCENES

    scene = rtgo.Scene.from_json_text(json.dumps(EDGE_SCENES[name]))
    for seed in (1, 2):
        st = make_settings(rtgo, {"samples": 4}, seed)
        lin_g, rgba_g = _render_gpu(scene, 72, 48, st)
        lin_r, rgba_r, _ = oracle.render(scene, 72, 48, st)
        rmse, maxd, rgba_mis = _compare(lin_g, rgba_g, lin_r, rgba_r)
        print(f"{name} seed={seed} rmse={rmse} max|d|={maxd:.3e} lit={np.mean(rgba_r[..., :3] > 0):.3f}")
        assert maxd == 0.0 and rgba_mis == 0.0, (name, seed, maxd, rgba_mis)


SKY_CASES = [("all_materials", ("json", None), 64, 48, "default"), ("silver_facing",
             ("file", "final_silver_prism_purple_cube_facing.json"), 64, 48, "sunset"),
             ("spheres_facing", ("file", "sphere_reflections_light_facing.json"), 64, 48, "night"),
             ("spheres_facing_white", ("file", "sphere_reflections_light_facing.json"), 48, 32, "white")]


@pytest.mark.parametrize("case", SKY_CASES, ids=[c[0] for c in SKY_CASES])
def test_opt_in_sky_matches_oracle(case):
    """rt_settings.sky (off by default): a miss returns GetSkyColor
    (atmosphere.go:100-135) instead of black, on the megakernel path.
    Tolerance: the sky's exp / pow come from the device and host libm,
    which may differ in the last bit of a binary64; asserted per-channel
    RMSE < 1e-7 of the float32 output (the north star allows 1e-4)."""
    name, loader, w, h, sky = case
    scene = load_case(rtgo, loader)
    st = make_settings(rtgo, {"samples": 4}, 3)
    st.sky = rtgo.SKIES[sky]
    lin_g, rgba_g = _render_gpu(scene, w, h, st)
    lin_r, rgba_r, _ = oracle.render(scene, w, h, st)
    rmse, maxd, rgba_mis = _compare(lin_g, rgba_g, lin_r, rgba_r)
    print(f"sky {sky} {name}: rmse={rmse} max|d|={maxd:.3e} rgba_mismatch={rgba_mis:.2e}")
    assert np.all(rmse < 1e-7) and maxd < 1e-6 and rgba_mis < 1e-3
    assert np.all(lin_r[0, :, :] >= 0.0) and (rgba_r[..., :3] > 0).mean() > 0.9  # the sky is visible


def test_opt_in_sky_on_the_wavefront_path():
    """The same on the BVH + wavefront path (a 300-sphere field)."""
    import json

    from test_gpu_paths import _sphere_field

    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(300, seed=5)))
    st = make_settings(rtgo, {"samples": 3}, 2)
    st.sky = rtgo.SKIES["default"]
    lin_g, rgba_g = _render_gpu(scene, 60, 40, st)
    lin_r, rgba_r, _ = oracle.render(scene, 60, 40, st)
    rmse, maxd, rgba_mis = _compare(lin_g, rgba_g, lin_r, rgba_r)
    print(f"wavefront sky: rmse={rmse} max|d|={maxd:.3e} rgba_mismatch={rgba_mis:.2e}")
    assert np.all(rmse < 1e-7) and maxd < 1e-6 and rgba_mis < 1e-3


@pytest.mark.parametrize("case,spp", [(("spheres_facing", ("file", "sphere_reflections_light_facing.json")), 2100),
                                      (("silver_facing", ("file", "final_silver_prism_purple_cube_facing.json")),
                                       1501)], ids=["spheres_2100spp", "silver_1501spp"])
def test_sample_passes_match_oracle(case, spp):
    """More samples per pixel than a block holds (1024) render as sample
    passes that continue every pixel's running sum (rt_api.cpp,
    KParams.acc): SetSamples takes any count in the reference
    (settings.go:3-5), and the image is still tracePixel's sum in sample
    order, bit for bit.  1501 = 750 + 751: the passes differ in size, so the
    work schedule is rebuilt between them on the same stream."""
    name, loader = case
    scene = load_case(rtgo, loader)
    w, h = 20, 14
    st = make_settings(rtgo, {"samples": spp}, 6)
    lin_g, rgba_g = _render_gpu(scene, w, h, st)
    lin_r, rgba_r, _ = oracle.render(scene, w, h, st)
    rmse, maxd, rgba_mis = _compare(lin_g, rgba_g, lin_r, rgba_r)
    print(f"{name} {spp} spp: rmse={rmse} max|d|={maxd:.3e} lit={np.mean(rgba_r[..., :3] > 0):.2f}")
    assert (rgba_r[..., :3] > 0).any()
    assert maxd == 0.0 and rgba_mis == 0.0, (name, maxd, rgba_mis)

"""GPU: the wavefront path of BVH scenes (rt_wavefront.hip) against the
megakernel and the oracle.

The wavefront path cuts traceRay's bounce loop into staged kernels over
compacted path arrays.  It must give the megakernel's image
bit for bit (and hence the oracle's: the megakernel is pinned to the oracle
by the other GPU tests) and the same path counts, for every setting, layout,
path-array capacity and chunking of the frame.
"""
import copy
import json

import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import ALL_MATERIALS, make_settings
from gpu_util import render_dev
from test_gpu_paths import _sphere_field

pytestmark = pytest.mark.gpu

# path counts that do not depend on how a query is answered (the two paths
# answer the primary query differently: any-hit vs closest hit)
PATH_KEYS = ("camera_rays", "bounce_rays", "shadow_rays", "shade_events", "light_evals", "rng_draws")


def _spheres_only_all_materials():
    s = copy.deepcopy(ALL_MATERIALS)
    s["objects"] = [o for o in s["objects"] if o["type"] == "sphere"]
    return s


def _render(scene, w, h, st, mega, force_bvh=0, rank=0, world=1, tuning=None, count=False):
    t = tuning or rtgo.default_tuning()
    t.path = rtgo.RT_PATH_MEGAKERNEL if mega else rtgo.RT_PATH_AUTO
    lin, rgba, _, counts = render_dev(scene, w, h, st, rank=rank, world=world, tuning=t, force_bvh=force_bvh,
                                      count=count)
    return lin, rgba, counts


SETTINGS = [
    ("default", {"samples": 5}),
    ("no_soft", {"samples": 4, "soft_shadows": 0}),
    ("no_recursive", {"samples": 4, "recursive_reflections": 0}),
    ("depth1", {"samples": 3, "max_depth": 1}),
    ("depth0", {"samples": 3, "max_depth": 0}),
    ("seed7_deep", {"samples": 6, "max_depth": 50, "seed": 7}),
]


@pytest.mark.parametrize("name,over", SETTINGS, ids=[s[0] for s in SETTINGS])
def test_wavefront_equals_megakernel(name, over):
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(300, seed=5)))
    st = make_settings(rtgo, over)
    w, h = 72, 40
    lw, rw, cw = _render(scene, w, h, st, mega=False, count=True)
    lm, rm, cm = _render(scene, w, h, st, mega=True, count=True)
    assert lw.tobytes() == lm.tobytes()
    assert rw.tobytes() == rm.tobytes()
    assert {k: cw[k] for k in PATH_KEYS} == {k: cm[k] for k in PATH_KEYS}
    if over.get("max_depth", 50) > 0:
        assert cw["shade_events"] > 0


def test_wavefront_all_sphere_materials_matches_oracle():
    """Every sphere material (incl. dielectric, shiny, mirror, light) through
    the forced BVH + wavefront path, against the oracle's linear scan."""
    scene = rtgo.Scene.from_json_text(json.dumps(_spheres_only_all_materials()))
    st = make_settings(rtgo, {"samples": 6})
    lin, rgba, _ = _render(scene, 60, 40, st, mega=False, force_bvh=1)
    ref, ref_rgba, _ = oracle.render(scene, 60, 40, st)
    assert lin.reshape(40, 60, 3).tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.reshape(40, 60, 4).tobytes() == ref_rgba.tobytes()


@pytest.mark.parametrize("tun", [{"wf_paths": 64}, {"wf_paths": 4096}, {"wf_chunk": 700},
                                 {"wf_paths": 128, "wf_chunk": 3000}, {"wf_lds_nodes": 0}, {"wf_lds_nodes": 31},
                                 {"wf_trav_block": 256, "wf_trav_wgs": 4}, {"bvh_leaf": 1}, {"bvh_leaf": 7, "bvh_bins": 4}],
                         ids=["64_paths", "4096_paths", "chunks", "both", "bvh_all_global", "bvh_top_in_lds",
                              "small_traversal_groups", "leaf1", "leaf7_bins4"])
def test_capacity_and_chunks_do_not_change_the_image(tun):
    """... nor how much of the BVH the traversal kernels stage in LDS (by
    default all of it; here none, or only the top 31 nodes).  With
    wf_lds_nodes set, occlusion and cone walks take the binary tree instead
    of the 4-wide one (WfParams.use4), so those cases also hold the two
    walks to the same bits."""
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(200, seed=9)))
    st = make_settings(rtgo, {"samples": 7})
    base = _render(scene, 50, 37, st, mega=False)
    other = _render(scene, 50, 37, st, mega=False, tuning=rtgo.default_tuning(**tun))
    assert base[0].tobytes() == other[0].tobytes()
    assert base[1].tobytes() == other[1].tobytes()


@pytest.mark.parametrize("rank,world", [(0, 3), (2, 3)])
def test_wavefront_packed_tiles_equal_megakernel(rank, world):
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(150, seed=2)))
    st = make_settings(rtgo, {"samples": 3})
    a = _render(scene, 100, 70, st, mega=False, rank=rank, world=world)
    b = _render(scene, 100, 70, st, mega=True, rank=rank, world=world)
    assert a[0].tobytes() == b[0].tobytes()
    assert a[1].tobytes() == b[1].tobytes()


def test_more_than_32_lights_match_the_oracle():
    """The wavefront kernels keep per-light state in 32-light chunks: a
    BVH scene (> 64 spheres) with 40 lights equals the oracle's linear scan,
    which loops over the lights with no limit (renderer.go:248-294)."""
    field = _sphere_field(80, seed=13)
    rng = np.random.default_rng(4)
    field["lights"] = [{"position": [float(v) for v in rng.uniform(-15, 15, 3)], "color": [1, 1, 1],
                        "intensity": float(rng.uniform(20, 200))} for _ in range(40)]
    scene = rtgo.Scene.from_json_text(json.dumps(field))
    st = make_settings(rtgo, {"samples": 2, "max_depth": 5})
    lin, rgba, _ = _render(scene, 40, 24, st, mega=False)
    ref, ref_rgba, _ = oracle.render(scene, 40, 24, st)
    assert lin.reshape(24, 40, 3).tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.reshape(24, 40, 4).tobytes() == ref_rgba.tobytes()
    mk = _render(scene, 40, 24, st, mega=True)
    assert mk[0].tobytes() == lin.tobytes()


def test_more_than_1024_samples_on_both_bvh_paths():
    """A sample count past one block's 1024 on a BVH scene: the wavefront
    path (no per-pixel limit) and the megakernel's BVH path (sample passes,
    rt_api.cpp) both give the oracle's image."""
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(300, seed=8)))
    st = make_settings(rtgo, {"samples": 1100, "max_depth": 6}, seed=2)
    w, h = 16, 12
    ref, ref_rgba, _ = oracle.render(scene, w, h, st)
    ref32 = ref.astype(np.float32).reshape(-1, 3)
    for mega in (False, True):
        lin, rgba, _ = _render(scene, w, h, st, mega)
        assert lin.tobytes() == ref32.tobytes(), mega
        assert rgba.tobytes() == ref_rgba.reshape(-1, 4).tobytes(), mega


@pytest.mark.parametrize("name", sorted(__import__("scene_cases").EDGE_SCENES))
def test_cone_edge_scenes_on_the_wavefront_path(name):
    """The shadow cones of the wavefront path (wf_cone's binary32 node test
    and binary64 sphere test, the hit sphere's exclusion)
    at the culling edge scenes: radius-1e6 ground, coordinates near 1e5,
    radius-1e-3 spheres seen from 2 cm, lights 2e-3 above a surface.  The
    scene's spheres (cubes dropped: the BVH path is sphere-only) through the
    forced BVH, against the oracle's linear scan."""
    from scene_cases import EDGE_SCENES

    sc = copy.deepcopy(EDGE_SCENES[name])
    sc["objects"] = [o for o in sc["objects"] if o["type"] == "sphere"]
    scene = rtgo.Scene.from_json_text(json.dumps(sc))
    w, h = 60, 40
    for seed in (1, 2):
        st = make_settings(rtgo, {"samples": 4}, seed)
        lin, rgba, _ = _render(scene, w, h, st, mega=False, force_bvh=1)
        ref, ref_rgba, _ = oracle.render(scene, w, h, st)
        assert lin.reshape(h, w, 3).tobytes() == ref.astype(np.float32).tobytes(), (name, seed)
        assert rgba.reshape(h, w, 4).tobytes() == ref_rgba.tobytes(), (name, seed)


def _curtain_scene():
    """Spheres under a light with a dense curtain of 360 small spheres
    between them: the clear hard rays' shadow cones meet from zero to many
    candidates, so every soft-shadow route of the wavefront path runs
    (empty cone, a candidate list, more than 16 candidates: traced)."""
    objs = [{"type": "sphere", "position": [0, -1001, -8], "radius": 1000,
             "material": {"type": "lambertian", "color": [0.6, 0.6, 0.5]}}]
    for i in range(9):
        objs.append({"type": "sphere", "position": [-4 + i, -0.3, -8 - (i % 3)], "radius": 0.6,
                     "material": {"type": ["metal", "glass", "lambertian"][i % 3], "color": [0.8, 0.7, 0.6],
                                  "roughness": 0.05}})
    for i in range(360):  # a 24 x 15 curtain at y = 3, gaps of ~0.1
        x, z = i % 24, i // 24
        objs.append({"type": "sphere", "position": [-6 + 0.5 * x, 3.0, -4 - 0.5 * z], "radius": 0.2,
                     "material": {"type": "lambertian", "color": [0.3, 0.4, 0.8]}})
    return {"camera": {"position": [0, 1, 2], "aspectRatio": 1.5}, "objects": objs,
            "lights": [{"position": [1, 9, -7], "color": [1, 1, 1], "intensity": 200},
                       {"position": [-9, 4, -2], "color": [1, 0.9, 0.8], "intensity": 120}]}


def test_cone_routes_match_megakernel_and_oracle():
    scene = rtgo.Scene.from_json_text(json.dumps(_curtain_scene()))
    st = make_settings(rtgo, {"samples": 4, "max_depth": 6})
    w, h = 60, 40
    lw, rw, cw = _render(scene, w, h, st, mega=False, count=True)
    lm, rm, cm = _render(scene, w, h, st, mega=True, count=True)
    assert lw.tobytes() == lm.tobytes() and rw.tobytes() == rm.tobytes()
    assert {k: cw[k] for k in PATH_KEYS} == {k: cm[k] for k in PATH_KEYS}
    ref, ref_rgba, _ = oracle.render(scene, w, h, st)
    assert lw.reshape(h, w, 3).tobytes() == ref.astype(np.float32).tobytes()
    assert rw.reshape(h, w, 4).tobytes() == ref_rgba.tobytes()
    # every route ran: soft rays traced through the BVH (cones with more
    # than 16 candidates) and list tests (the soft stage's sphere tests
    # exceed what its traced rays' leaves alone would give)
    ctx = rtgo.Context(0)
    ctx.set_tuning(rtgo.default_tuning())
    ctx.set_scene(scene)
    import torch

    lin = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    c = ctx.count(w, h, st, lin.data_ptr(), 0, full=True)
    soft = c.soft_occlusion_dict()
    ext, hard = c.extend_dict(), c.hard_occlusion_dict()
    ctx.close()
    # the closest-hit and hard-ray traversals' own counts (bench.py per-kernel
    # roofline): every closest-hit query runs in wf_extend; the hard rays not
    # settled by their own sphere (wf_shade1) run in wf_occlude<hard>
    assert ext["bounce_rays"] == c.bounce_rays and ext["box_tests"] > 0 and ext["sphere_tests"] > 0, ext
    assert 0 < hard["shadow_rays"] < c.shadow_rays and hard["box_tests"] > 0, hard
    assert ext["sphere_tests"] + hard["sphere_tests"] + soft["sphere_tests"] <= c.sphere_tests
    assert soft["shadow_rays"] > 0, soft                     # traced (overflowing cones)
    assert soft["shadow_rays"] < c.shadow_rays, (soft, c.shadow_rays)  # not all: lists and empty cones
    assert soft["sphere_tests"] > 0 and soft["box_tests"] > 0


@pytest.mark.parametrize("tries", [1, 8, 20])
def test_listed_cones_past_their_try_mask(tries):
    """wf_listtest rebuilds a listed cone's 16 points from its stream state
    and the mask of accepted tries among its first wf_list_tries (64) tries,
    and continues the sequential rejection loop past them when the 16th point
    needs more (about once in 10^6 cones at 64).  Forced low here, so most
    listed cones take that path: the image and the path counts (RNG draws
    included) stay the oracle's."""
    scene = rtgo.Scene.from_json_text(json.dumps(_curtain_scene()))
    st = make_settings(rtgo, {"samples": 4, "max_depth": 6})
    w, h = 60, 40
    lb, rb, cb = _render(scene, w, h, st, mega=False, count=True)
    lo, ro, co = _render(scene, w, h, st, mega=False, count=True, tuning=rtgo.default_tuning(wf_list_tries=tries))
    assert lo.tobytes() == lb.tobytes() and ro.tobytes() == rb.tobytes()
    assert {k: co[k] for k in PATH_KEYS} == {k: cb[k] for k in PATH_KEYS}
    ref, ref_rgba, _ = oracle.render(scene, w, h, st)
    assert lo.reshape(h, w, 3).tobytes() == ref.astype(np.float32).tobytes()
    assert ro.reshape(h, w, 4).tobytes() == ref_rgba.tobytes()

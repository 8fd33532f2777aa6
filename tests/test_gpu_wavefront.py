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
    default all of it; here none, or only the top 31 nodes)."""
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

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
from test_gpu_paths import _sphere_field

pytestmark = pytest.mark.gpu

# path counts that do not depend on how a query is answered (the two paths
# answer the primary query differently: any-hit vs closest hit)
PATH_KEYS = ("camera_rays", "bounce_rays", "shadow_rays", "shade_events", "light_evals", "rng_draws")


def _spheres_only_all_materials():
    s = copy.deepcopy(ALL_MATERIALS)
    s["objects"] = [o for o in s["objects"] if o["type"] == "sphere"]
    return s


def _render(scene, w, h, st, monkeypatch, mega, force_bvh=0, rank=0, world=1, env=None, count=False):
    import torch

    monkeypatch.delenv("RTGO_MEGAKERNEL", raising=False)
    if mega:
        monkeypatch.setenv("RTGO_MEGAKERNEL", "1")
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene, force_bvh=force_bvh)
    packed = world > 1
    n = rtgo.tiles_for_rank(w, h, rank, world) * 1024 if packed else w * h
    lin = torch.full((n * 3,), float("nan"), dtype=torch.float32, device="cuda")
    rgba = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    layout = rtgo.RT_LAYOUT_PACKED_TILES if packed else rtgo.RT_LAYOUT_IMAGE
    counts = None
    if count:
        counts = ctx.count(w, h, st, lin.data_ptr(), rgba.data_ptr(), 0, rank, world, layout)
    else:
        ctx.render_async(w, h, st, lin.data_ptr(), rgba.data_ptr(), 0, rank, world, layout)
    torch.cuda.synchronize()
    out = lin.cpu().numpy(), rgba.cpu().numpy(), counts
    ctx.close()
    for k in (env or {}):
        monkeypatch.delenv(k)
    monkeypatch.delenv("RTGO_MEGAKERNEL", raising=False)
    return out


SETTINGS = [
    ("default", {"samples": 5}),
    ("no_soft", {"samples": 4, "soft_shadows": 0}),
    ("no_recursive", {"samples": 4, "recursive_reflections": 0}),
    ("depth1", {"samples": 3, "max_depth": 1}),
    ("depth0", {"samples": 3, "max_depth": 0}),
    ("seed7_deep", {"samples": 6, "max_depth": 50, "seed": 7}),
]


@pytest.mark.parametrize("name,over", SETTINGS, ids=[s[0] for s in SETTINGS])
def test_wavefront_equals_megakernel(name, over, monkeypatch):
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(300, seed=5)))
    st = make_settings(rtgo, over)
    w, h = 72, 40
    lw, rw, cw = _render(scene, w, h, st, monkeypatch, mega=False, count=True)
    lm, rm, cm = _render(scene, w, h, st, monkeypatch, mega=True, count=True)
    assert lw.tobytes() == lm.tobytes()
    assert rw.tobytes() == rm.tobytes()
    assert {k: cw[k] for k in PATH_KEYS} == {k: cm[k] for k in PATH_KEYS}
    if over.get("max_depth", 50) > 0:
        assert cw["shade_events"] > 0


def test_wavefront_all_sphere_materials_matches_oracle(monkeypatch):
    """Every sphere material (incl. dielectric, shiny, mirror, light) through
    the forced BVH + wavefront path, against the oracle's linear scan."""
    scene = rtgo.Scene.from_json_text(json.dumps(_spheres_only_all_materials()))
    st = make_settings(rtgo, {"samples": 6})
    lin, rgba, _ = _render(scene, 60, 40, st, monkeypatch, mega=False, force_bvh=1)
    ref, ref_rgba, _ = oracle.render(scene, 60, 40, st)
    assert lin.reshape(40, 60, 3).tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.reshape(40, 60, 4).tobytes() == ref_rgba.tobytes()


@pytest.mark.parametrize("env", [{"RTGO_WF_PATHS": "64"}, {"RTGO_WF_PATHS": "4096"},
                                 {"RTGO_WF_CHUNK": "700"}, {"RTGO_WF_PATHS": "128", "RTGO_WF_CHUNK": "3000"},
                                 {"RTGO_WF_LDS_NODES": "0"}, {"RTGO_WF_LDS_NODES": "31"}],
                         ids=["64_paths", "4096_paths", "chunks", "both", "bvh_all_global", "bvh_top_in_lds"])
def test_capacity_and_chunks_do_not_change_the_image(env, monkeypatch):
    """... nor how much of the BVH the traversal kernels stage in LDS (by
    default all of it; here none, or only the top 31 nodes)."""
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(200, seed=9)))
    st = make_settings(rtgo, {"samples": 7})
    base = _render(scene, 50, 37, st, monkeypatch, mega=False)
    other = _render(scene, 50, 37, st, monkeypatch, mega=False, env=env)
    assert base[0].tobytes() == other[0].tobytes()
    assert base[1].tobytes() == other[1].tobytes()


@pytest.mark.parametrize("rank,world", [(0, 3), (2, 3)])
def test_wavefront_packed_tiles_equal_megakernel(rank, world, monkeypatch):
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(150, seed=2)))
    st = make_settings(rtgo, {"samples": 3})
    a = _render(scene, 100, 70, st, monkeypatch, mega=False, rank=rank, world=world)
    b = _render(scene, 100, 70, st, monkeypatch, mega=True, rank=rank, world=world)
    assert a[0].tobytes() == b[0].tobytes()
    assert a[1].tobytes() == b[1].tobytes()

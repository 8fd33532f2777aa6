"""GPU parity for rays inside cubes (scene_cases.CUBE_SCENES).

createCube (internal/scene/scene.go:150-190) winds its triangles so that
calculateNormal (internal/geometry/triangle.go:29-33) points INTO the box, so
FrontFace (triangle.go:70-73) is true for a hit from inside.  The kernels'
shadow-cone culling leaves the hit object out of its own shadow rays only
when the hit is on the object's OUTSIDE (rt_kernel.hip box_self_out): a ray
that leaves an inner face toward an outside light must still cross the box
(calculateSmartShadow, renderer.go:299-331).  These scenes reach that case
through glass and dielectric cubes, a camera inside a cube, lights inside
and outside cubes and mirrored (negative-size) cubes, on the megakernel's
main loop, a 50-bounce mirror probe (the lone-path form's case, held to
the product in tests/test_gpu_xlane.py) and a 70-sphere
scene without cone masks.  Bar: bit-identical float32 radiance and RGBA8 at
seeds 1 and 2, and identical integer path counts (shadow rays included).
"""
import json

import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import CUBE_SCENES, make_settings

pytestmark = pytest.mark.gpu

W, H = 72, 48


def _scene(name):
    return rtgo.Scene.from_json_text(json.dumps(CUBE_SCENES[name]))


def _render(scene, st, tun=None):
    r = rtgo.ParallelRenderer()
    r.settings = st
    if tun:
        r.set_tuning(rtgo.default_tuning(**tun))
    rgba = r.render(scene, W, H)
    return r.last_linear, rgba


@pytest.mark.parametrize("name", sorted(CUBE_SCENES))
def test_cube_scene_matches_oracle(name):
    scene = _scene(name)
    for seed in (1, 2):
        st = make_settings(rtgo, {"samples": 4}, seed)
        lin, rgba = _render(scene, st)
        ref, ref_rgba, _ = oracle.render(scene, W, H, st)
        ref32 = ref.astype(np.float32)
        nd = int(np.count_nonzero(lin != ref32))
        print(f"{name} seed={seed} differing channels={nd} lit={np.mean(ref_rgba[..., :3] > 0):.2f}")
        assert (ref_rgba[..., :3] > 0).any(), name
        assert lin.tobytes() == ref32.tobytes(), (name, seed, nd)
        assert rgba.tobytes() == ref_rgba.tobytes(), (name, seed)


@pytest.mark.parametrize("name", sorted(CUBE_SCENES))
def test_cube_scene_path_counts_match_oracle(name):
    """Identical camera rays, closest-hit queries, shadow rays, shading
    events, light evaluations and RNG draws: a shadow ray wrongly taken as
    clear adds 16 soft rays and their draws."""
    import torch

    scene = _scene(name)
    st = make_settings(rtgo, {"samples": 3}, 3)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    lin = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    rgba = torch.zeros(H * W * 4, dtype=torch.uint8, device="cuda")
    cg = ctx.count(W, H, st, lin.data_ptr(), rgba.data_ptr())
    torch.cuda.synchronize()
    _, _, cr = oracle.render(scene, W, H, st, counts=True)
    for k in ("camera_rays", "bounce_rays", "shadow_rays", "shade_events", "light_evals", "rng_draws"):
        assert cg[k] == cr[k], (name, k, cg[k], cr[k])
    ctx.close()


@pytest.mark.parametrize("tun", [{"block_work": 1}, {"frustum": 0, "stage": 0}, {"block_work": 1e6}],
                         ids=["every_pixel_split", "no_frustum_no_stage", "huge_blocks"])
@pytest.mark.parametrize("name", ["glass_dielectric_cubes", "camera_inside_cube", "mirrored_cubes"])
def test_cube_scene_schedules_match_oracle(name, tun):
    """Other work cuts: more lanes share a block's shading rounds (huge
    blocks), or nearly every pixel runs split (lone paths in small blocks)."""
    scene = _scene(name)
    st = make_settings(rtgo, {"samples": 5}, 4)
    lin, rgba = _render(scene, st, tun)
    ref, ref_rgba, _ = oracle.render(scene, W, H, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes(), (name, tun)
    assert rgba.tobytes() == ref_rgba.tobytes(), (name, tun)

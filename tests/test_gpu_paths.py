"""GPU: the remaining paths of the kernel through the C ABI.

* committed oracle fixtures reproduced bit for bit (float32 store of the
  binary64 mean, RGBA8);
* the packed-tile layout of a rank (RT_LAYOUT_PACKED_TILES) and the unpack
  kernel: every world size reassembles exactly the 1-rank image;
* the BVH path (> 64 spheres) against the oracle's linear scan;
* the CLI (cmd/raytracer/main.go mirror) writes the same pixels as the API.
"""
import json
import os
import subprocess
import zlib

import numpy as np
import pytest

import oracle
import rtgo
from conftest import GOLDEN, ROOT
from rtgo import shard
from scene_cases import GOLDEN_CASES, load_case, make_settings

pytestmark = pytest.mark.gpu


def _gpu(scene, w, h, st):
    r = rtgo.ParallelRenderer()
    r.settings = st
    rgba = r.render(scene, w, h)
    return r.last_linear, rgba


@pytest.mark.parametrize("case", GOLDEN_CASES, ids=[c[0] for c in GOLDEN_CASES])
def test_kernel_reproduces_committed_fixture(case):
    name, loader, w, h, over, seed = case
    g = np.load(os.path.join(GOLDEN, f"oracle_{name}.npz"))
    lin, rgba = _gpu(load_case(rtgo, loader), w, h, make_settings(rtgo, over, seed))
    ref = g["linear"].astype(np.float32)
    # identical paths and the same in-order sample sums: bit for bit
    assert lin.tobytes() == ref.tobytes()
    assert rgba.tobytes() == g["rgba"].tobytes()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_packed_tiles_and_unpack_reassemble_the_image(world):
    import torch

    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3})
    w, h = 75, 50
    ref_lin, ref_rgba = _gpu(scene, w, h, st)
    ctx = rtgo.Context(0)
    ctx.set_scene(scene)
    ml = shard.max_local_tiles(w, h, world)
    g_lin = torch.zeros(world * ml * 1024 * 3, dtype=torch.float32, device="cuda")
    g_rgba = torch.zeros(world * ml * 1024 * 4, dtype=torch.uint8, device="cuda")
    for r in range(world):
        pl = g_lin[r * ml * 1024 * 3:(r + 1) * ml * 1024 * 3]
        pr = g_rgba[r * ml * 1024 * 4:(r + 1) * ml * 1024 * 4]
        ctx.render_async(w, h, st, pl.data_ptr(), pr.data_ptr(), 0, r, world, rtgo.RT_LAYOUT_PACKED_TILES)
    img_lin = torch.full((h * w * 3,), float("nan"), dtype=torch.float32, device="cuda")
    img_rgba = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda")
    rtgo.unpack_tiles_async(w, h, world, ml, g_lin.data_ptr(), g_rgba.data_ptr(), img_lin.data_ptr(),
                            img_rgba.data_ptr(), 0)
    torch.cuda.synchronize()
    assert img_lin.cpu().numpy().reshape(h, w, 3).tobytes() == ref_lin.tobytes()
    assert img_rgba.cpu().numpy().reshape(h, w, 4).tobytes() == ref_rgba.tobytes()
    # the packed layout is exactly rtgo.shard's (the gloo CPU test relies on it)
    packed = g_rgba.cpu().numpy().reshape(world * ml * 1024, 4)
    want = np.concatenate([shard.pack_host(ref_rgba, r, world) for r in range(world)])
    assert np.array_equal(packed, want)
    ctx.close()


def _sphere_field(n, seed=42):
    rng = np.random.default_rng(seed)
    kinds = ["metal", "glass", "lambertian"]
    objs = []
    for i in range(n):
        k = kinds[i % 3]
        m = {"type": k, "color": [float(v) for v in rng.uniform(0.2, 0.9, 3)]}
        if k == "metal":
            m["roughness"] = float(rng.uniform(0, 0.3))
        objs.append({"type": "sphere", "radius": float(rng.uniform(0.3, 1.0)),
                     "position": [float(rng.uniform(-12, 12)), float(rng.uniform(-8, 8)),
                                  float(rng.uniform(-40, -6))], "material": m})
    return {"camera": {"position": [0, 0, 0], "aspectRatio": 1.5}, "objects": objs,
            "lights": [{"position": [10, 10, 5], "color": [1, 1, 1], "intensity": 300},
                       {"position": [-10, 5, 0], "color": [1, 0.9, 0.8], "intensity": 150}]}


def test_bvh_matches_linear_oracle():
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(400)))
    st = make_settings(rtgo, {"samples": 2, "max_depth": 6})
    lin, rgba = _gpu(scene, 64, 40, st)  # > 64 spheres: BVH path
    ref, ref_rgba, _ = oracle.render(scene, 64, 40, st)
    # the BVH returns the linear scan's closest hit (ties by hittable index)
    assert lin.tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()


def test_forced_bvh_equals_linear_scan_on_gpu():
    import torch

    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(40, seed=3)))
    st = make_settings(rtgo, {"samples": 2})
    outs = []
    for force in (-1, 1):  # -1: never BVH, 1: always
        ctx = rtgo.Context(0)
        ctx.set_scene(scene, force_bvh=force)
        lin = torch.zeros(48 * 32 * 3, dtype=torch.float32, device="cuda")
        rgba = torch.zeros(48 * 32 * 4, dtype=torch.uint8, device="cuda")
        ctx.render_async(48, 32, st, lin.data_ptr(), rgba.data_ptr())
        torch.cuda.synchronize()
        outs.append(lin.cpu().numpy())
        ctx.close()
    assert outs[0].tobytes() == outs[1].tobytes()


def _read_png(path):
    data = open(path, "rb").read()
    i, idat, w, h = 8, b"", 0, 0
    while i < len(data):
        n = int.from_bytes(data[i:i + 4], "big")
        typ = data[i + 4:i + 8]
        if typ == b"IHDR":
            w, h = int.from_bytes(data[i + 8:i + 12], "big"), int.from_bytes(data[i + 12:i + 16], "big")
        if typ == b"IDAT":
            idat += data[i + 8:i + 8 + n]
        i += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[r * (1 + 3 * w) + 1:(r + 1) * (1 + 3 * w)] for r in range(h)]
    return np.frombuffer(b"".join(rows), np.uint8).reshape(h, w, 3)


def test_cli_writes_png_and_benchmark_data(tmp_path):
    exe = os.path.join(ROOT, "concurrent-raytracer-go_amd", "build", "raytracer")
    scene_file = os.path.join(ROOT, "scenes", "sphere_reflections_light_facing.json")
    out = tmp_path / "out"  # no extension: main.go:53-56 appends ".png"
    p = subprocess.run([exe, scene_file, str(out), "64", "48", "--samples", "3"], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr
    assert "Created 5 hittables total" in p.stdout
    img = _read_png(str(out) + ".png")
    bd = json.load(open(tmp_path / "benchmark_data.json"))
    assert bd["resolution"] == "64x48" and bd["samples"] == 3 and bd["objects"] == 5
    assert bd["rays_per_second"] > 0
    r = rtgo.ParallelRenderer()
    r.set_samples(3)
    rgba = r.render(rtgo.Scene.load_from_file(scene_file), 64, 48)
    assert np.array_equal(img, rgba[:, :, :3])


def test_ten_thousand_sphere_field_matches_oracle():
    """Config C4's scene (scenes/gen_spheres.py, 10k spheres: the BVH path)
    at a size the linear-scan oracle finishes in seconds."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("gen_spheres", os.path.join(ROOT, "scenes", "gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    scene = rtgo.Scene.from_json_text(g.dumps(g.generate(10000)))
    st = make_settings(rtgo, {"samples": 2, "max_depth": 4})
    lin, rgba = _gpu(scene, 32, 18, st)
    ref, ref_rgba, _ = oracle.render(scene, 32, 18, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()

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
from gpu_util import render_dev, unpack_dev
from rtgo import shard
from scene_cases import GOLDEN_CASES, load_case, make_settings, spheres10k_scene

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
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3})
    w, h = 75, 50
    ref_lin, ref_rgba = _gpu(scene, w, h, st)
    shares = [render_dev(scene, w, h, st, rank=r, world=world)[2] for r in range(world)]
    img_lin, img_rgba = unpack_dev(w, h, world, shares)
    assert img_lin.tobytes() == ref_lin.tobytes()
    assert img_rgba.tobytes() == ref_rgba.tobytes()
    # the packed layout is exactly rtgo.shard's (the gloo CPU test relies on it):
    # compare the RGBA8 half and the non-padding float3 slots
    for r in range(world):
        want = shard.pack_share_host(ref_lin, ref_rgba, r, world)
        off = rtgo.packed_rgba_offset(w, h, world)
        assert np.array_equal(shares[r][off:], want[off:])
        ok = shard.packed_index(w, h, r, world) >= 0
        assert shares[r][:off].view(np.float32).reshape(-1, 3)[ok].tobytes() == \
            want[:off].view(np.float32).reshape(-1, 3)[ok].tobytes()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]], ids=["1_device", "3_ranks_on_device_0"])
def test_renderer_multi_rank_equals_one_rank(devices):
    """rt_renderer_render (the persistent renderer of the C ABI) with several
    ranks on device 0: every rank renders its share straight into the gather
    buffer, one kernel unpacks; the image equals the 1-rank image, and a
    second call (same scene, new seed) equals a fresh renderer's."""
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 3}, seed=9)
    w, h = 75, 50
    ref_lin, ref_rgba = _gpu(scene, w, h, st)
    r = rtgo.ParallelRenderer(devices=devices)
    st.num_devices = len(devices)
    r.settings = st
    rgba = r.render(scene, w, h)
    assert r.last_linear.tobytes() == ref_lin.tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()
    st2 = make_settings(rtgo, {"samples": 3}, seed=10)
    r.settings.seed = 10
    rgba2 = r.render(scene, w, h)
    lin2 = r.last_linear.copy()
    ref2_lin, ref2_rgba = _gpu(scene, w, h, st2)
    assert lin2.tobytes() == ref2_lin.tobytes()
    assert rgba2.tobytes() == ref2_rgba.tobytes()
    r.close()


@pytest.mark.parametrize("size", [(80, 48), (75, 50)], ids=["16B_multiple", "ragged"])
def test_renderer_rgba_only_equals_full_render(size):
    """Render without the float3 image (out_linear_rgb NULL: Go's Render
    returns the RGBA image only, renderer.go:67), on a new renderer's first
    call (its image goes down through the download kernel when the sizes are
    multiples of 16 B) and on a later call (a copy from the idle stream):
    the same RGBA bytes as the full render."""
    scene = load_case(rtgo, ("json", None))
    w, h = size
    r = rtgo.ParallelRenderer()
    for seed in (3, 4):
        st = make_settings(rtgo, {"samples": 3}, seed=seed)
        _, ref_rgba = _gpu(scene, w, h, st)
        r.settings = make_settings(rtgo, {"samples": 3}, seed=seed)
        rgba = r.render(scene, w, h, keep_linear=False)
        assert r.last_linear is None
        assert rgba.tobytes() == ref_rgba.tobytes()
    r.close()


def test_renderer_ranks_drive_bvh_frames_concurrently():
    """A BVH scene runs the wavefront path, whose host loop returns only when
    the frame is done; rt_renderer_render drives each rank from its own
    thread.  3 ranks on device 0 (their loops interleaved on one GPU) give
    the 1-rank image, twice in a row."""
    scene = spheres10k_scene(rtgo)
    w, h = 96, 64
    r = rtgo.ParallelRenderer(devices=[0, 0, 0])
    for seed in (4, 5):
        st = make_settings(rtgo, {"samples": 2, "max_depth": 6}, seed=seed)
        ref_lin, ref_rgba = _gpu(scene, w, h, st)
        st.num_devices = 3
        r.settings = st
        rgba = r.render(scene, w, h)
        assert r.last_linear.tobytes() == ref_lin.tobytes()
        assert rgba.tobytes() == ref_rgba.tobytes()
    r.close()


def test_comm_of_one_rank_and_one_shot_render():
    """rt_comm over one rank (ncclCommInitRank, world 1: the gather moves
    nothing) and the one-shot rt_render with num_devices = 1."""
    import torch

    uid = rtgo.Comm.unique_id()
    assert len(uid) == rtgo.RT_COMM_ID_BYTES
    c = rtgo.Comm(uid, 1, 0, 0)
    buf = torch.zeros(rtgo.packed_bytes(64, 64, 1), dtype=torch.uint8, device="cuda")
    c.gather_tiles_async(64, 64, buf.data_ptr(), buf.data_ptr(), 0)
    torch.cuda.synchronize()
    c.close()
    scene = load_case(rtgo, ("json", None))
    st = make_settings(rtgo, {"samples": 2}, seed=3)
    rgba, lin, stats = rtgo.render(scene, 40, 30, st)
    ref, ref_rgba, _ = oracle.render(scene, 40, 30, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()
    assert stats.render_seconds >= stats.kernel_seconds > 0


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
    scene = rtgo.Scene.from_json_text(json.dumps(_sphere_field(40, seed=3)))
    st = make_settings(rtgo, {"samples": 2})
    outs = [render_dev(scene, 48, 32, st, force_bvh=force)[0] for force in (-1, 1)]  # -1: never BVH, 1: always
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
    scene = spheres10k_scene(rtgo)
    st = make_settings(rtgo, {"samples": 2, "max_depth": 4})
    lin, rgba = _gpu(scene, 32, 18, st)
    ref, ref_rgba, _ = oracle.render(scene, 32, 18, st)
    assert lin.tobytes() == ref.astype(np.float32).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()

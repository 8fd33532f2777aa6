"""The multi-rank renderer's watchdog on the GPU (rt_renderer_set_watchdog).

Two ranks on the box's one device (devices [0, 0]: the same wait path as N
devices, without RCCL).  A test-hook stall on rank 1 (a kernel that sleeps
3 s of device time and then exits on its own) against a 0.5 s watchdog: the
Render returns RT_E_TIMEOUT naming the rank, device, frame and partition
instead of waiting, later Renders of that renderer refuse with the same
error, and a renderer with the default watchdog renders the oracle's image
as before.  The frame's deadline bounds every host wait of the frame, not
only the waits after its launches: the stall also ends a frame
whose rank must first rebuild its schedule (new settings: the previous
render's wait and the block count read-back) and a BVH scene's frame (the
host-driven wavefront bounce loop)."""
import time

import numpy as np
import pytest

import oracle
import rtgo
from scene_cases import make_settings, scene_path, spheres10k_scene

pytestmark = pytest.mark.gpu

W, H = 160, 120


def _scene():
    return rtgo.Scene.load_from_file(scene_path("sphere_reflections_light_facing.json"))


def test_watchdog_returns_timeout_on_a_stalled_rank():
    scene = _scene()
    r = rtgo.ParallelRenderer(devices=[0, 0])
    r.settings = make_settings(rtgo, {"samples": 2}, seed=3)
    r.render(scene, W, H)  # a normal frame first (contexts, partition)
    r.set_watchdog(0.5)
    r.test_stall(1, 3000.0)
    t0 = time.monotonic()
    with pytest.raises(rtgo.RenderError) as ei:
        r.render(scene, W, H)
    took = time.monotonic() - t0
    msg = str(ei.value)
    assert f"error {rtgo.RT_E_TIMEOUT}" in msg, msg
    assert "watchdog: rank 1 (device 0) did not finish frame 1" in msg and "partition" in msg, msg
    assert took < 2.5, took  # returned at the watchdog, not after the 3 s stall
    with pytest.raises(rtgo.RenderError) as again:
        r.render(scene, W, H)
    assert "watchdog" in str(again.value)
    r.close()  # (releases only what does not wait on the stall)
    time.sleep(3.0)  # the stall kernel ends on its own


@pytest.mark.parametrize("case", ["schedule_rebuild", "bvh_wavefront"])
def test_watchdog_bounds_the_waits_inside_a_rank_render(case):
    """The stall is enqueued on rank 1's stream before the rank renders, so
    the rank's own host waits (inside rt_context_render_async) meet it first:
    a new schedule waits for the previous render and reads the block counts
    back; a BVH scene's bounce loop reads its state back every bounce."""
    if case == "bvh_wavefront":
        scene, w, h = spheres10k_scene(rtgo, 2000), 128, 96
    else:
        scene, w, h = _scene(), W, H
    r = rtgo.ParallelRenderer(devices=[0, 0])
    r.settings = make_settings(rtgo, {"samples": 2}, seed=3)
    r.render(scene, w, h)  # a normal frame first
    r.set_watchdog(0.5)
    if case == "schedule_rebuild":
        r.settings = make_settings(rtgo, {"samples": 3}, seed=3)  # a new schedule key
    r.test_stall(1, 3000.0)
    t0 = time.monotonic()
    with pytest.raises(rtgo.RenderError) as ei:
        r.render(scene, w, h)
    took = time.monotonic() - t0
    msg = str(ei.value)
    assert f"error {rtgo.RT_E_TIMEOUT}" in msg, msg
    assert "watchdog: rank 1 (device 0) did not finish frame 1" in msg, msg
    assert took < 2.5, took
    r.close()
    time.sleep(3.0)


def test_default_watchdog_renders_as_before():
    scene = _scene()
    st = make_settings(rtgo, {"samples": 2}, seed=4)
    r = rtgo.ParallelRenderer(devices=[0, 0])
    r.settings = st
    rgba = r.render(scene, W, H)
    lin = r.last_linear
    r.close()
    ref, ref_rgba, _ = oracle.render(scene, W, H, st)
    assert lin.astype(np.float64).tobytes() == ref.astype(np.float32).astype(np.float64).tobytes()
    assert rgba.tobytes() == ref_rgba.tobytes()

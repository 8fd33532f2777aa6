"""rtgo — Python mirror of the reference's renderer interface over librtgo.so.

The reference's seam is the Go method set of ``*renderer.ParallelRenderer``
(internal/renderer/renderer.go:54-126, settings.go:3-36) plus
``scene.LoadFromFile`` (internal/scene/scene.go:45-57).  This module exposes
the same names (snake_case) on top of the C ABI in include/rt_api.h; the
compute path is the gfx950 kernel inside librtgo.so.  There is no CPU
fallback: rendering without a GPU raises ``RenderError``.

The library is loaded lazily.  When PyTorch is already imported its HIP
runtime (same soname, libamdhip64.so.7) is the one librtgo binds to, so
torch device pointers and streams can be passed to ``Context``.
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from datetime import datetime, timezone

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTGO_LIB selects an alternative build of the same library (the RT_WG_TIMING
# instrumented build of scripts/wg_timing.py); the library itself reads no
# environment variable
LIB_PATH = os.environ.get("RTGO_LIB") or os.path.join(os.path.dirname(_HERE), "build", "librtgo.so")

RT_OK = 0
RT_E_TIMEOUT = -6  # a multi-rank frame did not finish in time (rt_renderer_set_watchdog)
RT_OBJ_SPHERE, RT_OBJ_CUBE = 0, 1
MATERIAL_KINDS = {
    "lambertian": 0,
    "metal": 1,
    "shiny": 2,
    "perfectmirror": 3,
    "glass": 4,
    "dielectric": 5,
    "diffuselight": 6,
}
RT_LAYOUT_IMAGE, RT_LAYOUT_PACKED_TILES = 0, 1
RT_PATH_AUTO, RT_PATH_MEGAKERNEL = 0, 1
RT_PARTITION_AUTO, RT_PARTITION_STRIDED, RT_PARTITION_BALANCED = 0, 1, 2
SKIES = {"none": 0, "default": 1, "white": 2, "sunset": 3, "night": 4}  # RT_SKY_*
RT_COMM_ID_BYTES = 128
RT_MAX_FRAMES = 32  # frames per launch (rt_context_render_frames_async)
# wavefront kernel classes (RT_WF_*, rt_context_kernel_seconds)
WF_KERNELS = ["extend", "shade1", "occlude_hard", "cone", "softgen", "cone_rays", "occlude_soft", "shade", "regen", "resolve"]


class RenderError(RuntimeError):
    """A librtgo call failed (message from rt_last_error)."""


# --------------------------------------------------------------- C structs
class Material(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("color", ctypes.c_double * 3),
        ("roughness", ctypes.c_double),
        ("metallic", ctypes.c_double),
        ("specular", ctypes.c_double),
        ("refraction_index", ctypes.c_double),
    ]


class Object(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("position", ctypes.c_double * 3),
        ("size", ctypes.c_double * 3),
        ("radius", ctypes.c_double),
        ("material", Material),
    ]


class Light(ctypes.Structure):
    _fields_ = [
        ("position", ctypes.c_double * 3),
        ("color", ctypes.c_double * 3),
        ("intensity", ctypes.c_double),
    ]


class Camera(ctypes.Structure):
    _fields_ = [
        ("position", ctypes.c_double * 3),
        ("look_at", ctypes.c_double * 3),
        ("up", ctypes.c_double * 3),
        ("fov", ctypes.c_double),
        ("aspect_ratio", ctypes.c_double),
    ]


class SceneView(ctypes.Structure):
    _fields_ = [
        ("camera", Camera),
        ("objects", ctypes.POINTER(Object)),
        ("num_objects", ctypes.c_int32),
        ("_pad0", ctypes.c_int32),
        ("lights", ctypes.POINTER(Light)),
        ("num_lights", ctypes.c_int32),
        ("_pad1", ctypes.c_int32),
    ]


class Settings(ctypes.Structure):
    _fields_ = [
        ("samples", ctypes.c_int32),
        ("max_depth", ctypes.c_int32),
        ("anti_aliasing", ctypes.c_int32),
        ("recursive_reflections", ctypes.c_int32),
        ("soft_shadows", ctypes.c_int32),
        ("depth_of_field", ctypes.c_int32),
        ("num_workers", ctypes.c_int32),
        ("num_devices", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("sky", ctypes.c_int32),
        ("_pad2", ctypes.c_int32),
    ]


class Tuning(ctypes.Structure):
    """rt_tuning: how the same work is cut and ordered (never the image)."""

    _fields_ = [
        ("path", ctypes.c_int32),
        ("pilot", ctypes.c_int32),
        ("frustum", ctypes.c_int32),
        ("stage", ctypes.c_int32),
        ("block_work", ctypes.c_double),
        ("block_samples", ctypes.c_int32),
        ("bvh_bins", ctypes.c_int32),
        ("bvh_leaf", ctypes.c_int32),
        ("wf_paths", ctypes.c_int32),
        ("wf_chunk", ctypes.c_int64),
        ("wf_lds_nodes", ctypes.c_int32),
        ("wf_trav_block", ctypes.c_int32),
        ("wf_trav_wgs", ctypes.c_int32),
        ("pilot_depth", ctypes.c_int32),
        ("split_samples", ctypes.c_int32),
        ("measure", ctypes.c_int32),
        ("split_depth", ctypes.c_int32),
        ("partition", ctypes.c_int32),
        ("wf_list_tries", ctypes.c_int32),
        ("tail_helpers", ctypes.c_int32),
        ("tail_paths", ctypes.c_int32),
        ("tail_depth", ctypes.c_int32),
        ("tail_every", ctypes.c_int32),
        ("tail_at", ctypes.c_int32),
        ("_tail_pad", ctypes.c_int32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("render_seconds", ctypes.c_double),
        ("kernel_seconds", ctypes.c_double),
        ("rays_per_second", ctypes.c_double),
        ("pixels_per_second", ctypes.c_double),
        ("objects", ctypes.c_int32),
        ("lights", ctypes.c_int32),
        ("create_seconds", ctypes.c_double),
        ("scene_seconds", ctypes.c_double),
        ("bvh_build_seconds", ctypes.c_double),
        ("launch_seconds", ctypes.c_double),
        ("download_seconds", ctypes.c_double),
        ("destroy_seconds", ctypes.c_double),
    ]


class ContextStats(ctypes.Structure):
    """rt_context_stats (rt_context_get_stats)."""

    _fields_ = [(n, ctypes.c_int64) for n in ("schedules_built", "measuring_frames", "frames", "launches",
                                             "batched_launches", "blocks", "split_pixels", "tail_exported",
                                             "tail_errors")]


COUNT_FIELDS = [
    "camera_rays",
    "bounce_rays",
    "shadow_rays",
    "sphere_tests",
    "triangle_tests",
    "box_tests",
    "shade_events",
    "light_evals",
    "rng_draws",
]


class Counts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in COUNT_FIELDS] + [("culled", ctypes.c_uint64 * 9),
                                                               ("soft_occlusion", ctypes.c_uint64 * 9),
                                                               ("extend", ctypes.c_uint64 * 9),
                                                               ("hard_occlusion", ctypes.c_uint64 * 9)]

    def as_dict(self):
        """The nine counts (the reference's: every camera sample walked)."""
        return {n: int(getattr(self, n)) for n in COUNT_FIELDS}

    def culled_dict(self):
        """The part of each count the product never executes (culled pixels' camera samples)."""
        return {n: int(self.culled[i]) for i, n in enumerate(COUNT_FIELDS)}

    def soft_occlusion_dict(self):
        """The wavefront soft-shadow traversal kernel's share of the counts."""
        return {n: int(self.soft_occlusion[i]) for i, n in enumerate(COUNT_FIELDS)}

    def extend_dict(self):
        """The wavefront closest-hit traversal kernel's share of the counts."""
        return {n: int(self.extend[i]) for i, n in enumerate(COUNT_FIELDS)}

    def hard_occlusion_dict(self):
        """The wavefront hard-ray traversal kernel's share of the counts."""
        return {n: int(self.hard_occlusion[i]) for i, n in enumerate(COUNT_FIELDS)}

    def executed_dict(self):
        """Executed work: count - culled."""
        return {n: int(getattr(self, n)) - int(self.culled[i]) for i, n in enumerate(COUNT_FIELDS)}


# the symbols include/rt_api.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "rt_settings_default",
    "rt_abi_version",
    "rt_last_error",
    "rt_scene_load_json",
    "rt_scene_parse_json",
    "rt_scene_view",
    "rt_scene_warnings",
    "rt_scene_free",
    "rt_scene_print_hittables",
    "rt_render",
    "rt_validate",
    "rt_renderer_create",
    "rt_renderer_render",
    "rt_renderer_destroy",
    "rt_renderer_set_tuning",
    "rt_tuning_default",
    "rt_context_set_tuning",
    "rt_context_create",
    "rt_context_destroy",
    "rt_context_set_scene",
    "rt_num_tiles",
    "rt_tiles_for_rank",
    "rt_max_local_tiles",
    "rt_packed_bytes",
    "rt_packed_rgba_offset",
    "rt_context_render_async",
    "rt_unpack_tiles_async",
    "rt_comm_unique_id",
    "rt_comm_create",
    "rt_comm_destroy",
    "rt_comm_gather_tiles_async",
    "rt_context_last_kernel_seconds",
    "rt_context_set_debug_buffer",
    "rt_tonemap_rgba",
    "rt_write_png",
    "rt_write_ppm",
    "rt_partition_create",
    "rt_partition_balanced",
    "rt_partition_destroy",
    "rt_partition_world",
    "rt_partition_owner",
    "rt_partition_local_tiles",
    "rt_partition_tile",
    "rt_partition_max_local",
    "rt_partition_packed_bytes",
    "rt_partition_rgba_offset",
    "rt_partition_work",
    "rt_context_set_partition",
    "rt_unpack_partition_async",
    "rt_comm_gather_bytes_async",
    "rt_renderer_rank_seconds",
    "rt_renderer_num_ranks",
    "rt_debug_xlane_faults",
    "rt_context_tail_debug",
    "rt_context_profile",
    "rt_context_kernel_seconds",
    "rt_context_render_frames_async",
    "rt_unpack_partition_frames_async",
    "rt_release_cached_memory",
    "rt_renderer_set_watchdog",
    "rt_renderer_test_stall",
    "rt_context_get_stats",
]

_lib = None


def lib():
    """Load librtgo.so (once) and declare the C signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RenderError(
            f"{LIB_PATH} is missing: build it with `make -C concurrent-raytracer-go_amd` "
            "(or __graft_entry__.build())"
        )
    # One HIP runtime per process: torch bundles libamdhip64.so (soname
    # libamdhip64.so.7) and loads it by a path the dynamic loader cannot
    # match against an already-loaded /opt/rocm copy, so torch must come
    # first; librtgo's DT_NEEDED libamdhip64.so.7 then binds to torch's copy.
    if os.environ.get("RTGO_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
    sig = {
        "rt_settings_default": (None, [ctypes.POINTER(Settings)]),
        "rt_abi_version": (i32, []),
        "rt_last_error": (ctypes.c_char_p, []),
        "rt_scene_load_json": (ctypes.c_int, [ctypes.c_char_p, i32, ctypes.POINTER(vp)]),
        "rt_scene_parse_json": (ctypes.c_int, [ctypes.c_char_p, sz, i32, ctypes.POINTER(vp)]),
        "rt_scene_view": (ctypes.POINTER(SceneView), [vp]),
        "rt_scene_warnings": (i32, [vp]),
        "rt_scene_free": (None, [vp]),
        "rt_scene_print_hittables": (ctypes.c_int, [vp]),
        "rt_render": (
            ctypes.c_int,
            [ctypes.POINTER(SceneView), i32, i32, ctypes.POINTER(Settings), vp, vp, ctypes.POINTER(Stats)],
        ),
        "rt_validate": (ctypes.c_int, [ctypes.POINTER(SceneView), i32, i32, ctypes.POINTER(Settings)]),
        "rt_renderer_create": (ctypes.c_int, [ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]),
        "rt_renderer_render": (
            ctypes.c_int,
            [vp, ctypes.POINTER(SceneView), i32, i32, ctypes.POINTER(Settings), vp, vp, ctypes.POINTER(Stats)],
        ),
        "rt_renderer_destroy": (None, [vp]),
        "rt_renderer_set_tuning": (ctypes.c_int, [vp, ctypes.POINTER(Tuning)]),
        "rt_tuning_default": (None, [ctypes.POINTER(Tuning)]),
        "rt_context_set_tuning": (ctypes.c_int, [vp, ctypes.POINTER(Tuning)]),
        "rt_max_local_tiles": (i32, [i32, i32, i32]),
        "rt_packed_bytes": (sz, [i32, i32, i32]),
        "rt_packed_rgba_offset": (sz, [i32, i32, i32]),
        "rt_comm_unique_id": (ctypes.c_int, [vp]),
        "rt_comm_create": (ctypes.c_int, [vp, i32, i32, i32, ctypes.POINTER(vp)]),
        "rt_comm_destroy": (None, [vp]),
        "rt_comm_gather_tiles_async": (ctypes.c_int, [vp, i32, i32, vp, vp, vp]),
        "rt_context_create": (ctypes.c_int, [i32, ctypes.POINTER(vp)]),
        "rt_context_destroy": (None, [vp]),
        "rt_context_set_scene": (ctypes.c_int, [vp, ctypes.POINTER(SceneView), i32]),
        "rt_num_tiles": (i32, [i32, i32]),
        "rt_tiles_for_rank": (i32, [i32, i32, i32, i32]),
        "rt_context_render_async": (
            ctypes.c_int,
            [vp, i32, i32, ctypes.POINTER(Settings), i32, i32, i32, vp, vp, vp, ctypes.POINTER(Counts)],
        ),
        "rt_unpack_tiles_async": (ctypes.c_int, [i32, i32, i32, vp, vp, vp, vp]),
        "rt_context_last_kernel_seconds": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "rt_context_set_debug_buffer": (ctypes.c_int, [vp, vp]),
        "rt_tonemap_rgba": (None, [vp, i32, vp]),
        "rt_write_png": (ctypes.c_int, [ctypes.c_char_p, vp, i32, i32]),
        "rt_write_ppm": (ctypes.c_int, [ctypes.c_char_p, vp, i32, i32]),
        "rt_partition_create": (ctypes.c_int, [i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(vp)]),
        "rt_partition_balanced": (ctypes.c_int, [vp, i32, i32, ctypes.POINTER(Settings), i32, ctypes.POINTER(vp)]),
        "rt_partition_destroy": (None, [vp]),
        "rt_partition_world": (i32, [vp]),
        "rt_partition_owner": (i32, [vp, i32]),
        "rt_partition_local_tiles": (i32, [vp, i32]),
        "rt_partition_tile": (i32, [vp, i32, i32]),
        "rt_partition_max_local": (i32, [vp]),
        "rt_partition_packed_bytes": (sz, [vp]),
        "rt_partition_rgba_offset": (sz, [vp]),
        "rt_partition_work": (ctypes.c_double, [vp, i32]),
        "rt_context_set_partition": (ctypes.c_int, [vp, vp]),
        "rt_unpack_partition_async": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "rt_comm_gather_bytes_async": (ctypes.c_int, [vp, sz, vp, vp, vp]),
        "rt_renderer_rank_seconds": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int32]),
        "rt_renderer_num_ranks": (ctypes.c_int32, [vp]),
        "rt_debug_xlane_faults": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)]),
        "rt_context_tail_debug": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "rt_context_profile": (ctypes.c_int, [vp, i32]),
        "rt_context_render_frames_async": (
            ctypes.c_int,
            [vp, i32, i32, ctypes.POINTER(Settings), i32, ctypes.POINTER(ctypes.c_uint64), i32, i32, i32,
             ctypes.POINTER(vp), ctypes.POINTER(vp), vp],
        ),
        "rt_unpack_partition_frames_async": (ctypes.c_int, [vp, i32, vp, vp, vp, vp]),
        "rt_release_cached_memory": (ctypes.c_int, []),
        "rt_renderer_set_watchdog": (ctypes.c_int, [vp, ctypes.c_double]),
        "rt_renderer_test_stall": (ctypes.c_int, [vp, i32, ctypes.c_double]),
        "rt_context_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(ContextStats)]),
        "rt_context_kernel_seconds": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                                     ctypes.POINTER(ctypes.c_int64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RenderError(f"librtgo error {rc}: {msg.decode() if msg else ''}")


def default_settings() -> Settings:
    s = Settings()
    lib().rt_settings_default(ctypes.byref(s))
    return s


def default_tuning(**over) -> Tuning:
    t = Tuning()
    lib().rt_tuning_default(ctypes.byref(t))
    for k, v in over.items():
        setattr(t, k, v)
    return t


# --------------------------------------------------------------- scene
class Scene:
    """A loaded scene (scene.Scene, internal/scene/scene.go:12-16)."""

    def __init__(self, handle=None, objects=None, lights=None, camera=None):
        self._handle = handle
        if handle is not None:
            self._view = lib().rt_scene_view(handle).contents
        else:
            self._objects = (Object * max(1, len(objects)))(*objects)
            self._lights = (Light * max(1, len(lights)))(*lights)
            v = SceneView()
            v.camera = camera
            v.objects = ctypes.cast(self._objects, ctypes.POINTER(Object))
            v.num_objects = len(objects)
            v.lights = ctypes.cast(self._lights, ctypes.POINTER(Light))
            v.num_lights = len(lights)
            self._view = v

    @classmethod
    def load_from_file(cls, path: str) -> "Scene":
        """scene.LoadFromFile (scene.go:45-57)."""
        h = ctypes.c_void_p()
        _check(lib().rt_scene_load_json(path.encode(), 0, ctypes.byref(h)))
        return cls(handle=h)

    @classmethod
    def from_json_text(cls, text: str) -> "Scene":
        h = ctypes.c_void_p()
        b = text.encode()
        _check(lib().rt_scene_parse_json(b, len(b), 0, ctypes.byref(h)))
        return cls(handle=h)

    @classmethod
    def from_python(cls, camera: dict, objects: list, lights: list) -> "Scene":
        """Build a scene from already-decoded values (loader defaults applied)."""
        cam = Camera()
        cam.position[:] = camera.get("position", (0, 0, 0))
        cam.look_at[:] = camera.get("lookAt", (0, 0, 0))
        cam.up[:] = camera.get("up", (0, 0, 0))
        cam.fov = camera.get("fov", 0.0)
        cam.aspect_ratio = camera.get("aspectRatio", 0.0)
        objs = []
        for o in objects:
            ob = Object()
            ob.type = RT_OBJ_SPHERE if o["type"] == "sphere" else RT_OBJ_CUBE
            ob.position[:] = o.get("position", (0, 0, 0))
            ob.size[:] = o.get("size", (0, 0, 0))
            ob.radius = o.get("radius", 0.0)
            # the fields each material kind reads, with scene.go:104-148's defaults
            m = o["material"]
            t = m["type"] if m["type"] in MATERIAL_KINDS else "lambertian"
            ob.material.kind = MATERIAL_KINDS[t]
            if t != "dielectric":
                ob.material.color[:] = m.get("color", (0, 0, 0))
            if t in ("metal", "shiny", "perfectmirror"):
                ob.material.roughness = m.get("roughness", 0.0)
            if t in ("metal", "shiny"):
                ob.material.metallic = m.get("metallic", 1.0 if t == "metal" else 0.0)
                ob.material.specular = m.get("specular", 1.0)
            if t in ("glass", "dielectric"):
                ob.material.refraction_index = m.get("refractionIndex", 1.5)
            objs.append(ob)
        ls = []
        for l in lights:
            li = Light()
            li.position[:] = l["position"]
            li.color[:] = l.get("color", (0, 0, 0))
            li.intensity = l.get("intensity", 0.0)
            ls.append(li)
        return cls(objects=objs, lights=ls, camera=cam)

    @property
    def view(self) -> SceneView:
        return self._view

    @property
    def num_objects(self) -> int:
        return self._view.num_objects

    @property
    def warnings(self) -> int:
        return lib().rt_scene_warnings(self._handle) if self._handle is not None else 0

    def print_hittables(self):
        if self._handle is not None:
            lib().rt_scene_print_hittables(self._handle)

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and _lib is not None:
            _lib.rt_scene_free(h)
            self._handle = None


# --------------------------------------------------------------- renderer
class ParallelRenderer:
    """renderer.ParallelRenderer (renderer.go:20-29) backed by the GPU kernel."""

    FEATURES = [
        "Improved metallic reflections with Fresnel effect",
        "Shiny materials with configurable roughness and specular",
        "Enhanced light source reflections",
        "Better specular highlights for metallic surfaces",
    ]

    def __init__(self, num_workers: int = 1, num_devices: int = 1, devices=None):
        """devices: the device of each rank (default 0..num_devices-1; a
        device may repeat: its ranks share it)."""
        self.settings = default_settings()  # NewParallelRenderer defaults, renderer.go:54-65
        self.settings.num_workers = num_workers
        self.settings.num_devices = len(devices) if devices else num_devices
        self.devices = list(devices) if devices else None
        self.benchmark_data: dict = {}
        self.last_linear = None
        self.last_stats = None
        self._r = None  # the rt_renderer (made by the first render, kept like the Go object)
        self._tuning = None

    def set_tuning(self, tuning: Tuning):
        self._tuning = tuning
        if self._r is not None:
            _check(lib().rt_renderer_set_tuning(self._r, ctypes.byref(tuning)))

    def _renderer(self):
        if self._r is None:
            h = ctypes.c_void_p()
            if self.devices:
                devs = (ctypes.c_int32 * len(self.devices))(*self.devices)
                _check(lib().rt_renderer_create(devs, len(self.devices), ctypes.byref(h)))
            else:
                _check(lib().rt_renderer_create(None, max(1, self.settings.num_devices), ctypes.byref(h)))
            self._r = h
            if self._tuning is not None:
                _check(lib().rt_renderer_set_tuning(self._r, ctypes.byref(self._tuning)))
        return self._r

    def close(self):
        if self._r is not None and _lib is not None:
            _lib.rt_renderer_destroy(self._r)
        self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_watchdog(self, seconds: float):
        """rt_renderer_set_watchdog: bound a multi-rank Render's wait (RT_E_TIMEOUT after `seconds`)."""
        _check(lib().rt_renderer_set_watchdog(self._renderer(), float(seconds)))

    def test_stall(self, rank: int, ms: float):
        """rt_renderer_test_stall (test hook): the next multi-rank frame's rank first sleeps `ms` on the GPU."""
        _check(lib().rt_renderer_test_stall(self._renderer(), rank, float(ms)))

    # settings.go:3-25
    def set_samples(self, samples: int):
        self.settings.samples = samples

    def set_max_depth(self, max_depth: int):
        self.settings.max_depth = max_depth

    def set_anti_aliasing(self, on: bool):
        self.settings.anti_aliasing = int(on)

    def set_recursive_reflections(self, on: bool):
        self.settings.recursive_reflections = int(on)

    def set_soft_shadows(self, on: bool):
        self.settings.soft_shadows = int(on)

    def set_depth_of_field(self, on: bool):
        self.settings.depth_of_field = int(on)

    def set_seed(self, seed: int):
        self.settings.seed = seed

    def set_sky(self, sky: str):
        """Opt-in sky on miss (atmosphere.go presets); "none" = black, the reference."""
        self.settings.sky = SKIES[sky]

    def get_stats(self) -> dict:  # settings.go:27-36
        s = self.settings
        return {
            "workers": s.num_workers,
            "samples": s.samples,
            "maxDepth": s.max_depth,
            "antiAliasing": bool(s.anti_aliasing),
            "recursiveReflections": bool(s.recursive_reflections),
            "softShadows": bool(s.soft_shadows),
            "depthOfField": bool(s.depth_of_field),
        }

    def render(self, scene: Scene, width: int, height: int, keep_linear: bool = True) -> np.ndarray:
        """Render (renderer.go:67-126): returns an (H, W, 4) uint8 RGBA image.

        The mean linear radiance (before tone mapping) is kept in
        ``self.last_linear`` as an (H, W, 3) float32 array; keep_linear=False
        skips it (None), as Go's Render returns the RGBA image only.
        """
        _check(lib().rt_validate(ctypes.byref(scene.view), width, height, ctypes.byref(self.settings)))
        lin = np.zeros((height, width, 3), np.float32) if keep_linear else None
        rgba = np.zeros((height, width, 4), np.uint8)
        st = Stats()
        _check(
            lib().rt_renderer_render(
                self._renderer(),
                ctypes.byref(scene.view),
                width,
                height,
                ctypes.byref(self.settings),
                lin.ctypes.data if lin is not None else None,
                rgba.ctypes.data,
                ctypes.byref(st),
            )
        )
        self.last_linear = lin
        self.last_stats = st
        self.benchmark_data = {
            "scene_name": "demo_scene",
            "resolution": f"{width}x{height}",
            "render_time_seconds": st.render_seconds,
            "samples": self.settings.samples,
            "max_depth": self.settings.max_depth,
            "num_workers": self.settings.num_workers,
            "objects": st.objects,
            "lights": st.lights,
            "timestamp": datetime.now(timezone.utc).isoformat(),
            "features": list(self.FEATURES),
            "kernel_time_seconds": st.kernel_seconds,
            "pixels_per_second": st.pixels_per_second,
            "rays_per_second": st.rays_per_second,
        }
        return rgba

    def rank_seconds(self) -> list:
        """Device seconds of each rank's render launches in the last render (load balance)."""
        r = self._renderer()
        n = lib().rt_renderer_num_ranks(r)  # (the renderer's own count, not the mutable settings)
        out = (ctypes.c_double * max(1, n))()
        _check(lib().rt_renderer_rank_seconds(r, out, n))
        return list(out)

    def save_image(self, img: np.ndarray, filename: str):
        """SaveImage (renderer.go:438-451); '.ppm' writes a P3 PPM."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape[:2]
        f = lib().rt_write_ppm if filename.endswith(".ppm") else lib().rt_write_png
        _check(f(filename.encode(), img.ctypes.data, w, h))

    def save_benchmark_data(self, path: str):
        """SaveBenchmarkData (renderer.go:473-485)."""
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(self.benchmark_data, f, indent=2)


# --------------------------------------------------------------- device API
class Context:
    """A scene resident on one device (rt_context_*)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().rt_context_create(device, ctypes.byref(self._h)))

    def set_scene(self, scene: Scene, force_bvh: int = 0):
        self._scene = scene  # keep alive
        _check(lib().rt_context_set_scene(self._h, ctypes.byref(scene.view), force_bvh))

    def set_tuning(self, tuning: Tuning):
        _check(lib().rt_context_set_tuning(self._h, ctypes.byref(tuning)))

    def render_async(self, width, height, settings: Settings, d_linear: int, d_rgba: int, stream: int = 0,
                     rank: int = 0, world: int = 1, layout: int = RT_LAYOUT_IMAGE):
        _check(
            lib().rt_context_render_async(
                self._h, width, height, ctypes.byref(settings), rank, world, layout,
                ctypes.c_void_p(d_linear), ctypes.c_void_p(d_rgba), ctypes.c_void_p(stream), None,
            )
        )

    def count(self, width, height, settings: Settings, d_linear: int, d_rgba: int, stream: int = 0,
              rank: int = 0, world: int = 1, layout: int = RT_LAYOUT_IMAGE, full: bool = False):
        """The counting variant: the reference's nine counts (dict); full=True
        returns the Counts struct (with the culled part, Counts.culled_dict)."""
        c = Counts()
        _check(
            lib().rt_context_render_async(
                self._h, width, height, ctypes.byref(settings), rank, world, layout,
                ctypes.c_void_p(d_linear), ctypes.c_void_p(d_rgba), ctypes.c_void_p(stream), ctypes.byref(c),
            )
        )
        return c if full else c.as_dict()

    def render_frames_async(self, width, height, settings: Settings, seeds, d_linear, d_rgba=None, stream: int = 0,
                            rank: int = 0, world: int = 1, layout: int = RT_LAYOUT_IMAGE):
        """rt_context_render_frames_async: len(seeds) frames of one schedule in one launch;
        d_linear / d_rgba: per-frame device pointers (d_rgba None: no RGBA8)."""
        n = len(seeds)
        sd = (ctypes.c_uint64 * n)(*seeds)
        lp = (ctypes.c_void_p * n)(*d_linear)
        rp = (ctypes.c_void_p * n)(*d_rgba) if d_rgba is not None else None
        _check(lib().rt_context_render_frames_async(self._h, width, height, ctypes.byref(settings), n, sd, rank, world,
                                                     layout, lp, rp, ctypes.c_void_p(stream)))

    def set_partition(self, partition):
        """Render the tiles of `partition` (a Partition, or None: strided)."""
        self._partition = partition  # (copied by the library; kept for symmetry)
        _check(lib().rt_context_set_partition(self._h, partition._h if partition is not None else None))

    def balanced_partition(self, width, height, settings: Settings, world: int) -> "Partition":
        """rt_partition_balanced: a pilot-estimated, work-balanced tile partition."""
        h = ctypes.c_void_p()
        _check(lib().rt_partition_balanced(self._h, width, height, ctypes.byref(settings), world, ctypes.byref(h)))
        return Partition(_handle=h)

    def set_debug_buffer(self, d_buf: int):
        _check(lib().rt_context_set_debug_buffer(self._h, ctypes.c_void_p(d_buf)))

    def profile(self, on: bool = True):
        """Per-kernel HIP-event timing of the wavefront path (resets the totals)."""
        _check(lib().rt_context_profile(self._h, 1 if on else 0))

    def kernel_seconds(self) -> dict:
        """{kernel class: (total seconds, launches)} since profile(True)."""
        s = (ctypes.c_double * len(WF_KERNELS))()
        n = (ctypes.c_int64 * len(WF_KERNELS))()
        _check(lib().rt_context_kernel_seconds(self._h, s, n))
        return {k: (s[i], int(n[i])) for i, k in enumerate(WF_KERNELS)}

    def tail_debug(self) -> dict:
        """rt_context_tail_debug: tail-helper counters since the layout (ticks at 100 MHz)."""
        out = (ctypes.c_uint64 * 6)()
        _check(lib().rt_context_tail_debug(self._h, out))
        return dict(zip(("exported", "paths_done", "solo_ticks", "export_ticks", "helper_ticks", "err"), out))

    def stats(self) -> dict:
        """rt_context_get_stats: schedules built, measuring frames, frames, launches, batched launches;
        the last schedule's work blocks and split pixels."""
        s = ContextStats()
        _check(lib().rt_context_get_stats(self._h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in ContextStats._fields_}

    def last_kernel_seconds(self) -> float:
        s = ctypes.c_double()
        _check(lib().rt_context_last_kernel_seconds(self._h, ctypes.byref(s)))
        return s.value

    def close(self):
        if self._h:
            lib().rt_context_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def num_tiles(width: int, height: int) -> int:
    return lib().rt_num_tiles(width, height)


def tiles_for_rank(width: int, height: int, rank: int, world: int) -> int:
    return lib().rt_tiles_for_rank(width, height, rank, world)


def render(scene: Scene, width: int, height: int, settings: Settings):
    """One-shot rt_render: (rgba (H,W,4) u8, linear (H,W,3) f32, Stats)."""
    lin = np.zeros((height, width, 3), np.float32)
    rgba = np.zeros((height, width, 4), np.uint8)
    st = Stats()
    _check(lib().rt_render(ctypes.byref(scene.view), width, height, ctypes.byref(settings), lin.ctypes.data,
                           rgba.ctypes.data, ctypes.byref(st)))
    return rgba, lin, st


def max_local_tiles(width: int, height: int, world: int) -> int:
    return lib().rt_max_local_tiles(width, height, world)


def packed_bytes(width: int, height: int, world: int) -> int:
    """Bytes of one rank's packed share: float3 + RGBA8 per pixel of rank 0's tiles."""
    return lib().rt_packed_bytes(width, height, world)


def packed_rgba_offset(width: int, height: int, world: int) -> int:
    return lib().rt_packed_rgba_offset(width, height, world)


def unpack_tiles_async(width, height, world, d_gathered, d_linear, d_rgba, stream=0):
    """Scatter gathered shares [world][packed_bytes] into W*H images."""
    _check(
        lib().rt_unpack_tiles_async(
            width, height, world, ctypes.c_void_p(d_gathered), ctypes.c_void_p(d_linear), ctypes.c_void_p(d_rgba),
            ctypes.c_void_p(stream),
        )
    )


class Partition:
    """rt_partition: which rank renders each 32x32 tile (include/rt_api.h)."""

    def __init__(self, width=0, height=0, world=1, owner=None, _handle=None):
        if _handle is not None:
            self._h = _handle
            return
        self._h = ctypes.c_void_p()
        arr = None
        if owner is not None:
            owner = list(owner)
            arr = (ctypes.c_int32 * len(owner))(*owner)
        _check(lib().rt_partition_create(width, height, world, arr, ctypes.byref(self._h)))

    @property
    def world(self) -> int:
        return lib().rt_partition_world(self._h)

    def owner(self, tile: int) -> int:
        return lib().rt_partition_owner(self._h, tile)

    def owners(self, width: int, height: int) -> np.ndarray:
        return np.array([self.owner(t) for t in range(num_tiles(width, height))], np.int32)

    def local_tiles(self, rank: int) -> int:
        return lib().rt_partition_local_tiles(self._h, rank)

    def tiles(self, rank: int) -> list:
        return [lib().rt_partition_tile(self._h, rank, k) for k in range(self.local_tiles(rank))]

    @property
    def max_local(self) -> int:
        return lib().rt_partition_max_local(self._h)

    @property
    def packed_bytes(self) -> int:
        return lib().rt_partition_packed_bytes(self._h)

    @property
    def rgba_offset(self) -> int:
        return lib().rt_partition_rgba_offset(self._h)

    def work(self, rank: int) -> float:
        return lib().rt_partition_work(self._h, rank)

    def unpack_async(self, d_gathered, d_linear, d_rgba, stream=0):
        _check(lib().rt_unpack_partition_async(self._h, ctypes.c_void_p(d_gathered), ctypes.c_void_p(d_linear),
                                               ctypes.c_void_p(d_rgba), ctypes.c_void_p(stream)))

    def unpack_frames_async(self, nframes, d_gathered, d_linear, d_rgba, stream=0):
        """[world][nframes][packed bytes] -> [nframes][W*H] images."""
        _check(lib().rt_unpack_partition_frames_async(self._h, nframes, ctypes.c_void_p(d_gathered),
                                                      ctypes.c_void_p(d_linear), ctypes.c_void_p(d_rgba),
                                                      ctypes.c_void_p(stream)))

    def close(self):
        if self._h and _lib is not None:
            _lib.rt_partition_destroy(self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """rt_comm: the RCCL communicator of one process per GPU (rank 0 makes
    the id with ``unique_id()``; the caller broadcasts it)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES)()
        _check(lib().rt_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid: bytes, world: int, rank: int, device: int):
        buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES)(*uid)
        self._h = ctypes.c_void_p()
        _check(lib().rt_comm_create(buf, world, rank, device, ctypes.byref(self._h)))

    def gather_bytes_async(self, share_bytes, d_share, d_gathered, stream=0):
        _check(lib().rt_comm_gather_bytes_async(self._h, share_bytes, ctypes.c_void_p(d_share),
                                                ctypes.c_void_p(d_gathered), ctypes.c_void_p(stream)))

    def gather_tiles_async(self, width, height, d_share, d_gathered, stream=0):
        _check(lib().rt_comm_gather_tiles_async(self._h, width, height, ctypes.c_void_p(d_share),
                                                ctypes.c_void_p(d_gathered), ctypes.c_void_p(stream)))

    def close(self):
        if self._h:
            lib().rt_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

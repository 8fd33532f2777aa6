"""ctypes wrapper of the CPU oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product (concurrent-raytracer-go_amd/).
The oracle is a plain-C restatement of the reference's Go hot path (see
oracle.c for the file:line map).  Parity pinning: the reference's own known
answers (internal/math/vector_test.go, math_benchmarks_test.go) plus
hand-derived known answers; whole-image results are "parity unpinned" at the
reference level (no Go toolchain here, no reference goldens — SURVEY.md §4).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

_lib = None
# Worker threads of a render without an explicit count: None = the affinity
# count (Go's runtime.NumCPU()).  The test suite caps it (tests/conftest.py)
# to stay inside a GPU box's CPU share; bench.py passes its count explicitly.
DEFAULT_THREADS = None


def _rtgo():
    import sys

    pkg = os.path.join(os.path.dirname(_HERE), "concurrent-raytracer-go_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    import rtgo

    return rtgo


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
    rt = _rtgo()
    L = ctypes.CDLL(LIB_PATH)
    d3 = ctypes.c_double * 3
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    L.oracle_render.restype = ctypes.c_int
    L.oracle_render.argtypes = [
        ctypes.POINTER(rt.SceneView), i32, i32, ctypes.POINTER(rt.Settings), i32, i32, i32, i32, vp, vp,
        ctypes.POINTER(rt.Counts),
    ]
    L.oracle_render_ex.restype = ctypes.c_int
    L.oracle_render_ex.argtypes = L.oracle_render.argtypes + [i32]
    L.oracle_go_pow.restype = ctypes.c_double
    L.oracle_go_pow.argtypes = [ctypes.c_double, ctypes.c_double]
    L.oracle_go_max.restype = ctypes.c_double
    L.oracle_go_max.argtypes = [ctypes.c_double, ctypes.c_double]
    L.oracle_go_min.restype = ctypes.c_double
    L.oracle_go_min.argtypes = [ctypes.c_double, ctypes.c_double]
    L.oracle_tonemap.restype = None
    L.oracle_tonemap.argtypes = [d3, d3]
    L.oracle_to_rgb.restype = None
    L.oracle_to_rgb.argtypes = [d3, ctypes.c_uint8 * 3]
    L.oracle_vec_op.restype = None
    L.oracle_vec_op.argtypes = [ctypes.c_int, d3, d3, ctypes.c_double, d3]
    L.oracle_vec_dot.restype = ctypes.c_double
    L.oracle_vec_dot.argtypes = [d3, d3]
    L.oracle_vec_length.restype = ctypes.c_double
    L.oracle_vec_length.argtypes = [d3]
    L.oracle_sphere_hit.restype = ctypes.c_int
    L.oracle_sphere_hit.argtypes = [d3, ctypes.c_double, d3, d3, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double * 8]
    L.oracle_triangle_hit.restype = ctypes.c_int
    L.oracle_triangle_hit.argtypes = [d3, d3, d3, d3, d3, ctypes.c_double, ctypes.c_double, ctypes.c_double * 8]
    L.oracle_scatter.restype = ctypes.c_int
    L.oracle_scatter.argtypes = [ctypes.POINTER(rt.Material), d3, d3, ctypes.c_double * 8, ctypes.c_uint64,
                                 ctypes.c_uint32, ctypes.c_uint32, i32, ctypes.c_double * 6,
                                 ctypes.POINTER(i32)]
    L.oracle_rng_draws.restype = None
    L.oracle_rng_draws.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, i32, vp, vp]
    L.oracle_soft_points.restype = None
    L.oracle_soft_points.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, vp, ctypes.POINTER(i32)]
    L.oracle_path_lengths.restype = ctypes.c_int
    L.oracle_path_lengths.argtypes = [ctypes.POINTER(rt.SceneView), i32, i32, ctypes.POINTER(rt.Settings), i32, vp]
    L.oracle_cube_triangles.restype = None
    L.oracle_cube_triangles.argtypes = [d3, d3, ctypes.c_double * 108]
    _lib = L
    return L


def d3(v):
    return (ctypes.c_double * 3)(*v)


def render(scene, width, height, settings, rank=0, world=1, nthreads=None, max_tiles=-1, counts=False, bvh=False):
    """Render with the oracle. Returns (linear float64 (H,W,3), rgba uint8 (H,W,4), counts|None).

    bvh=True: the secondary CPU baseline (sphere BVH + any-hit shadow rays,
    oracle_render_ex) -- the same image, not the reference's algorithm; its
    counts are not the reference's either."""
    rt = _rtgo()
    if nthreads is None and DEFAULT_THREADS:
        nthreads = DEFAULT_THREADS
    if nthreads is None:
        # the CPUs this process may run on: Go's runtime.NumCPU(), the worker
        # count cmd/raytracer passes to NewParallelRenderer (main.go:46)
        try:
            nthreads = len(os.sched_getaffinity(0))
        except AttributeError:
            nthreads = os.cpu_count() or 1
    lin = np.full((height, width, 3), np.nan, np.float64)
    rgba = np.zeros((height, width, 4), np.uint8)
    c = rt.Counts()
    rc = lib().oracle_render_ex(
        ctypes.byref(scene.view), width, height, ctypes.byref(settings), rank, world, nthreads, max_tiles,
        lin.ctypes.data, rgba.ctypes.data, ctypes.byref(c), 1 if bvh else 0,
    )
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return lin, rgba, (c.as_dict() if counts else None)


def path_lengths(scene, width, height, settings, nthreads=None):
    """Bounces of every sample's path, uint8 (H, W, spp) (clamped at 255):
    scheduling analysis (scripts/path_stats.py), no image."""
    nthreads = nthreads or len(os.sched_getaffinity(0))
    out = np.zeros((height, width, settings.samples), np.uint8)
    rc = lib().oracle_path_lengths(ctypes.byref(scene.view), width, height, ctypes.byref(settings), nthreads,
                                   out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oracle_path_lengths failed: {rc}")
    return out


def go_pow(x, y):
    return lib().oracle_go_pow(x, y)


def go_max(x, y):
    return lib().oracle_go_max(x, y)


def go_min(x, y):
    return lib().oracle_go_min(x, y)


def tonemap(c):
    out = d3((0, 0, 0))
    lib().oracle_tonemap(d3(c), out)
    return tuple(out)


def to_rgb(c):
    out = (ctypes.c_uint8 * 3)()
    lib().oracle_to_rgb(d3(c), out)
    return tuple(out)


VEC_OPS = {"add": 0, "sub": 1, "mul": 2, "cross": 3, "normalize": 4, "reflect": 5, "refract": 6, "clamp": 7}


def vec_op(op, a, b=(0, 0, 0), eta=0.0):
    out = d3((0, 0, 0))
    lib().oracle_vec_op(VEC_OPS[op], d3(a), d3(b), eta, out)
    return tuple(out)


def dot(a, b):
    return lib().oracle_vec_dot(d3(a), d3(b))


def length(a):
    return lib().oracle_vec_length(d3(a))


def sphere_hit(center, radius, o, d, tmin, tmax):
    rec = (ctypes.c_double * 8)()
    ok = lib().oracle_sphere_hit(d3(center), radius, d3(o), d3(d), tmin, tmax, rec)
    return (tuple(rec) if ok else None)


def triangle_hit(v0, v1, v2, o, d, tmin, tmax):
    rec = (ctypes.c_double * 8)()
    ok = lib().oracle_triangle_hit(d3(v0), d3(v1), d3(v2), d3(o), d3(d), tmin, tmax, rec)
    return (tuple(rec) if ok else None)


def scatter(material, ray_o, ray_d, rec, seed=1, pixel=0, sample=0, skip=0):
    out = (ctypes.c_double * 6)()
    draws = ctypes.c_int32()
    r = (ctypes.c_double * 8)(*rec)
    ok = lib().oracle_scatter(ctypes.byref(material), d3(ray_o), d3(ray_d), r, seed, pixel, sample, skip, out,
                              ctypes.byref(draws))
    return bool(ok), tuple(out[:3]), tuple(out[3:]), draws.value


def rng_draws(seed, pixel, sample, n):
    vals = np.zeros(n, np.float64)
    raw = np.zeros(n, np.uint64)
    lib().oracle_rng_draws(seed, pixel, sample, n, vals.ctypes.data, raw.ctypes.data)
    return vals, raw


def soft_points(seed, pixel, sample, depth, light):
    """(16x3 points, tries) of the soft-shadow stream of (pixel, sample, depth, light), spec v4."""
    pts = np.zeros((16, 3), np.float64)
    t = ctypes.c_int32()
    lib().oracle_soft_points(seed, pixel, sample, depth, light, pts.ctypes.data, ctypes.byref(t))
    return pts, int(t.value)


def cube_triangles(position, size):
    out = (ctypes.c_double * 108)()
    lib().oracle_cube_triangles(d3(position), d3(size), out)
    return np.array(out[:]).reshape(12, 3, 3)

"""Oracle known answers (CPU): pins the C restatement (oracle/oracle.c).

Two kinds of pins:
  * the reference's own known answers — internal/math/vector_test.go:8-105
    (Add, Sub, Dot, Cross, Length, Normalize, Reflect, Clamp, ToRGB) and
    internal/math/math_benchmarks_test.go:126-165 (TestVectorMathAccuracy);
  * hand-derived answers of the Go formulas on the hot path:
    Sphere.Hit / Triangle.Hit t values and records (sphere.go:22-59,
    triangle.go:36-88), Metal's Fresnel attenuation (material.go:75-113),
    the Glass reflect / refract branch (advanced_materials.go:21-46), the
    tone map (renderer.go:348-367) and Go's math.Pow / Max / Min semantics.
Expected values are computed here in Python binary64 with the reference's
operation order, so most comparisons are exact.
"""
import math

import numpy as np
import pytest

import oracle

NAN = float("nan")


def same(a, b):
    """Bitwise-equal doubles (NaN == NaN, +0 != -0)."""
    return np.array(a, np.float64).tobytes() == np.array(b, np.float64).tobytes()


# ---------------------------------------------------------------- vector_test.go
def test_vec3_add_sub_dot_cross():  # vector_test.go:8-49
    assert oracle.vec_op("add", (1, 2, 3), (4, 5, 6)) == (5, 7, 9)
    assert oracle.vec_op("sub", (5, 7, 9), (1, 2, 3)) == (4, 5, 6)
    assert oracle.dot((1, 2, 3), (4, 5, 6)) == 32.0
    assert oracle.vec_op("cross", (1, 0, 0), (0, 1, 0)) == (0, 0, 1)


def test_vec3_length_normalize_reflect_clamp():  # vector_test.go:51-94
    assert abs(oracle.length((3, 4, 0)) - 5.0) <= 1e-10
    n = oracle.vec_op("normalize", (3, 4, 0))
    assert max(abs(n[0] - 0.6), abs(n[1] - 0.8), abs(n[2])) <= 1e-10
    r = oracle.vec_op("reflect", (1, -1, 0), (0, 1, 0))
    assert max(abs(r[0] - 1), abs(r[1] - 1), abs(r[2])) <= 1e-10
    assert oracle.vec_op("clamp", (-1, 0.5, 2)) == (0, 0.5, 1)


def test_vec3_to_rgb_truncates():  # vector_test.go:96-105
    assert oracle.to_rgb((0.5, 0.25, 1.0)) == (127, 63, 255)


def test_vector_math_accuracy():  # math_benchmarks_test.go:126-165
    a, b = (1.0, 2.0, 3.0), (4.0, 5.0, 6.0)
    assert oracle.vec_op("add", a, b) == (5.0, 7.0, 9.0)
    assert oracle.vec_op("sub", a, b) == (-3.0, -3.0, -3.0)
    assert oracle.vec_op("mul", a, b) == (4.0, 10.0, 18.0)
    assert abs(oracle.dot(a, b) - 32.0) <= 1e-10
    assert oracle.vec_op("cross", a, b) == (-3.0, 6.0, -3.0)
    assert abs(oracle.length(a) - math.sqrt(14.0)) <= 1e-10


def test_normalize_zero_stays_zero():  # vector.go Normalize: length 0 -> zero vector
    assert oracle.vec_op("normalize", (0, 0, 0)) == (0, 0, 0)


def test_refract_straight_through_and_total_internal_reflection():  # vector.go:81-96
    # normal incidence: direction unchanged (scaled by eta, minus n*(eta*ct + c2))
    assert oracle.vec_op("refract", (0, 0, -1), (0, 0, 1), eta=1 / 1.5) == pytest.approx((0, 0, -1), abs=1e-15)
    # grazing from the dense side: sin2 > 1 -> Reflect
    s = 0.8
    v = (s, 0.0, -math.sqrt(1 - s * s))
    got = oracle.vec_op("refract", v, (0, 0, 1), eta=1.5)
    assert got == oracle.vec_op("reflect", v, (0, 0, 1))


# ---------------------------------------------------------------- Go math
def test_go_pow_integer_exponents_and_specials():
    assert oracle.go_pow(2.0, 10.0) == 1024.0
    assert oracle.go_pow(0.7, 5.0) == 0.7 * ((0.7 * 0.7) * (0.7 * 0.7))  # Go: repeated squaring
    assert oracle.go_pow(5.0, 0.0) == 1.0
    assert oracle.go_pow(1.0, NAN) == 1.0
    assert math.isnan(oracle.go_pow(-8.0, 1 / 3))
    assert oracle.go_pow(0.0, 1 / 2.2) == 0.0
    x = 0.3
    assert oracle.go_pow(x, 1 / 2.2) == pytest.approx(x ** (1 / 2.2), rel=1e-15)


def test_go_max_min_nan_and_signed_zero():
    assert math.isnan(oracle.go_max(NAN, 1.0)) and math.isnan(oracle.go_max(1.0, NAN))
    assert math.isnan(oracle.go_min(NAN, 1.0)) and math.isnan(oracle.go_min(1.0, NAN))
    assert oracle.go_max(math.inf, NAN) == math.inf  # Go checks +Inf before NaN
    assert oracle.go_min(-math.inf, NAN) == -math.inf
    assert same(oracle.go_max(-0.0, 0.0), 0.0) and same(oracle.go_max(0.0, -0.0), 0.0)
    assert same(oracle.go_min(-0.0, 0.0), -0.0) and same(oracle.go_min(0.0, -0.0), -0.0)


def test_tonemap_and_nan_pixel():  # renderer.go:348-367, vector.go:106-109
    assert oracle.tonemap((0.0, 100.0, math.log(2.0))) == (0.0, 1.0, pytest.approx(0.5 ** (1 / 2.2), rel=1e-15))
    t = oracle.tonemap((-1.0, 0.0, 0.0))  # negative radiance: Pow(neg, 1/2.2) = NaN, Max/Min keep it
    assert math.isnan(t[0])
    assert oracle.to_rgb((NAN, 0.0, 1.0)) == (0, 0, 255)  # uint8(NaN) = 0 on amd64 (CVTTSD2SQ)


# ---------------------------------------------------------------- geometry
def test_sphere_hit_near_root_front_face():  # sphere.go:22-58
    rec = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), 0.001, math.inf)
    assert rec == (4.0, 0.0, 0.0, -4.0, 0.0, 0.0, 1.0, 1.0)


def test_sphere_hit_far_root_back_face_and_range():
    rec = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), 4.5, math.inf)
    # second root t=6, outward normal (0,0,-1) faces along the ray -> flipped, front=false
    assert rec == (6.0, 0.0, 0.0, -6.0, 0.0, 0.0, 1.0, 0.0)
    assert oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), 0.001, 3.9) is None
    assert oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 1, 0), 0.001, math.inf) is None


def test_sphere_hit_unnormalized_direction():  # getRay directions are not normalized
    rec = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -2), 0.001, math.inf)
    assert rec[:4] == (2.0, 0.0, 0.0, -4.0)


def test_sphere_boundary_equality_passes():  # equality passes `root < tMin || tMax < root`
    rec = oracle.sphere_hit((0, 0, -5), 1.0, (0, 0, 0), (0, 0, -1), 0.001, 4.0)
    assert rec is not None and rec[0] == 4.0


def test_triangle_hit_and_misses():  # triangle.go:36-82
    v0, v1, v2 = (-1, -1, -5), (1, -1, -5), (0, 1, -5)
    rec = oracle.triangle_hit(v0, v1, v2, (0, 0, 0), (0, 0, -1), 0.001, math.inf)
    assert rec == (5.0, 0.0, 0.0, -5.0, 0.0, 0.0, 1.0, 1.0)
    # from behind: normal flipped toward the ray, front=false
    rec = oracle.triangle_hit(v0, v1, v2, (0, 0, -10), (0, 0, 1), 0.001, math.inf)
    assert rec == (5.0, 0.0, 0.0, -5.0, 0.0, 0.0, -1.0, 0.0)
    assert oracle.triangle_hit(v0, v1, v2, (0, 0, 0), (1, 0, 0), 0.001, math.inf) is None  # parallel
    assert oracle.triangle_hit(v0, v1, v2, (5, 5, 0), (0, 0, -1), 0.001, math.inf) is None  # outside
    assert oracle.triangle_hit(v0, v1, v2, (0, 0, 0), (0, 0, -1), 0.001, 4.0) is None  # beyond tMax


def test_cube_triangles_follow_create_cube():  # scene.go:150-190
    pos, size = (1.0, -2.0, 3.0), (2.0, 4.0, 6.0)
    h = [s / 2.0 for s in size]
    sg = [(-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (-1, -1, 1), (1, -1, 1), (1, 1, 1), (-1, 1, 1)]
    v = [tuple(pos[k] + s[k] * h[k] for k in range(3)) for s in sg]
    faces = [(0, 1, 2, 3), (1, 5, 6, 2), (5, 4, 7, 6), (4, 0, 3, 7), (3, 2, 6, 7), (4, 5, 1, 0)]
    want = []
    for f in faces:
        want.append([v[f[0]], v[f[1]], v[f[2]]])
        want.append([v[f[0]], v[f[2]], v[f[3]]])
    assert np.array_equal(oracle.cube_triangles(pos, size), np.array(want))


# ---------------------------------------------------------------- materials
def _mat(kind, color=(0, 0, 0), roughness=0.0, metallic=0.0, specular=0.0, ior=1.5):
    import rtgo

    m = rtgo.Material()
    m.kind = rtgo.MATERIAL_KINDS[kind]
    m.color[:] = color
    m.roughness, m.metallic, m.specular, m.refraction_index = roughness, metallic, specular, ior
    return m


def _pow5(x):  # Go math.Pow(x, 5)
    return x * ((x * x) * (x * x))


def test_metal_fresnel_attenuation():  # material.go:75-113
    col = (0.8, 0.6, 0.2)
    m = _mat("metal", col, roughness=0.0, metallic=1.0)
    s = 1 / math.sqrt(2.0)
    d = (s, -s, 0.0)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), d, (1, 0, 0, 0, 0, 1, 0, 1))
    assert ok and draws == 0  # roughness 0: no perturbation draw
    f0 = ((1.5 - 1.0) / (1.5 + 1.0)) ** 2
    cos_t = abs(d[0] * 0 + d[1] * 1 + d[2] * 0)
    F = f0 + (1.0 - f0) * _pow5(1.0 - cos_t)
    fs = 0.6 + 1.0 * 0.4
    mf = 0.4 + 1.0 * 0.5
    want = []
    for c in col:
        a = max(0.0, min(1.0, c * (1.0 - fs) + F * fs))
        want.append(a * (1.0 - mf) + F * mf)
    assert att == tuple(want)
    assert nd == pytest.approx((s, s, 0.0), abs=1e-16)


def test_glass_refract_and_reflect_branches():  # advanced_materials.go:21-46
    m = _mat("glass", (0.9, 0.95, 1.0), ior=1.5)
    rec = (1, 0, 0, 0, 0, 0, 1, 1)  # front face, N = +Z
    # normal incidence: reflectance R = r0 = 0.04; the branch is `R > draw`
    r0 = ((1 - 1 / 1.5) / (1 + 1 / 1.5)) ** 2
    vals, _ = oracle.rng_draws(1, 7, 3, 400)
    refr = next(i for i, v in enumerate(vals) if not r0 > v)
    refl = next(i for i, v in enumerate(vals) if r0 > v)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), (0, 0, -1), rec, 1, 7, 3, skip=refr)
    assert ok and draws == 1 and att == (0.9, 0.95, 1.0)
    assert nd == pytest.approx((0, 0, -1), abs=1e-15)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), (0, 0, -1), rec, 1, 7, 3, skip=refl)
    assert draws == 1 and nd == (0.0, 0.0, 1.0)


def test_glass_total_internal_reflection_draws_nothing():
    m = _mat("glass", (1, 1, 1), ior=1.5)
    s = 0.8
    d = (s, 0.0, -math.sqrt(1 - s * s))
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), d, (1, 0, 0, 0, 0, 0, 1, 0))  # back face: ratio = 1.5
    assert ok and draws == 0  # cannotRefract short-circuits the reflectance draw
    assert nd == pytest.approx((0.8, 0.0, 0.6), abs=1e-15)


def test_dielectric_attenuation_is_white():  # material.go:235-260
    m = _mat("dielectric", (0.1, 0.2, 0.3), ior=1.33)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), (0, 0, -1), (1, 0, 0, 0, 0, 0, 1, 1))
    assert ok and att == (1.0, 1.0, 1.0)


def test_lambertian_direction_from_rejection_draws():  # material.go:26-35, vector.go:132-139
    m = _mat("lambertian", (0.5, 0.5, 0.5))
    N = (0.0, 1.0, 0.0)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), (0, -1, 0), (1, 0, 0, 0) + N + (1,), 5, 11, 2)
    vals, _ = oracle.rng_draws(5, 11, 2, 300)
    i = 0
    while True:
        p = [vals[i + k] * 2 - 1 for k in range(3)]
        i += 3
        if p[0] * p[0] + p[1] * p[1] + p[2] * p[2] < 1:
            break
    sd = [N[k] + p[k] for k in range(3)]
    ln = math.sqrt(sd[0] * sd[0] + sd[1] * sd[1] + sd[2] * sd[2])
    assert ok and draws == i and att == (0.5, 0.5, 0.5)
    assert nd == tuple(x / ln for x in sd)


def test_diffuse_light_does_not_scatter():  # material.go:296-298
    ok, nd, att, draws = oracle.scatter(_mat("diffuselight", (4, 4, 4)), (0, 0, 0), (0, 0, -1),
                                        (1, 0, 0, 0, 0, 0, 1, 1))
    assert not ok and draws == 0


def test_perfect_mirror_blend_uses_folded_constant():  # advanced_materials.go:125-151
    col = (0.8, 0.5, 0.2)
    m = _mat("perfectmirror", col, roughness=0.0)
    ok, nd, att, draws = oracle.scatter(m, (0, 0, 0), (0, 0, -1), (1, 0, 0, 0, 0, 0, 1, 1))
    f0 = ((2.0 - 1.0) / (2.0 + 1.0)) ** 2
    F = f0 + (1.0 - f0) * _pow5(1.0 - 1.0)
    # Go folds the untyped constant (1.0 - 0.9) to exactly float64(0.1)
    assert ok and draws == 0 and att == tuple(c * 0.1 + F * 0.9 for c in col)


def _go_sky(preset, d):
    """GetSkyColor (internal/atmosphere/atmosphere.go:100-135) restated in
    Python, FastVec3* as the Vec3 methods (a.Lerp(b, t) = a + (b - a) t)."""
    import math

    P = {  # atmosphere.go:28-98: top, bottom, sun dir, sun colour, sun intensity, size, rayleigh, mie, depth,
        #    fog density, fog colour, time of day
        1: ((0.6, 0.8, 1.0), (0.9, 0.95, 1.0), (0.0, 0.8, -0.6), (1.0, 0.98, 0.95), 1.2, 0.015, (0.6, 0.8, 1.0),
            (1.0, 0.98, 0.95), 0.3, 0.0, (0.9, 0.92, 0.95), 0.6),
        3: ((1.0, 0.4, 0.2), (1.0, 0.8, 0.6), (0.0, 0.3, -0.9), (1.0, 0.6, 0.3), 1.2, 0.03, (1.0, 0.4, 0.2),
            (1.0, 0.8, 0.6), 0.8, 0.1, (1.0, 0.8, 0.6), 0.8),
    }[preset]
    top, bot, sd, sc, si_, ss, ray, mie, depth_k, fog, fogc, tod = P
    lerp = lambda a, b, t: tuple(x + (y - x) * t for x, y in zip(a, b))  # noqa: E731
    ln = math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])
    u = tuple(x / ln for x in d)
    c = lerp(bot, top, 0.5 * (u[1] + 1.0))
    atm = math.exp(-max(0.0, u[1]) * depth_k)
    c = lerp(c, lerp(ray, mie, atm), 0.25)
    dot = u[0] * sd[0] + u[1] * sd[1] + u[2] * sd[2]
    if dot > 1.0 - ss:
        s = min((dot - (1.0 - ss)) / ss ** 1.0, 1e300) ** 1.5
        c = lerp(c, sc, min(s, 1.0) * si_ * 0.9)
    tf = tod if tod <= 0.5 else 1.0 - tod
    c = tuple(x * (1.0 - tf * 2.0 * 0.3) for x in c)
    if fog > 0:
        c = lerp(fogc, c, math.exp(-fog))
    return tuple(max(0.1, min(0.98, x)) for x in c)


@pytest.mark.parametrize("preset", [1, 3])
@pytest.mark.parametrize("d", [(0, 1, 0), (0, -1, 0), (0.3, 0.2, -1), (0.0, 0.8, -0.6), (0.0, 0.31, -0.9),
                               (1e-3, 0.8, -0.6)])
def test_sky_color_matches_restatement(preset, d):
    import ctypes

    out = (ctypes.c_double * 3)()
    oracle.lib().oracle_sky_color.argtypes = [ctypes.c_int, ctypes.c_double * 3, ctypes.c_double * 3]
    oracle.lib().oracle_sky_color(preset, (ctypes.c_double * 3)(*d), out)
    want = _go_sky(preset, d)
    assert max(abs(a - b) for a, b in zip(out, want)) < 1e-14, (tuple(out), want)

"""Pure-Python statement of the random stream spec v4 (include/rt_rng.h):
v3's per-sample stream, plus v4's soft-shadow streams.

Independent of the C code: used to check the oracle's stream and to make
the committed known-answer vectors (tests/golden/make_rng_vectors.py).
"""
M64 = (1 << 64) - 1
MULT = 6364136223846793005
INC = 1442695040888963407


def mix64(z):  # SplitMix64 finaliser
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def init(seed, pixel, sample):
    return mix64(mix64(seed & M64) ^ (((pixel & 0xFFFFFFFF) << 32) | (sample & 0xFFFFFFFF)))


def out(x):  # PCG-XSH-RR output of a state
    xs = (((x >> 18) ^ x) >> 27) & 0xFFFFFFFF
    rot = x >> 59
    return ((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF


def step(x):
    return (x * MULT + INC) & M64


def draws(seed, pixel, sample, n):
    """(raw 32-bit outputs, doubles out * 2^-32) of the first n draws."""
    x = init(seed, pixel, sample)
    raw, vals = [], []
    for _ in range(n):
        r = out(x)
        x = step(x)
        raw.append(r)
        vals.append(r * 2.0**-32)
    return raw, vals


def jump(j):
    """(A_j, C_j) with x_{i+j} = A_j x_i + C_j mod 2^64."""
    a, c = 1, 0
    for _ in range(j):
        c = (c * MULT + INC) & M64
        a = (a * MULT) & M64
    return a, c


SOFT_TAG = 0x5F0F7A11E5EED5A1


def soft_init(seed, pixel, sample, depth, light):
    """v4: the state of the soft-shadow stream of (pixel, sample, depth, light)."""
    k = mix64(mix64(seed & M64) ^ SOFT_TAG ^ (((pixel & 0xFFFFFFFF) << 32) | (sample & 0xFFFFFFFF)))
    return mix64(k ^ (((depth & 0xFFFFFFFF) << 32) | (light & 0xFFFFFFFF)))


def soft_draws(seed, pixel, sample, depth, light, n):
    x = soft_init(seed, pixel, sample, depth, light)
    raw = []
    for _ in range(n):
        raw.append(out(x))
        x = step(x)
    return raw


def soft_points(seed, pixel, sample, depth, light):
    """calculateSmartShadow's 16 accepted RandomVec3InUnitSphere points of one
    (sample, bounce, light) and the tries taken (binary64 arithmetic of the
    kernel: 2 u - 1 per axis from u = raw * 2^-32, accepted when |p|^2 < 1)."""
    x = soft_init(seed, pixel, sample, depth, light)
    pts, tries = [], 0
    while len(pts) < 16:
        r = []
        for _ in range(3):
            r.append(out(x))
            x = step(x)
        tries += 1
        p = [v * 2.0**-32 * 2 - 1 for v in r]
        if p[0] * p[0] + p[1] * p[1] + p[2] * p[2] < 1:
            pts.append(tuple(p))
    return pts, tries

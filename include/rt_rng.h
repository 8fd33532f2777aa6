/*
 * rt_rng.h — the counter-keyed random stream shared (as a SPEC) by the CPU
 * oracle (oracle/oracle.c) and the gfx950 kernel.
 *
 * Why a new generator: the reference draws from Go's global math/rand
 * (internal/math/random.go:8-14), shared across goroutines and unseedable
 * under go 1.24 (rand.Seed is a no-op), so its draw order depends on the
 * goroutine schedule.  Bit-level parity with a Go run is
 * impossible; parity is defined against the oracle, which consumes exactly
 * the same draws as the kernel because both key the stream by
 * (seed, pixel, sample) — never by tile, rank or thread.
 *
 * Spec (v3, kept by v4 below): one PCG32 stream (O'Neill 2014, PCG-XSH-RR 64/32) per sample.
 *   key0    = mix64(seed)                               (once per render)
 *   x_0     = mix64(key0 ^ (pixel << 32 | sample))      pixel = y*W + x
 *   x_{i+1} = x_i * 6364136223846793005 + 1442695040888963407   (mod 2^64)
 *   out_i   = rotr32((uint32)(((x_i >> 18) ^ x_i) >> 27), x_i >> 59)
 *   draw_i  = out_i * 2^-32   (uniform on [0,1), 32 random bits, exact in
 *             binary64; the Go equivalent is rand.Float64(), random.go:12-14)
 * mix64 is the SplitMix64 finaliser.  Why PCG: the LCG state jumps ahead in
 * O(1) — x_{i+j} = A_j x_i + C_j — so the kernel can evaluate later draws
 * of a stream on other lanes (cooperative rejection sampling, DESIGN.md
 * §Kernels) and still consume exactly this sequence.
 *
 * The draw ORDER is the reference's call order:
 * per sample u, v (renderer.go:155-156); per bounce, for every light whose
 * hard shadow ray is unoccluded, 16 RandomVec3InUnitSphere
 * (renderer.go:315-316, vector.go:132-139: 3 draws per rejection try);
 * then the material's scatter draws.
 *
 * Spec v4 (round 5): the 16 soft-shadow points of one (sample, bounce,
 * light) draw from a stream of their own, not from the sample's stream:
 *   y_0 = mix64(mix64(key0 ^ RT_SOFT_TAG ^ (pixel << 32 | sample))
 *               ^ (depth << 32 | light))          depth = traceRay's depth
 * then the same PCG steps and outputs, 3 draws per rejection try until 16
 * points are accepted.  The sample's stream carries u, v and the scatter
 * draws only.  Why: a light whose 16 soft rays cannot be blocked (nothing
 * in their shadow cone) needs its points only to advance the sample's
 * stream; with a stream of their own, the kernels skip those ~31 tries per
 * (hit, light) -- a third of the headline kernel's time --
 * and a cone's points can be drawn by any lane in any order.  The
 * reference's draws are a global stream shared by every goroutine
 * (random.go:8-14), so which generator state feeds which call was never
 * reproducible; every draw is still an independent uniform draw, and the
 * rejection sampling, its 3 draws per try and the points are the
 * reference's.
 */
#ifndef RT_RNG_H
#define RT_RNG_H

#include <stdint.h>
#include <string.h>

#if defined(__HIP__) || defined(__HIPCC__)
#define RT_RNG_FN static inline __host__ __device__
#else
#define RT_RNG_FN static inline
#endif

#define RT_PCG_MULT 6364136223846793005ULL
#define RT_PCG_INC 1442695040888963407ULL

typedef struct {
  uint64_t x;
} rt_rng;

RT_RNG_FN uint64_t rt_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

RT_RNG_FN uint64_t rt_rng_seed_key(uint64_t seed) { return rt_mix64(seed); }

RT_RNG_FN void rt_rng_init(rt_rng* r, uint64_t seed_key, uint32_t pixel, uint32_t sample) {
  r->x = rt_mix64(seed_key ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
}

/* v4: the soft-shadow stream of (pixel, sample, depth, light), in two steps:
 * the sample's soft key (once per sample), then the stream of a bounce's light */
#define RT_SOFT_TAG 0x5F0F7A11E5EED5A1ULL
RT_RNG_FN uint64_t rt_soft_key(uint64_t seed_key, uint32_t pixel, uint32_t sample) {
  return rt_mix64(seed_key ^ RT_SOFT_TAG ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
}
RT_RNG_FN uint64_t rt_soft_state(uint64_t soft_key, uint32_t depth, uint32_t light) {
  return rt_mix64(soft_key ^ (((uint64_t)depth << 32) | (uint64_t)light));
}

/* PCG-XSH-RR output of a state value */
RT_RNG_FN uint32_t rt_pcg_out(uint64_t x) {
  const uint32_t xs = (uint32_t)(((x >> 18) ^ x) >> 27);
  const uint32_t rot = (uint32_t)(x >> 59);
  return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

RT_RNG_FN uint32_t rt_rng_next(rt_rng* r) {
  const uint64_t old = r->x;
  r->x = old * RT_PCG_MULT + RT_PCG_INC;
  return rt_pcg_out(old);
}

/* x * 2^-32, built from the bits: 1.x (x in the top 32 mantissa bits) - 1 */
RT_RNG_FN double rt_bits_to_unit(uint32_t x) {
  const uint64_t b = 0x3FF0000000000000ULL | ((uint64_t)x << 20);
  double d;
#if defined(__HIP_DEVICE_COMPILE__)
  d = __builtin_bit_cast(double, b);
#else
  memcpy(&d, &b, sizeof d);
#endif
  return d - 1.0;
}

RT_RNG_FN double rt_rng_draw(rt_rng* r) { return rt_bits_to_unit(rt_rng_next(r)); }

/* Jump coefficients: x_{i+j} = A_j * x_i + C_j (mod 2^64). */
RT_RNG_FN void rt_pcg_jump_coeffs(uint32_t j, uint64_t* A, uint64_t* C) {
  uint64_t a = 1, c = 0;
  for (uint32_t k = 0; k < j; ++k) {
    c = c * RT_PCG_MULT + RT_PCG_INC;
    a = a * RT_PCG_MULT;
  }
  *A = a;
  *C = c;
}

#endif /* RT_RNG_H */

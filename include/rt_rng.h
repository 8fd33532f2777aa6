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
 * Spec (v2):
 *   key0   = mix64(seed)                                (once per render)
 *   k      = mix64(key0 ^ (pixel << 32 | sample))       pixel = y*W + x
 *   b      = mix64(k + G)                               G = 0x9E3779B97F4A7C15
 *   state  = (lo32(k), hi32(k), lo32(b), hi32(b)); an all-zero state gets s0 = 1
 *   next() = xoshiro128** (Blackman & Vigna 2018): out = rotl(s1*5, 7)*9,
 *            then the standard update with t = s1 << 9 and rotl(s3, 11)
 *   draw() = next() * 2^-32   (uniform on [0,1), 32 random bits; exact in
 *            binary64; the Go equivalent is rand.Float64(), random.go:12-14)
 * mix64 is the SplitMix64 finaliser.  Every operation of next() is a 32-bit
 * integer op (full-rate VALU on CDNA4), which is why this generator was
 * chosen over 64-bit-state ones.
 *
 * The draw ORDER is the reference's call order:
 * per sample u, v (renderer.go:155-156); per bounce, for every light whose
 * hard shadow ray is unoccluded, 16 RandomVec3InUnitSphere
 * (renderer.go:315-316, vector.go:132-139: 3 draws per rejection try);
 * then the material's scatter draws.
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

#define RT_RNG_GAMMA 0x9E3779B97F4A7C15ULL

typedef struct {
  uint32_t s0, s1, s2, s3;
} rt_rng;

RT_RNG_FN uint64_t rt_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

RT_RNG_FN uint64_t rt_rng_seed_key(uint64_t seed) { return rt_mix64(seed); }

RT_RNG_FN void rt_rng_init(rt_rng* r, uint64_t seed_key, uint32_t pixel, uint32_t sample) {
  const uint64_t k = rt_mix64(seed_key ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
  const uint64_t b = rt_mix64(k + RT_RNG_GAMMA);
  r->s0 = (uint32_t)k;
  r->s1 = (uint32_t)(k >> 32);
  r->s2 = (uint32_t)b;
  r->s3 = (uint32_t)(b >> 32);
  r->s0 |= (uint32_t)((r->s0 | r->s1 | r->s2 | r->s3) == 0);
}

RT_RNG_FN uint32_t rt_rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

RT_RNG_FN uint32_t rt_rng_next(rt_rng* r) {
  const uint32_t result = rt_rotl32(r->s1 * 5u, 7) * 9u;
  const uint32_t t = r->s1 << 9;
  r->s2 ^= r->s0;
  r->s3 ^= r->s1;
  r->s1 ^= r->s2;
  r->s0 ^= r->s3;
  r->s2 ^= t;
  r->s3 = rt_rotl32(r->s3, 11);
  return result;
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

#endif /* RT_RNG_H */

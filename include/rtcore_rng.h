/*
 * rtcore_rng.h -- the shared, seeded, counter-based random stream of the path tracer.
 *
 * Why this exists: the reference draws every random number from an unseeded
 * System.Random per worker thread (RaytracerCore/Raytracing/Raytracer.cs:48), so its
 * per-sample output is not reproducible and no fixture can pin it.  This header
 * DEFINES the stream both the GPU kernels and the CPU oracle consume, so that a
 * sample of pixel (x, y) with index s makes the same decisions on both sides.
 *
 * Stream definition (normative):
 *   key   = splitmix64( splitmix64( splitmix64(seed) + pixel ) + sample )
 *           pixel  = y * frame_width + x   (whole-frame index, independent of tiling)
 *           sample = sample_base + s       (the s-th sample rendered for this pixel)
 *   draw n (n = 0, 1, 2, ...):
 *           h = lowbias32( (lo32(key) + n * 0x9E3779B9) ^ hi32(key) )    (mod 2^32)
 *           U = (h >> 8) * 2^-24            in [0, 1 - 2^-24]
 *   i.e. one hash round of a Weyl sequence whose offset and mask are the per-sample key.
 * U has 24 significant bits, so it is exact in float and in double: the fp32 kernel
 * and the fp64 oracle see bit-identical uniforms.  Draws are consumed in the
 * reference's order: camera subX, subY, [dof radius, angle],
 * then per bounce [pow draw unless shininess is +inf], theta, [rayRand], [acos, theta].
 *
 * Plain C99 + optional HIP qualifiers; no dependencies.
 */
#ifndef RTCORE_RNG_H
#define RTCORE_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define RT_HD static inline
#endif

#ifdef __cplusplus
extern "C" {
#endif

RT_HD uint64_t rt_splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

RT_HD uint32_t rt_lowbias32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

typedef struct rt_rng {
    uint32_t k0; /* lo32(key) + n * 0x9E3779B9 for the next draw n */
    uint32_t k1; /* hi32(key) */
} rt_rng;

/* The key factors as seed_key = splitmix64(seed), pixel_key = splitmix64(seed_key + pixel),
 * key = splitmix64(pixel_key + sample): a kernel hoists the first two out of its sample loop. */
RT_HD uint64_t rt_rng_pixel_key(uint64_t seed_key, uint64_t pixel) { return rt_splitmix64(seed_key + pixel); }

RT_HD rt_rng rt_rng_from_pixel_key(uint64_t pixel_key, uint64_t sample)
{
    uint64_t k = rt_splitmix64(pixel_key + sample);
    rt_rng r;
    r.k0 = (uint32_t)k;
    r.k1 = (uint32_t)(k >> 32);
    return r;
}

RT_HD uint64_t rt_rng_key(uint64_t seed, uint64_t pixel, uint64_t sample)
{
    return rt_splitmix64(rt_rng_pixel_key(rt_splitmix64(seed), pixel) + sample);
}

RT_HD rt_rng rt_rng_init(uint64_t seed, uint64_t pixel, uint64_t sample)
{
    return rt_rng_from_pixel_key(rt_rng_pixel_key(rt_splitmix64(seed), pixel), sample);
}

/* 24-bit draw as an integer in [0, 2^24). */
RT_HD uint32_t rt_rng_next24(rt_rng* r)
{
    uint32_t h = rt_lowbias32(r->k0 ^ r->k1);
    r->k0 += 0x9E3779B9u;
    return h >> 8;
}

RT_HD double rt_rng_next_double(rt_rng* r) { return (double)rt_rng_next24(r) * (1.0 / 16777216.0); }
RT_HD float rt_rng_next_float(rt_rng* r) { return (float)rt_rng_next24(r) * (1.0f / 16777216.0f); }

#ifdef __cplusplus
}
#endif

#endif /* RTCORE_RNG_H */

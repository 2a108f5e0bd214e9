/*
 * rtcore_rng.h -- the shared, seeded random stream of the path tracer (keyed by seed, pixel, sample).
 *
 * Why this exists: the reference draws every random number from an unseeded
 * System.Random per worker thread (RaytracerCore/Raytracing/Raytracer.cs:48), so its
 * per-sample output is not reproducible and no fixture can pin it.  This header
 * DEFINES the stream both the GPU kernels and the CPU oracle consume, so that a
 * sample of pixel (x, y) with index s makes the same decisions on both sides.
 *
 * Stream definition (normative; all arithmetic mod 2^32, H = lowbias32 below):
 *   seed key   s0 = H(lo32(seed) + 0x9E3779B9),   s1 = H(hi32(seed) ^ 0x85EBCA6B ^ s0)
 *   pixel key  p0 = H(lo32(pixel) ^ s0),           p1 = H(hi32(pixel) + p0 + s1)
 *              pixel  = y * frame_width + x   (whole-frame index, independent of tiling)
 *   sample state  x = ( H(lo32(sample) ^ p0) ^ (p1 + hi32(sample) * 0x9E3779B9) ) | 1
 *              sample = sample_base + s       (the s-th sample rendered for this pixel)
 *   draw n (n = 0, 1, 2, ...): one xorshift32 step (Marsaglia 2003, shifts 13, 17, 5) of x,
 *              x ^= x << 13;  x ^= x >> 17;  x ^= x << 5
 *              U = (x >> 8) * 2^-24            in [0, 1 - 2^-24]
 *   i.e. a hashed per-sample start (odd, so never the xorshift's fixed point 0) and a
 *   full-period (2^32 - 1) shift-register sequence from it; shifts and xors only per draw, and
 *   a kernel hoists the seed and pixel keys out of its sample loop.
 *   (Rounds 1-5 drew h = H((k0 + n * 0x9E3779B9) ^ k1) from a two-word sample key: two multiplies
 *   more per draw and one more hash per sample.  The per-draw hash was ~12 % of the brute-force
 *   kernels' VALU cycles; this stream took C2 17.89 -> 16.72 ms and C3 23.6 -> 21.7 ms in one
 *   call, profiles/r06/ab_rng.log.  tests/test_oracle.py checks uniformity and the lag-1 and
 *   cross-sample correlations, and tests/test_oracle_pin.py pins the renders to the reference's
 *   screenshots.)
 * U has 24 significant bits, so it is exact in float and in double: the fp32 kernel
 * and the fp64 oracle see bit-identical uniforms.  Draws are consumed in the
 * reference's order: camera subX, subY, [dof radius, angle],
 * then per bounce [pow draw unless shininess is +inf], theta, [rayRand], [acos, theta].
 *
 * Plain C99 + optional HIP qualifiers; no dependencies.
 */
#ifndef RTCORE_RNG_H
#define RTCORE_RNG_H

#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define RT_HD static inline
#endif

#ifdef __cplusplus
extern "C" {
#endif

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
    uint32_t x; /* xorshift32 state: the sample state, then one step per draw */
} rt_rng;

typedef struct rt_key2 {
    uint32_t a, b;
} rt_key2;

RT_HD rt_key2 rt_rng_seed_key(uint64_t seed)
{
    rt_key2 k;
    k.a = rt_lowbias32((uint32_t)seed + 0x9E3779B9u);
    k.b = rt_lowbias32((uint32_t)(seed >> 32) ^ 0x85EBCA6Bu ^ k.a);
    return k;
}

RT_HD rt_key2 rt_rng_pixel_key(rt_key2 seed_key, uint64_t pixel)
{
    rt_key2 k;
    k.a = rt_lowbias32((uint32_t)pixel ^ seed_key.a);
    k.b = rt_lowbias32((uint32_t)(pixel >> 32) + k.a + seed_key.b);
    return k;
}

RT_HD rt_rng rt_rng_from_pixel_key(rt_key2 pixel_key, uint64_t sample)
{
    rt_rng r;
    r.x = (rt_lowbias32((uint32_t)sample ^ pixel_key.a) ^ (pixel_key.b + (uint32_t)(sample >> 32) * 0x9E3779B9u)) | 1u;
    return r;
}

RT_HD rt_rng rt_rng_init(uint64_t seed, uint64_t pixel, uint64_t sample)
{
    return rt_rng_from_pixel_key(rt_rng_pixel_key(rt_rng_seed_key(seed), pixel), sample);
}

/* 24-bit draw as an integer in [0, 2^24). */
RT_HD uint32_t rt_rng_next24(rt_rng* r)
{
    uint32_t x = r->x;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    r->x = x;
    return x >> 8;
}

RT_HD double rt_rng_next_double(rt_rng* r) { return (double)rt_rng_next24(r) * (1.0 / 16777216.0); }
RT_HD float rt_rng_next_float(rt_rng* r) { return (float)rt_rng_next24(r) * (1.0f / 16777216.0f); }

#ifdef __cplusplus
}
#endif

#endif /* RTCORE_RNG_H */

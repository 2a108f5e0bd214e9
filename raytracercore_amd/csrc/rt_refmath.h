// rt_refmath.h -- fp64 Vec4D / Mat4x4D arithmetic in the reference's rounding order,
// shared by the host-side scene preparation and the exact (fp64) device kernel.
//
// The reference runs its AVX2+FMA paths (Vectors/SIMDHelpers.cs:15); these helpers
// restate the summation orders of Vec4D.Dot (Vec4D.cs:343-349), SIMDHelpers.Dot/PreDot
// ((x+y)+(z+w), SIMDHelpers.cs:70-100), SIMDHelpers.Normalize (:332-335), the FMA cross
// (:44-61) and Mat x Vec (Sum4, :111-125,220-235).  Compile with -ffp-contract=off: the
// only fused operations are the explicit fma() calls.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "rt_internal.h"

#define RT_HDI __host__ __device__ inline

namespace rtc {

RT_HDI Vec4d v4d(double x, double y, double z, double w) { return Vec4d{x, y, z, w}; }
RT_HDI Vec4d add(Vec4d a, Vec4d b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
RT_HDI Vec4d sub(Vec4d a, Vec4d b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
RT_HDI Vec4d mul(Vec4d a, Vec4d b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
RT_HDI Vec4d scale(Vec4d a, double s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
RT_HDI Vec4d divs(Vec4d a, double s) { return {a.x / s, a.y / s, a.z / s, a.w / s}; }
RT_HDI Vec4d neg(Vec4d a) { return {-a.x, -a.y, -a.z, -a.w}; }
RT_HDI bool eq3(Vec4d a, Vec4d b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
// Vec4D.Dot / SquaredLength: left-to-right scalar sums.
RT_HDI double dot_s(Vec4d a, Vec4d b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
RT_HDI double sqlen_s(Vec4d a) { return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w; }
// hadd order used by SIMDHelpers.Dot / Add2(PreDot)
RT_HDI double hsum(Vec4d a) { return (a.x + a.y) + (a.z + a.w); }
RT_HDI double dot_v(Vec4d a, Vec4d b) { return hsum(mul(a, b)); }
// Vec4D.Cross (scalar, W = 0)
RT_HDI Vec4d cross_s(Vec4d a, Vec4d b)
{
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x, 0.0};
}
// SIMDHelpers.Cross: fmsub(leftA, rightA, leftB * rightB)
RT_HDI Vec4d cross_fma(Vec4d l, Vec4d r)
{
    return {fma(l.y, r.z, -(l.z * r.y)), fma(l.z, r.x, -(l.x * r.z)), fma(l.x, r.y, -(l.y * r.x)),
            fma(l.w, r.w, -(l.w * r.w))};
}
RT_HDI Vec4d normalize_v(Vec4d v)
{
    Vec4d s = mul(v, v);
    double len = sqrt((s.x + s.y) + (s.z + s.w));
    return {v.x / len, v.y / len, v.z / len, v.w / len};
}
RT_HDI double length_s(Vec4d a) { return sqrt(sqlen_s(a)); }
RT_HDI Vec4d fma4(double s, Vec4d d, Vec4d o) { return {fma(s, d.x, o.x), fma(s, d.y, o.y), fma(s, d.z, o.z), fma(s, d.w, o.w)}; }
// Mat4x4D * Vec4D (Sum4 order)
RT_HDI Vec4d mat_vec(const double* m, Vec4d v)
{
    double o[4];
    for (int r = 0; r < 4; r++) {
        double p0 = m[r * 4 + 0] * v.x, p1 = m[r * 4 + 1] * v.y, p2 = m[r * 4 + 2] * v.z, p3 = m[r * 4 + 3] * v.w;
        o[r] = (p0 + p1) + (p2 + p3);
    }
    return {o[0], o[1], o[2], o[3]};
}
// .NET Core 3.x Math.Min / Math.Max
RT_HDI double net_min(double a, double b)
{
    if (a != b) return (a == a) ? (a < b ? a : b) : a;
    return signbit(a) ? a : b;
}
RT_HDI double net_max(double a, double b)
{
    if (a != b) return (a == a) ? (b < a ? a : b) : a;
    return signbit(b) ? a : b;
}
// SSE maxpd / minpd lane semantics (second operand unless the first compares greater/less)
RT_HDI double sse_max(double a, double b) { return a > b ? a : b; }
RT_HDI double sse_min(double a, double b) { return a < b ? a : b; }

// AABB.IntersectAVX (AABB.cs:107-142).  Returns false (and NaNs) on a miss.
RT_HDI bool aabb_hit_ref(Vec4d mn, Vec4d mx, Vec4d o, Vec4d d, double& nr, double& fr)
{
    const double os[4] = {o.x, o.y, o.z, o.w}, ds[4] = {d.x, d.y, d.z, d.w};
    const double lo[4] = {mn.x, mn.y, mn.z, mn.w}, hi[4] = {mx.x, mx.y, mx.z, mx.w};
    double n[4], f[4];
    const double inf = __builtin_huge_val();
    for (int i = 0; i < 4; i++) {
        bool mask = (ds[i] == 0) && (os[i] >= lo[i]) && (os[i] <= hi[i]);
        double l = mask ? -inf : lo[i], h = mask ? inf : hi[i];
        bool ng = signbit(ds[i]);
        double lm = ng ? h : l, hm = ng ? l : h;
        double inv = 1.0 / ds[i];
        n[i] = (lm - os[i]) * inv;
        f[i] = (hm - os[i]) * inv;
    }
    double nn = sse_max(sse_max(n[0], n[2]), sse_max(n[1], n[3]));
    double ff = sse_min(sse_min(f[0], f[2]), sse_min(f[1], f[3]));
    if ((nn > ff) | (ff < 0)) {
        nr = fr = __builtin_nan("");
        return false;
    }
    nr = nn;
    fr = ff;
    return true;
}

} // namespace rtc

// oracle_math.h -- fp64 vector / matrix arithmetic with the reference's rounding order.
// TEST INFRASTRUCTURE (see oracle.h).  Every operation names the reference code whose
// summation order / FMA use it restates; compile with -ffp-contract=off so that the only
// fused operations are the explicit std::fma calls mirroring Fma.* intrinsics.
#pragma once
#include <cmath>
#include <cstdint>
#include <limits>

namespace orc {

static const double kInf = std::numeric_limits<double>::infinity();
static const double kNaN = std::numeric_limits<double>::quiet_NaN();
// Math.PI and Consts.RAD2DEG (Consts.cs:9).
static const double kPi = 3.14159265358979323846;
static const double kRad2Deg = kPi / 180.0;

// Vec4D (Vectors/Vec4D.cs); scalar arithmetic (SIMDArithmetic = false, :20-21).
struct V4 {
    double x, y, z, w;
};
inline V4 v4(double x, double y, double z, double w) { return V4{x, y, z, w}; }
inline V4 operator+(V4 a, V4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline V4 operator-(V4 a, V4 b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline V4 operator*(V4 a, V4 b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
inline V4 operator*(V4 a, double s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline V4 operator/(V4 a, double s) { return {a.x / s, a.y / s, a.z / s, a.w / s}; }
inline V4 operator-(V4 a) { return {-a.x, -a.y, -a.z, -a.w}; }
// Vec4D.operator== compares X, Y, Z only (Vec4D.cs:464-481).
inline bool eq3(V4 a, V4 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
// Vec4D.Dot scalar: X*X' + Y*Y' + Z*Z' + W*W' left to right (Vec4D.cs:343-349).
inline double dot(V4 a, V4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
// Vec4D.SquaredLength / Length scalar (Vec4D.cs:274-315).
inline double sqlen(V4 a) { return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w; }
inline double length(V4 a) { return std::sqrt(sqlen(a)); }
// Vec4D.Cross scalar (Vec4D.cs:357-366).
inline V4 cross(V4 a, V4 b)
{
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x, 0.0};
}
// SIMDHelpers.Cross: Fma.MultiplySubtract(leftA, rightA, leftB*rightB) with the
// YZXW / ZXYW permutes (SIMDHelpers.cs:44-61).  The W lane keeps fma(w,w',-(w*w')).
inline V4 cross_fma(V4 l, V4 r)
{
    return {std::fma(l.y, r.z, -(l.z * r.y)), std::fma(l.z, r.x, -(l.x * r.z)),
            std::fma(l.x, r.y, -(l.y * r.x)), std::fma(l.w, r.w, -(l.w * r.w))};
}
// Horizontal sum in hadd order: (x+y)+(z+w) (SIMDHelpers.Add2(PreDot), :70-100).
inline double hsum(V4 a) { return (a.x + a.y) + (a.z + a.w); }
inline double dot_simd(V4 a, V4 b) { return hsum(a * b); }
// SIMDHelpers.Normalize: v / sqrt(Sum4(v*v)) (SIMDHelpers.cs:133-143,261-264,332-335).
inline V4 normalize(V4 v)
{
    V4 s = v * v;
    double len = std::sqrt((s.x + s.y) + (s.z + s.w));
    return {v.x / len, v.y / len, v.z / len, v.w / len};
}
// .NET Core 3.x Math.Min / Math.Max (IEEE 754:2019 minimum / maximum).
inline double net_min(double a, double b)
{
    if (a != b) {
        if (!std::isnan(a)) return a < b ? a : b;
        return a;
    }
    return std::signbit(a) ? a : b;
}
inline double net_max(double a, double b)
{
    if (a != b) {
        if (!std::isnan(a)) return b < a ? a : b;
        return a;
    }
    return std::signbit(b) ? a : b;
}
inline V4 vmin(V4 a, V4 b) { return {net_min(a.x, b.x), net_min(a.y, b.y), net_min(a.z, b.z), net_min(a.w, b.w)}; }
inline V4 vmax(V4 a, V4 b) { return {net_max(a.x, b.x), net_max(a.y, b.y), net_max(a.z, b.z), net_max(a.w, b.w)}; }
// SSE maxpd / minpd lane semantics: the second operand unless the first compares greater/less.
inline double sse_max(double a, double b) { return a > b ? a : b; }
inline double sse_min(double a, double b) { return a < b ? a : b; }

// Mat4x4D row-major D00..D33 (Vectors/Mat4x4D.cs).
struct M4 {
    double d[16];
};
inline M4 identity4()
{
    M4 m{};
    m.d[0] = m.d[5] = m.d[10] = m.d[15] = 1.0;
    return m;
}
inline bool meq(const M4& a, const M4& b)
{
    for (int i = 0; i < 16; i++)
        if (!(a.d[i] == b.d[i])) return false;
    return true;
}
// Mat4x4D * Mat4x4D via Vector<double>.Dot of a row and a column (Mat4x4D.cs:99-124),
// taken as the AVX vmulpd + hadd + 128-bit add order (p0+p1)+(p2+p3).
inline M4 mmul(const M4& a, const M4& b)
{
    M4 r;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            double p0 = a.d[y * 4 + 0] * b.d[0 * 4 + x], p1 = a.d[y * 4 + 1] * b.d[1 * 4 + x];
            double p2 = a.d[y * 4 + 2] * b.d[2 * 4 + x], p3 = a.d[y * 4 + 3] * b.d[3 * 4 + x];
            r.d[y * 4 + x] = (p0 + p1) + (p2 + p3);
        }
    return r;
}
// Mat4x4D * Vec4D = SIMDHelpers.MultiplyMatrixVector: Sum4 of the row products
// (SIMDHelpers.cs:111-125,220-235): component = (r0*v0 + r1*v1) + (r2*v2 + r3*v3).
inline V4 mvmul(const M4& m, V4 v)
{
    double o[4];
    for (int r = 0; r < 4; r++) {
        double p0 = m.d[r * 4 + 0] * v.x, p1 = m.d[r * 4 + 1] * v.y;
        double p2 = m.d[r * 4 + 2] * v.z, p3 = m.d[r * 4 + 3] * v.w;
        o[r] = (p2 + p3) + (p0 + p1);
    }
    return {o[0], o[1], o[2], o[3]};
}
inline M4 transpose3x3(const M4& m)
{
    M4 r{};
    r.d[0] = m.d[0]; r.d[1] = m.d[4]; r.d[2] = m.d[8];
    r.d[4] = m.d[1]; r.d[5] = m.d[5]; r.d[6] = m.d[9];
    r.d[8] = m.d[2]; r.d[9] = m.d[6]; r.d[10] = m.d[10];
    r.d[15] = 1.0;
    return r;
}
// MatrixTransforms (Vectors/MatrixTransforms.cs).
inline M4 m_translate(double x, double y, double z)
{
    M4 m = identity4();
    m.d[3] = x; m.d[7] = y; m.d[11] = z;
    return m;
}
inline M4 m_scale(double x, double y, double z)
{
    M4 m{};
    m.d[0] = x; m.d[5] = y; m.d[10] = z; m.d[15] = 1.0;
    return m;
}
inline M4 m_rotate(double angle, V4 a)
{
    double c = std::cos(angle), s = std::sin(angle), co = 1 - c;
    M4 m{};
    m.d[0] = c + a.x * a.x * co;       m.d[1] = a.x * a.y * co - a.z * s; m.d[2] = a.x * a.z * co + a.y * s;
    m.d[4] = a.y * a.x * co + a.z * s; m.d[5] = c + a.y * a.y * co;       m.d[6] = a.y * a.z * co - a.x * s;
    m.d[8] = a.z * a.x * co - a.y * s; m.d[9] = a.z * a.y * co + a.x * s; m.d[10] = c + a.z * a.z * co;
    m.d[15] = 1.0;
    return m;
}

// DoubleColor (DoubleColor.cs).
struct Col {
    double r, g, b;
};
inline Col col(double v) { return {v, v, v}; }
inline Col operator+(Col a, Col b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
inline Col operator*(Col a, Col b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
inline Col operator*(Col a, double s) { return {a.r * s, a.g * s, a.b * s}; }
inline bool ceq(Col a, Col b) { return a.r == b.r && a.g == b.g && a.b == b.b; }
inline double lum(Col c) { return 0.299 * c.r + 0.587 * c.g + 0.114 * c.b; } // DoubleColor.cs:76-79

// Ray (Vectors/Ray.cs).
struct Ray {
    V4 o, d;
};
inline Ray ray_directional(V4 o, V4 d) { return {o, normalize(d)}; }
inline V4 ray_point(const Ray& r, double t) { return r.o + r.d * t; }

} // namespace orc

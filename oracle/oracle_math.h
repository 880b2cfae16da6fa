// oracle_math.h — TEST INFRASTRUCTURE ONLY (see oracle/README.md).
//
// CPU restatement of the reference's scalar/vector/matrix arithmetic with the
// exact operation order of the reference (no FMA contraction: the oracle is
// built with -ffp-contract=off).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may use the oracle, never the product path.
//
// Citations: Math/Vector.h, Math/MathFunc.h, Math/float4x4.h, Math/Frame.h,
// Math/half.h, Math/Compression.h of the reference (Ilinite/CudaTracerLib).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cfloat>
#include <climits>

namespace oracle {

#define O_PI 3.14159265358979f          // MathFunc.h:12
#define O_INV_PI (1.0f / O_PI)          // MathFunc.h:13

// --- scalar helpers (MathFunc.h:83-90: min/max are (a<b)?a:b) -------------
template <class T> static inline T omin(T a, T b) { return (a < b) ? a : b; }
template <class T> static inline T omax(T a, T b) { return (a > b) ? a : b; }
static inline float as_float(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }
static inline int32_t as_int(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }
static inline uint32_t as_uint(float f) { uint32_t i; std::memcpy(&i, &f, 4); return i; }
// copysignf host restatement (MathFunc.h:66-69)
static inline float o_copysign(float a, float b) {
    return as_float((as_int(b) & (int32_t)0x80000000) | (as_int(a) & ~(int32_t)0x80000000));
}
static inline float frac(float f) { return f - floorf(f); }                 // MathFunc.h:138-141
static inline int floor2int(float v) { return (int)floorf(v); }            // MathFunc.h:143-145

// Transcendentals: correctly-rounded fp32 obtained through fp64 evaluation.
// The reference's own two paths already disagree here (host libm sinf vs
// CUDA __sinf / sincosf, MathFunc.h:272-288); both the oracle and the HIP
// kernels pin the correctly-rounded result so they agree bit for bit.
static inline float cr_sin(float x) { return (float)std::sin((double)x); }
static inline float cr_cos(float x) { return (float)std::cos((double)x); }
static inline float cr_tan(float x) { return (float)std::tan((double)x); }
static inline float cr_acos(float x) { return (float)std::acos((double)x); }
static inline float cr_atan2(float y, float x) { return (float)std::atan2((double)y, (double)x); }
static inline float cr_atan(float x) { return (float)std::atan((double)x); }
static inline float cr_exp(float x) { return (float)std::exp((double)x); }
static inline float cr_log(float x) { return (float)std::log((double)x); }
static inline float cr_log2(float x) { return (float)std::log2((double)x); }
static inline float cr_pow(float a, float b) { return (float)std::pow((double)a, (double)b); }

// --- vectors (Vector.h VectorBase: component-wise ops, dot/lenSqr start at 0)
struct V2 { float x, y; };
struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };

static inline V2 v2(float x, float y) { return {x, y}; }
static inline V3 v3(float x, float y, float z) { return {x, y, z}; }
static inline V3 v3s(float s) { return {s, s, s}; }
static inline V4 v4(float x, float y, float z, float w) { return {x, y, z, w}; }
static inline V4 v4(V3 a, float w) { return {a.x, a.y, a.z, w}; }
static inline V3 xyz(V4 a) { return {a.x, a.y, a.z}; }

static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 operator*(float s, V3 a) { return a * s; }                // Vector.h:384
static inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline V2 operator+(V2 a, V2 b) { return {a.x + b.x, a.y + b.y}; }
static inline V2 operator-(V2 a, V2 b) { return {a.x - b.x, a.y - b.y}; }
static inline V2 operator*(V2 a, float s) { return {a.x * s, a.y * s}; }
static inline V2 operator*(float s, V2 a) { return a * s; }

static inline float dot(V3 a, V3 b) {                                       // Vector.h:97
    float r = 0.0f; r += a.x * b.x; r += a.y * b.y; r += a.z * b.z; return r;
}
static inline float dot(V4 a, V4 b) {
    float r = 0.0f; r += a.x * b.x; r += a.y * b.y; r += a.z * b.z; r += a.w * b.w; return r;
}
static inline float lenSqr(V3 a) {                                          // Vector.h:46
    float r = 0.0f; r += a.x * a.x; r += a.y * a.y; r += a.z * a.z; return r;
}
static inline float length(V3 a) { return sqrtf(lenSqr(a)); }
static inline float rcp(float a) { return a ? 1.0f / a : 0.0f; }            // MathFunc.h:399
static inline V3 normalize(V3 a) { return a * rcp(length(a)); }            // Vector.h:369-372
static inline V3 cross(V3 a, V3 b) {                                        // Vector.h:329
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline float absdot(V3 a, V3 b) { return fabsf(dot(a, b)); }
static inline V3 vmin(V3 a, V3 b) { return {omin(a.x, b.x), omin(a.y, b.y), omin(a.z, b.z)}; }
static inline V3 vmax(V3 a, V3 b) { return {omax(a.x, b.x), omax(a.y, b.y), omax(a.z, b.z)}; }
static inline float vget(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(V3& a, int i, float f) { if (i == 0) a.x = f; else if (i == 1) a.y = f; else a.z = f; }

// --- float4x4 (float4x4.h): row-major data[i*4+j] --------------------------
struct M44 {
    float d[16];
    float operator()(int i, int j) const { return d[i * 4 + j]; }
    float& operator()(int i, int j) { return d[i * 4 + j]; }
    V4 row(int i) const { return {d[i * 4 + 0], d[i * 4 + 1], d[i * 4 + 2], d[i * 4 + 3]}; }
    V4 col(int j) const { return {d[0 * 4 + j], d[1 * 4 + j], d[2 * 4 + j], d[3 * 4 + j]}; }
    void setRow(int i, V4 r) { d[i * 4 + 0] = r.x; d[i * 4 + 1] = r.y; d[i * 4 + 2] = r.z; d[i * 4 + 3] = r.w; }
    void setCol(int j, V4 c) { d[0 * 4 + j] = c.x; d[1 * 4 + j] = c.y; d[2 * 4 + j] = c.z; d[3 * 4 + j] = c.w; }
    static M44 zeros() { M44 m; for (int i = 0; i < 16; i++) m.d[i] = 0; return m; }
    static M44 identity() { M44 m = zeros(); m.d[0] = m.d[5] = m.d[10] = m.d[15] = 1.0f; return m; }
};
static inline V4 mul(const M44& m, V4 v) {                                 // float4x4.h:377-385
    return {dot(m.row(0), v), dot(m.row(1), v), dot(m.row(2), v), dot(m.row(3), v)};
}
static inline M44 matmul(const M44& a, const M44& b) {                     // operator% float4x4.h:368-375
    M44 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r(i, j) = dot(a.row(i), b.col(j));
    return r;
}
static inline V3 transformPoint(const M44& m, V3 p) {                      // float4x4.h:398-402
    V4 f = mul(m, v4(p, 1.0f));
    return xyz(f) / f.w;
}
static inline V3 transformDirection(const M44& m, V3 d) {                  // float4x4.h:404-408
    V4 f = mul(m, v4(d, 0.0f));
    return xyz(f);
}
static inline M44 inverse(const M44& Q) {                                  // float4x4.h:132-190
    float m00 = Q(0, 0), m01 = Q(0, 1), m02 = Q(0, 2), m03 = Q(0, 3);
    float m10 = Q(1, 0), m11 = Q(1, 1), m12 = Q(1, 2), m13 = Q(1, 3);
    float m20 = Q(2, 0), m21 = Q(2, 1), m22 = Q(2, 2), m23 = Q(2, 3);
    float m30 = Q(3, 0), m31 = Q(3, 1), m32 = Q(3, 2), m33 = Q(3, 3);
    float v0 = m20 * m31 - m21 * m30;
    float v1 = m20 * m32 - m22 * m30;
    float v2 = m20 * m33 - m23 * m30;
    float v3 = m21 * m32 - m22 * m31;
    float v4 = m21 * m33 - m23 * m31;
    float v5 = m22 * m33 - m23 * m32;
    float t00 = +(v5 * m11 - v4 * m12 + v3 * m13);
    float t10 = -(v5 * m10 - v2 * m12 + v1 * m13);
    float t20 = +(v4 * m10 - v2 * m11 + v0 * m13);
    float t30 = -(v3 * m10 - v1 * m11 + v0 * m12);
    float invDet = 1 / (t00 * m00 + t10 * m01 + t20 * m02 + t30 * m03);
    float d00 = t00 * invDet, d10 = t10 * invDet, d20 = t20 * invDet, d30 = t30 * invDet;
    float d01 = -(v5 * m01 - v4 * m02 + v3 * m03) * invDet;
    float d11 = +(v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    float d21 = -(v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    float d31 = +(v3 * m00 - v1 * m01 + v0 * m02) * invDet;
    v0 = m10 * m31 - m11 * m30;
    v1 = m10 * m32 - m12 * m30;
    v2 = m10 * m33 - m13 * m30;
    v3 = m11 * m32 - m12 * m31;
    v4 = m11 * m33 - m13 * m31;
    v5 = m12 * m33 - m13 * m32;
    float d02 = +(v5 * m01 - v4 * m02 + v3 * m03) * invDet;
    float d12 = -(v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    float d22 = +(v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    float d32 = -(v3 * m00 - v1 * m01 + v0 * m02) * invDet;
    v0 = m21 * m10 - m20 * m11;
    v1 = m22 * m10 - m20 * m12;
    v2 = m23 * m10 - m20 * m13;
    v3 = m22 * m11 - m21 * m12;
    v4 = m23 * m11 - m21 * m13;
    v5 = m23 * m12 - m22 * m13;
    float d03 = -(v5 * m01 - v4 * m02 + v3 * m03) * invDet;
    float d13 = +(v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    float d23 = -(v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    float d33 = +(v3 * m00 - v1 * m01 + v0 * m02) * invDet;
    M44 r;
    r.setRow(0, V4{d00, d01, d02, d03});
    r.setRow(1, V4{d10, d11, d12, d13});
    r.setRow(2, V4{d20, d21, d22, d23});
    r.setRow(3, V4{d30, d31, d32, d33});
    return r;
}

// --- Frame (Frame.h) -------------------------------------------------------
struct Frame { V3 s, t, n; };
static inline void coordinateSystem(V3 a, V3& s, V3& t) {                  // Frame.h:9-22
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        t = v3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        t = v3(0.0f, a.z * invLen, -a.y * invLen);
    }
    s = normalize(cross(t, a));
}
static inline V3 toLocal(const Frame& f, V3 v) { return v3(dot(v, f.s), dot(v, f.t), dot(v, f.n)); }
static inline V3 toWorld(const Frame& f, V3 v) { return f.s * v.x + f.t * v.y + f.n * v.z; }

// --- half (half.h) ---------------------------------------------------------
// HOST decode quirk (half.h:72-84): ((h&0x7fff)<<13) + 0x38000000 — wrong for
// zero/denormal/inf; the CUDA path (__half2float) is IEEE.
static inline float half_to_float_host(uint16_t val) {
    int32_t fltInt32 = ((val & 0x8000) << 16);
    fltInt32 |= ((val & 0x7fff) << 13) + 0x38000000;
    return as_float(fltInt32);
}
static inline float half_to_float_ieee(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000) << 16;
    uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) bits = sign;
        else {  // denormal: value = man * 2^-24
            float f = (float)man * 5.9604644775390625e-08f;
            bits = as_uint(f) | sign;
        }
    } else if (exp == 31) bits = sign | 0x7f800000u | (man << 13);
    else bits = sign | ((exp + 112) << 23) | (man << 13);
    float r; std::memcpy(&r, &bits, 4); return r;
}
static inline uint16_t float_to_half(float f) {                            // half.h:21-60 (host branch)
    uint32_t ia; std::memcpy(&ia, &f, 4);
    uint16_t ir = (ia >> 16) & 0x8000;
    if ((ia & 0x7f800000) == 0x7f800000) {
        if ((ia & 0x7fffffff) == 0x7f800000) ir |= 0x7c00;
        else ir = 0x7fff;
    } else if ((ia & 0x7f800000) >= 0x33000000) {
        int shift = (int)((ia >> 23) & 0xff) - 127;
        if (shift > 15) ir |= 0x7c00;
        else {
            ia = (ia & 0x007fffff) | 0x00800000;
            if (shift < -14) {
                ir |= ia >> (-1 - shift);
                ia = ia << (32 - (-1 - shift));
            } else {
                ir |= ia >> (24 - 11);
                ia = ia << (32 - (24 - 11));
                ir = ir + ((14 + shift) << 10);
            }
            if ((ia > 0x80000000u) || ((ia == 0x80000000u) && (ir & 1))) ir++;
        }
    }
    return ir;
}

// --- spherical 16-bit normal codec (Compression.h:12-31) -------------------
static inline uint16_t normal_encode(V3 v) {
    float theta = (cr_acos(v.z) * (255.0f / O_PI));
    float phi = (cr_atan2(v.y, v.x) * (255.0f / (2.0f * O_PI)));
    phi = phi < 0 ? (phi + 255) : phi;
    auto u16 = [](float f) { return (f != f) ? (uint16_t)0 : (uint16_t)(int32_t)f; };   // NaN -> 0
    return (uint16_t)(((uint32_t)u16(theta) << 8) | (uint32_t)u16(phi));
}
static inline V3 normal_decode(uint16_t v) {
    const float PI_4 = O_PI / 4.0f, PI_2 = O_PI / 2.0f;
    unsigned char x = v >> 8, y = v & 0xff;
    float theta = x == 63 ? PI_4 : (x == 127 ? PI_2 : (x == 191 ? 3 * PI_4 : float(x) * (1.0f / 255.0f) * O_PI));
    float phi = y == 63 ? PI_2 : (y == 127 ? O_PI : (y == 191 ? 3 * PI_2 : float(y) * (1.0f / 255.0f) * O_PI * 2.0f));
    float sinphi = cr_sin(phi), cosphi = cr_cos(phi), sintheta = cr_sin(theta), costheta = cr_cos(theta);
    return v3(sintheta * cosphi, sintheta * sinphi, costheta);
}

}  // namespace oracle

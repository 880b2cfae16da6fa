// ctl_math.h — fp32 scalar/vector/matrix arithmetic shared by the host scene
// compiler and the gfx950 kernels of libctl_trace.so.
//
// Every function keeps the operation order of the reference
// (Ilinite/CudaTracerLib Math/Vector.h, MathFunc.h, float4x4.h, Frame.h) and
// the library is compiled with -ffp-contract=off, so the GPU results are bit
// identical to the CPU oracle's.  Transcendentals are evaluated as
// correctly-rounded fp32 through fp64: the
// reference itself uses host libm on its CPU path and __sinf-class
// intrinsics on its CUDA path (MathFunc.h:222-288), which disagree.
#pragma once
#include <stdint.h>
#include <math.h>
#include <float.h>
#include <string.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define CTL_HD __host__ __device__ __forceinline__
#else
#define CTL_HD static inline
#endif

namespace ctl {

#define CTL_PI 3.14159265358979f          // MathFunc.h:12
#define CTL_INV_PI (1.0f / CTL_PI)        // MathFunc.h:13

template <class T> CTL_HD T tmin(T a, T b) { return (a < b) ? a : b; }   // MathFunc.h:83-90
template <class T> CTL_HD T tmax(T a, T b) { return (a > b) ? a : b; }

CTL_HD float bits_f(int32_t i) { float f; memcpy(&f, &i, 4); return f; }
CTL_HD int32_t f_bits(float f) { int32_t i; memcpy(&i, &f, 4); return i; }
CTL_HD float copysign_ref(float a, float b) {                            // MathFunc.h:66-69
    return bits_f((f_bits(b) & (int32_t)0x80000000) | (f_bits(a) & ~(int32_t)0x80000000));
}
CTL_HD float fracf_ref(float f) { return f - floorf(f); }                 // MathFunc.h:138-141

// On the device the fp64 library bodies are large (range reduction, ~30-60
// fp64 ops and their register pairs); each one stays out of line so a caller's
// register peak does not include them (rough_sample: 148 -> 69 VGPRs, which is
// what lets the C5 path kernel run at 4 waves/SIMD).
#if defined(__HIP__)
#define CTL_CR static __host__ __device__ __noinline__
#else
#define CTL_CR CTL_HD
#endif
CTL_CR float cr_sin(float x) { return (float)sin((double)x); }
CTL_CR float cr_cos(float x) { return (float)cos((double)x); }
CTL_CR float cr_tan(float x) { return (float)tan((double)x); }
CTL_CR float cr_acos(float x) { return (float)acos((double)x); }
CTL_CR float cr_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
CTL_CR float cr_atan(float x) { return (float)atan((double)x); }
CTL_CR float cr_exp(float x) { return (float)exp((double)x); }
CTL_CR float cr_log(float x) { return (float)log((double)x); }
CTL_CR float cr_log2(float x) { return (float)log2((double)x); }
CTL_CR float cr_pow(float a, float b) { return (float)pow((double)a, (double)b); }

struct f2 { float x, y; };
struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };

CTL_HD f2 mk2(float x, float y) { f2 r; r.x = x; r.y = y; return r; }
CTL_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
CTL_HD f3 mk3s(float s) { return mk3(s, s, s); }
CTL_HD f4 mk4(float x, float y, float z, float w) { f4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
CTL_HD f4 mk4(f3 a, float w) { return mk4(a.x, a.y, a.z, w); }
CTL_HD f3 xyz(f4 a) { return mk3(a.x, a.y, a.z); }

CTL_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
CTL_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
CTL_HD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
CTL_HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
CTL_HD f3 operator*(float s, f3 a) { return a * s; }                     // Vector.h:384
CTL_HD f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
CTL_HD f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
CTL_HD f2 operator+(f2 a, f2 b) { return mk2(a.x + b.x, a.y + b.y); }
CTL_HD f2 operator-(f2 a, f2 b) { return mk2(a.x - b.x, a.y - b.y); }
CTL_HD f2 operator*(f2 a, float s) { return mk2(a.x * s, a.y * s); }
CTL_HD f2 operator*(float s, f2 a) { return a * s; }

// VectorBase::dot / lenSqr accumulate from (T)0 (Vector.h:46,97)
CTL_HD float dot(f3 a, f3 b) { float r = 0.0f; r += a.x * b.x; r += a.y * b.y; r += a.z * b.z; return r; }
CTL_HD float dot(f4 a, f4 b) {
    float r = 0.0f; r += a.x * b.x; r += a.y * b.y; r += a.z * b.z; r += a.w * b.w; return r;
}
CTL_HD float lenSqr(f3 a) { float r = 0.0f; r += a.x * a.x; r += a.y * a.y; r += a.z * a.z; return r; }
CTL_HD float length(f3 a) { return sqrtf(lenSqr(a)); }
CTL_HD float rcp_ref(float a) { return a ? 1.0f / a : 0.0f; }           // MathFunc.h:399
CTL_HD f3 normalize(f3 a) { return a * rcp_ref(length(a)); }             // Vector.h:369-372
CTL_HD f3 cross(f3 a, f3 b) {                                            // Vector.h:329
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
CTL_HD float absdot(f3 a, f3 b) { return fabsf(dot(a, b)); }
CTL_HD f3 vmin(f3 a, f3 b) { return mk3(tmin(a.x, b.x), tmin(a.y, b.y), tmin(a.z, b.z)); }
CTL_HD f3 vmax(f3 a, f3 b) { return mk3(tmax(a.x, b.x), tmax(a.y, b.y), tmax(a.z, b.z)); }
CTL_HD float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// float4x4, row-major (float4x4.h:12-17)
struct m44 {
    float d[16];
    CTL_HD float at(int i, int j) const { return d[i * 4 + j]; }
    CTL_HD float& at(int i, int j) { return d[i * 4 + j]; }
    CTL_HD f4 row(int i) const { return mk4(d[i * 4 + 0], d[i * 4 + 1], d[i * 4 + 2], d[i * 4 + 3]); }
    CTL_HD f4 col(int j) const { return mk4(d[j], d[4 + j], d[8 + j], d[12 + j]); }
    CTL_HD void set_row(int i, f4 r) { d[i * 4 + 0] = r.x; d[i * 4 + 1] = r.y; d[i * 4 + 2] = r.z; d[i * 4 + 3] = r.w; }
    CTL_HD void set_col(int j, f4 c) { d[j] = c.x; d[4 + j] = c.y; d[8 + j] = c.z; d[12 + j] = c.w; }
};
CTL_HD m44 m44_zero() { m44 m; for (int i = 0; i < 16; i++) m.d[i] = 0.0f; return m; }
CTL_HD m44 m44_identity() { m44 m = m44_zero(); m.d[0] = m.d[5] = m.d[10] = m.d[15] = 1.0f; return m; }
CTL_HD f4 mul(const m44& m, f4 v) { return mk4(dot(m.row(0), v), dot(m.row(1), v), dot(m.row(2), v), dot(m.row(3), v)); }
CTL_HD m44 matmul(const m44& a, const m44& b) {                          // operator% (float4x4.h:368-375)
    m44 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.at(i, j) = dot(a.row(i), b.col(j));
    return r;
}
CTL_HD f3 xform_point(const m44& m, f3 p) { f4 f = mul(m, mk4(p, 1.0f)); return xyz(f) / f.w; }   // :398-402
CTL_HD f3 xform_dir(const m44& m, f3 d) { return xyz(mul(m, mk4(d, 0.0f))); }                      // :404-408

// float4x4::inverse (float4x4.h:132-190), same expression trees.
CTL_HD m44 inverse(const m44& Q) {
    float m00 = Q.at(0, 0), m01 = Q.at(0, 1), m02 = Q.at(0, 2), m03 = Q.at(0, 3);
    float m10 = Q.at(1, 0), m11 = Q.at(1, 1), m12 = Q.at(1, 2), m13 = Q.at(1, 3);
    float m20 = Q.at(2, 0), m21 = Q.at(2, 1), m22 = Q.at(2, 2), m23 = Q.at(2, 3);
    float m30 = Q.at(3, 0), m31 = Q.at(3, 1), m32 = Q.at(3, 2), m33 = Q.at(3, 3);
    float a0 = m20 * m31 - m21 * m30, a1 = m20 * m32 - m22 * m30, a2 = m20 * m33 - m23 * m30;
    float a3 = m21 * m32 - m22 * m31, a4 = m21 * m33 - m23 * m31, a5 = m22 * m33 - m23 * m32;
    float t00 = +(a5 * m11 - a4 * m12 + a3 * m13);
    float t10 = -(a5 * m10 - a2 * m12 + a1 * m13);
    float t20 = +(a4 * m10 - a2 * m11 + a0 * m13);
    float t30 = -(a3 * m10 - a1 * m11 + a0 * m12);
    float invDet = 1 / (t00 * m00 + t10 * m01 + t20 * m02 + t30 * m03);
    m44 r;
    r.at(0, 0) = t00 * invDet; r.at(1, 0) = t10 * invDet; r.at(2, 0) = t20 * invDet; r.at(3, 0) = t30 * invDet;
    r.at(0, 1) = -(a5 * m01 - a4 * m02 + a3 * m03) * invDet;
    r.at(1, 1) = +(a5 * m00 - a2 * m02 + a1 * m03) * invDet;
    r.at(2, 1) = -(a4 * m00 - a2 * m01 + a0 * m03) * invDet;
    r.at(3, 1) = +(a3 * m00 - a1 * m01 + a0 * m02) * invDet;
    a0 = m10 * m31 - m11 * m30; a1 = m10 * m32 - m12 * m30; a2 = m10 * m33 - m13 * m30;
    a3 = m11 * m32 - m12 * m31; a4 = m11 * m33 - m13 * m31; a5 = m12 * m33 - m13 * m32;
    r.at(0, 2) = +(a5 * m01 - a4 * m02 + a3 * m03) * invDet;
    r.at(1, 2) = -(a5 * m00 - a2 * m02 + a1 * m03) * invDet;
    r.at(2, 2) = +(a4 * m00 - a2 * m01 + a0 * m03) * invDet;
    r.at(3, 2) = -(a3 * m00 - a1 * m01 + a0 * m02) * invDet;
    a0 = m21 * m10 - m20 * m11; a1 = m22 * m10 - m20 * m12; a2 = m23 * m10 - m20 * m13;
    a3 = m22 * m11 - m21 * m12; a4 = m23 * m11 - m21 * m13; a5 = m23 * m12 - m22 * m13;
    r.at(0, 3) = -(a5 * m01 - a4 * m02 + a3 * m03) * invDet;
    r.at(1, 3) = +(a5 * m00 - a2 * m02 + a1 * m03) * invDet;
    r.at(2, 3) = -(a4 * m00 - a2 * m01 + a0 * m03) * invDet;
    r.at(3, 3) = +(a3 * m00 - a1 * m01 + a0 * m02) * invDet;
    return r;
}

// Frame (Frame.h:9-45)
struct frame { f3 s, t, n; };
CTL_HD void coordinate_system(f3 a, f3& s, f3& t) {
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        t = mk3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        t = mk3(0.0f, a.z * invLen, -a.y * invLen);
    }
    s = normalize(cross(t, a));
}
CTL_HD f3 to_local(const frame& f, f3 v) { return mk3(dot(v, f.s), dot(v, f.t), dot(v, f.n)); }
CTL_HD f3 to_world(const frame& f, f3 v) { return f.s * v.x + f.t * v.y + f.n * v.z; }

// half -> float.  host_quirk reproduces Math/half.h:72-84 (reference CPU path);
// otherwise IEEE binary16 (the reference CUDA path, __half2float).
CTL_HD float half_to_float(uint32_t h16, bool host_quirk) {
    uint32_t val = h16 & 0xffffu;
    if (host_quirk) {
        int32_t b = (int32_t)((val & 0x8000u) << 16);
        b |= (int32_t)(((val & 0x7fffu) << 13) + 0x38000000u);
        return bits_f(b);
    }
    uint32_t sign = (val & 0x8000u) << 16, ex = (val >> 10) & 0x1fu, man = val & 0x3ffu;
    uint32_t b;
    if (ex == 0) {
        if (man == 0) b = sign;
        else { float f = (float)man * 5.9604644775390625e-08f; b = (uint32_t)f_bits(f) | sign; }
    } else if (ex == 31) b = sign | 0x7f800000u | (man << 13);
    else b = sign | ((ex + 112u) << 23) | (man << 13);
    return bits_f((int32_t)b);
}

// float -> unsigned short of a value in [0, 65536); NaN -> 0 (the conversion
// both targets' cvt instructions give, made explicit).
CTL_HD uint16_t u16_trunc(float f) { return (f != f) ? (uint16_t)0 : (uint16_t)(int32_t)f; }

// NormalizedFloat3ToUchar2_Spherical (Compression.h:12-18)
CTL_HD uint16_t normal_encode16(f3 v) {
    float theta = (cr_acos(v.z) * (255.0f / CTL_PI));
    float phi = (cr_atan2(v.y, v.x) * (255.0f / (2.0f * CTL_PI)));
    phi = phi < 0 ? (phi + 255) : phi;
    return (uint16_t)(((uint32_t)u16_trunc(theta) << 8) | (uint32_t)u16_trunc(phi));
}

// half((float)x).ToFloat() for a pixel coordinate x <= 65504: __float2half_rn
// (Math/half.h:21-24, device branch) keeps 11 significant bits, ties to even.
CTL_HD float half_round_int(uint32_t x) {
    if (x < 2048u) return (float)x;
    uint32_t sh = 0;
    while ((x >> sh) >= 2048u) sh++;
    uint32_t q = x >> sh, r = x & ((1u << sh) - 1u), h = 1u << (sh - 1u);
    if (r > h || (r == h && (q & 1u))) q++;
    return (float)(q << sh);
}

// Uchar2ToNormalizedFloat3_Spherical (Compression.h:20-31)
CTL_HD f3 normal_decode16(uint32_t v16) {
    const float PI_4 = CTL_PI / 4.0f, PI_2 = CTL_PI / 2.0f;
    unsigned char x = (unsigned char)((v16 >> 8) & 0xff), y = (unsigned char)(v16 & 0xff);
    float theta = x == 63 ? PI_4 : (x == 127 ? PI_2 : (x == 191 ? 3 * PI_4 : float(x) * (1.0f / 255.0f) * CTL_PI));
    float phi = y == 63 ? PI_2 : (y == 127 ? CTL_PI : (y == 191 ? 3 * PI_2 : float(y) * (1.0f / 255.0f) * CTL_PI * 2.0f));
    float sinphi = cr_sin(phi), cosphi = cr_cos(phi), sintheta = cr_sin(theta), costheta = cr_cos(theta);
    return mk3(sintheta * cosphi, sintheta * sinphi, costheta);
}

}  // namespace ctl

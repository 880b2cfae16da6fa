// ctl_bsdf.h — the C5 shading pieces of the PathTracer path (row a12 of
// SURVEY.md §8): image textures with MIP-map filtering, the microfacet
// distribution and the roughdielectric BSDF, plus the BSDF dispatch.  fp32 in
// the reference's operation order (no contraction; transcendentals through
// fp64, see ctl_math.h).
//
//   tex_*              KernelMIPMap::Texel/triangle/eval/evalEWA   Engine/MIPMap.cu:15-233
//                      WrapCoordinates                             Engine/MIPMap_device.h:34-57
//                      ImageTexture::Evaluate                      SceneTypes/Texture.cu:7-33
//   mf_*               MicrofacetDistribution                      Engine/MicrofacetDistribution.{h,cu}
//   fresnel_*, reflect, refract                                    Math/FresnelHelper.h:27-160
//   rough_*            roughdielectric::sample/f/pdf               SceneTypes/BSDF_Simple.cu:373-615
//   bsdf_*             BSDFALL two-sided wrapper + dispatch        SceneTypes/BSDF.h:140-208
#pragma once
#include "ctl_shade.h"

namespace ctl {

// ---------------------------------------------------------------------------
// scalar helpers (Math/MathFunc.h)
CTL_HD float signum_ref(float v) { return copysign_ref(1.0f, v); }                  // :116-119
CTL_HD float safe_sqrt_ref(float v) { return sqrtf(tmax(0.0f, v)); }                // :112-114
CTL_HD float clampf_ref(float v, float lo, float hi) { return tmin(tmax(v, lo), hi); }   // :169-170
CTL_HD int clampi_ref(int v, int lo, int hi) { return tmin(tmax(v, lo), hi); }
CTL_HD uint32_t clampu_ref(uint32_t v, uint32_t lo, uint32_t hi) { return tmin(tmax(v, lo), hi); }
CTL_HD float hypot2_ref(float a, float b) {                                           // :326-340
    float r;
    if (fabsf(a) > fabsf(b)) {
        r = b / a;
        r = fabsf(a) * sqrtf(1.0f + r * r);
    } else if (b != 0.0f) {
        r = a / b;
        r = fabsf(b) * sqrtf(1.0f + r * r);
    } else {
        r = 0.0f;
    }
    return r;
}
CTL_HD float erfinv_ref(float x) {                                                    // :343-372 (Giles)
    float w = -cr_log((1.0f - x) * (1.0f + x));
    float p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = sqrtf(w) - 3;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
CTL_HD float erf_ref(float x) {                                                       // :374-392 (A&S 7.1.26)
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f, a5 = 1.061405429f;
    const float p = 0.3275911f;
    float sign = signum_ref(x);
    x = fabsf(x);
    float t = 1.0f / (1.0f + p * x);
    float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * cr_exp(-x * x);
    return sign * y;
}

// ---------------------------------------------------------------------------
// Image textures (KernelMIPMap, RGBCOL texels).  The bilinear, EWA and
// texture entry points are out of line on the device: the MIP/EWA filter is
// large and would otherwise be inlined at every call site (instruction-cache
// footprint of the path kernel).
#if defined(__HIP__)
#define CTL_TEX_FN static __host__ __device__ __noinline__
#else
#define CTL_TEX_FN static inline
#endif
struct TexView {
    const ctl_texture* tex;
    const uint32_t* data;
};

CTL_HD bool tex_wrap(f2 uv, f2 dim, uint32_t wrap, f2& loc) {                         // WrapCoordinates
    switch (wrap) {
        case CTL_WRAP_REPEAT:
            loc = mk2(fracf_ref(uv.x) * dim.x, fracf_ref(1.0f - uv.y) * dim.y);
            return true;
        case CTL_WRAP_CLAMP:
            loc = mk2(clampf_ref(uv.x, 0.0f, 1.0f) * dim.x, clampf_ref(1.0f - uv.y, 0.0f, 1.0f) * dim.y);
            return true;
        case CTL_WRAP_MIRROR: {
            const bool even = (int)uv.x % 2 == 0;
            float lx = even ? fracf_ref(uv.x) : 1.0f - fracf_ref(uv.x);
            float ly = even ? fracf_ref(uv.y) : 1.0f - fracf_ref(uv.y);
            loc = mk2(lx * dim.x, ly * dim.y);
            return true;
        }
        case CTL_WRAP_BLACK:
            if (uv.x < 0 || uv.x >= 1 || uv.y < 0 || uv.y >= 1) return false;
            loc = mk2(uv.x * dim.x, uv.y * dim.y);
            return true;
    }
    return false;
}

// float(b) / 255.0f for a byte b, bit for bit: one product and one FMA correction step give the
// correctly rounded quotient for every b in 0..255 (checked exhaustively by tests/test_unorm8.py),
// instead of a full division per colour channel of every texel.
CTL_HD float unorm8(uint32_t b) {
    const float x = (float)b, c = 1.0f / 255.0f;
    const float q0 = x * c;
    return fmaf(fmaf(-q0, 255.0f, x), c, q0);
}

CTL_HD spec tex_texel(TexView T, uint32_t level, f2 uv) {                     // MIPMap.cu:15-35
    const ctl_texture& t = *T.tex;
    f2 l;
    if (!tex_wrap(uv, mk2((float)(t.width >> level), (float)(t.height >> level)), t.wrap, l)) return mk3s(0.0f);
    const int wl = (int)(t.width >> level), hl = (int)(t.height >> level);
    const int x = clampi_ref((int)l.x, 0, wl - 1), y = clampi_ref((int)l.y, 0, hl - 1);
    const uint32_t c = T.data[t.offsets[level] + (uint32_t)y * (uint32_t)wl + (uint32_t)x];
    // Spectrum::fromRGBCOL -> SpectrumConverter::COLORREFToFloat3 (Spectrum.h:528-532)
    return mk3(unorm8(c & 0xffu), unorm8((c >> 8) & 0xffu), unorm8((c >> 16) & 0xffu));
}

// One MIP level's fields, read once per EWA lookup (tex_texel reads them per texel).
struct TexLevel {
    const uint32_t* data;
    uint32_t base, wl, hl;   // offsets[level], level size
    f2 dim;                  // level size as floats
};

// tex_texel for a fixed wrap mode (WRAP outside 0..3: no texel, as tex_wrap).
template <uint32_t WRAP>
CTL_HD spec level_texel(const TexLevel& L, f2 uv) {
    f2 l;
    if (!tex_wrap(uv, L.dim, WRAP, l)) return mk3s(0.0f);
    const int x = clampi_ref((int)l.x, 0, (int)L.wl - 1), y = clampi_ref((int)l.y, 0, (int)L.hl - 1);
    const uint32_t c = L.data[L.base + (uint32_t)y * L.wl + (uint32_t)x];
    return mk3(unorm8(c & 0xffu), unorm8((c >> 8) & 0xffu), unorm8((c >> 16) & 0xffu));
}

// tex_triangle with the texture's fields read per texel: fewer live registers
// (up to v31) than tex_triangle's per-wrap-mode form, for the alpha test's
// call inside the traversal loop, where a callee using v32..v39 costs the
// caller spills.  Same arithmetic.
CTL_TEX_FN spec tex_triangle_compact(TexView T, uint32_t level, f2 uv) {                  // MIPMap.cu:37-48
    const ctl_texture& t = *T.tex;
    level = clampu_ref(level, 0u, t.levels - 1);
    const f2 s = mk2((float)(t.width >> level), (float)(t.height >> level));
    const f2 is = mk2(1.0f / s.x, 1.0f / s.y);
    const f2 l = mk2(uv.x * s.x, uv.y * s.y);
    const float ds = fracf_ref(l.x), dt = fracf_ref(l.y);
    return (1.f - ds) * (1.f - dt) * tex_texel(T, level, uv) + (1.f - ds) * dt * tex_texel(T, level, uv + mk2(0, is.y)) +
           ds * (1.f - dt) * tex_texel(T, level, uv + mk2(is.x, 0)) + ds * dt * tex_texel(T, level, uv + mk2(is.x, is.y));
}

template <uint32_t WRAP>
CTL_HD spec level_bilerp(const TexLevel& L, f2 uv, f2 is, float ds, float dt) {
    return (1.f - ds) * (1.f - dt) * level_texel<WRAP>(L, uv) + (1.f - ds) * dt * level_texel<WRAP>(L, uv + mk2(0, is.y)) +
           ds * (1.f - dt) * level_texel<WRAP>(L, uv + mk2(is.x, 0)) + ds * dt * level_texel<WRAP>(L, uv + mk2(is.x, is.y));
}

CTL_TEX_FN spec tex_triangle(TexView T, uint32_t level, f2 uv) {                  // MIPMap.cu:37-48
    const ctl_texture& t = *T.tex;
    level = clampu_ref(level, 0u, t.levels - 1);
    const uint32_t wl = t.width >> level, hl = t.height >> level;
    const f2 s = mk2((float)wl, (float)hl);
    const f2 is = mk2(1.0f / s.x, 1.0f / s.y);
    const f2 l = mk2(uv.x * s.x, uv.y * s.y);
    const float ds = fracf_ref(l.x), dt = fracf_ref(l.y);
    const TexLevel L{T.data, t.offsets[level], wl, hl, s};
    switch (t.wrap) {   // the level's fields and the wrap mode resolved once for the four texels
        case CTL_WRAP_REPEAT: return level_bilerp<CTL_WRAP_REPEAT>(L, uv, is, ds, dt);
        case CTL_WRAP_CLAMP: return level_bilerp<CTL_WRAP_CLAMP>(L, uv, is, ds, dt);
        case CTL_WRAP_MIRROR: return level_bilerp<CTL_WRAP_MIRROR>(L, uv, is, ds, dt);
        case CTL_WRAP_BLACK: return level_bilerp<CTL_WRAP_BLACK>(L, uv, is, ds, dt);
        default: return level_bilerp<0xffffffffu>(L, uv, is, ds, dt);
    }
}

// The EWA footprint loop of tex_ewa.  P2: both level sizes are powers of two,
// so (float)ut / size.x is the exact product with the exact reciprocal (the
// quotient's value, without a division per texel).
template <uint32_t WRAP, bool P2>
CTL_HD void ewa_footprint(const TexLevel& L, const float* lut, int u0, int u1, int v0, int v1, float u, float v,
                          float As, float Bs, float Cs, spec& result, float& denominator) {
    const f2 size = L.dim, inv = mk2(1.0f / size.x, 1.0f / size.y);
    const float ddq = 2 * As, uu0 = u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = vt - v;
        const float tv = P2 ? (float)vt * inv.y : (float)vt / size.y;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < 64) {
                const uint32_t qi = (uint32_t)q;
                if (qi < 64) {
                    const float weight = lut[(int)q];
                    const float tu = P2 ? (float)ut * inv.x : (float)ut / size.x;
                    result = result + level_texel<WRAP>(L, mk2(tu, tv)) * weight;
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
}

CTL_TEX_FN spec tex_ewa(TexView T, uint32_t level, f2 uv, float A, float B, float C) {   // MIPMap.cu:50-111
    const ctl_texture& t = *T.tex;
    if (level >= t.levels) return tex_texel(T, t.levels - 1, mk2(0.0f, 0.0f));
    const uint32_t wl = t.width >> level, hl = t.height >> level;
    const f2 size = mk2((float)wl, (float)hl);
    const float u = uv.x * size.x - 0.5f;
    const float v = uv.y * size.y - 0.5f;
    // KernelMIPMap::m_fDim = (width - 1, height - 1) (MIPMap.cpp:108)
    const f2 ratio = mk2(size.x / ((float)t.width - 1), size.y / ((float)t.height - 1));
    A /= ratio.x * ratio.x;
    B /= ratio.x * ratio.y;
    C /= ratio.y * ratio.y;
    const float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * sqrtf(C * invDet),
                deltaV = 2.0f * sqrtf(A * invDet);
    const int u0 = (int)ceilf(u - deltaU), u1 = (int)floorf(u + deltaU);
    const int v0 = (int)ceilf(v - deltaV), v1 = (int)floorf(v + deltaV);
    const float As = A * 64, Bs = B * 64, Cs = C * 64;
    spec result = mk3s(0.0f);
    float denominator = 0.0f;
    const TexLevel L{T.data, t.offsets[level], wl, hl, size};
    const float* lut = t.weight_lut;
    const bool p2 = (wl & (wl - 1)) == 0 && (hl & (hl - 1)) == 0;
#define CTL_EWA(W)                                                                                     \
    (p2 ? ewa_footprint<W, true>(L, lut, u0, u1, v0, v1, u, v, As, Bs, Cs, result, denominator)        \
        : ewa_footprint<W, false>(L, lut, u0, u1, v0, v1, u, v, As, Bs, Cs, result, denominator))
    switch (t.wrap) {
        case CTL_WRAP_REPEAT: CTL_EWA(CTL_WRAP_REPEAT); break;
        case CTL_WRAP_CLAMP: CTL_EWA(CTL_WRAP_CLAMP); break;
        case CTL_WRAP_MIRROR: CTL_EWA(CTL_WRAP_MIRROR); break;
        case CTL_WRAP_BLACK: CTL_EWA(CTL_WRAP_BLACK); break;
        default: CTL_EWA(0xffffffffu); break;   // no texel, the weights still count
    }
#undef CTL_EWA
    if (denominator == 0) return tex_triangle(T, level, uv);
    return spec_div(result, denominator);
}

// KernelMIPMap::eval (MIPMap.cu:160-233): point / bilinear / trilinear / EWA
CTL_HD spec tex_eval(TexView T, f2 uv, f2 d0, f2 d1) {
    const ctl_texture& t = *T.tex;
    const float dimx = (float)t.width - 1, dimy = (float)t.height - 1;   // m_fDim (MIPMap.cpp:108)
    const float du0 = d0.x * dimx, dv0 = d0.y * dimy, du1 = d1.x * dimx, dv1 = d1.y * dimy, du = (du0 + du1) / 2.0f,
                dv = (dv0 + dv1) / 2.0f;
    if (t.filter == CTL_TEX_POINT) return tex_texel(T, 0, uv);
    if (t.filter == CTL_TEX_BILINEAR) return tex_triangle(T, 0, uv);
    if (t.filter == CTL_TEX_TRILINEAR) {
        const float levela = cr_log2(dimx / fabsf(du)), levelb = cr_log2(dimy / fabsf(dv)),
                    level = t.levels - clampf_ref((levela + levelb) / 2.0f, 1.0f, (float)t.levels);
        const int iLevel = (int)floorf(level), iLevel2 = clampi_ref(iLevel + 1, 0, (int)t.levels - 1);
        const float p = level - iLevel;
        const spec texelA = tex_triangle(T, (uint32_t)iLevel, uv), texelB = tex_triangle(T, (uint32_t)iLevel2, uv);
        return p * texelA + (1 - p) * texelB;
    }
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1,
          F = A * C - B * B * 0.25f;
    // MIPMap.cu's file-local hypot2 (sqrt(a*a + b*b)), not math::hypot2
    float root = sqrtf((A - C) * (A - C) + B * B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root),
          majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        const float level = cr_log2(tmax(majorRadius, 1e-4f));
        const int ilevel = (int)floorf(level);
        if (ilevel < 0) return tex_triangle(T, 0, uv);
        const float a = level - ilevel;
        return tex_triangle(T, (uint32_t)ilevel, uv) * (1.0f - a) + tex_triangle(T, (uint32_t)ilevel + 1, uv) * a;
    }
    const float m_maxAnisotropy = 16;
    if (minorRadius * m_maxAnisotropy < majorRadius) {
        minorRadius = majorRadius / m_maxAnisotropy;
        const float theta = 0.5f * cr_atan(B / (A - C));
        const float sinTheta = cr_sin(theta), cosTheta = cr_cos(theta);
        const float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                    cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    const float scale = 1.0f / F;
    A *= scale; B *= scale; C *= scale;
    const float level = tmax(0.0f, cr_log2(minorRadius));
    const int ilevel = (int)level;
    const float a = level - ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return tex_triangle(T, (uint32_t)ilevel, uv);
    return tex_ewa(T, (uint32_t)ilevel, uv, A, B, C) * (1.0f - a) + tex_ewa(T, (uint32_t)ilevel + 1, uv, A, B, C) * a;
}

// ImageTexture::Evaluate(const DifferentialGeometry&) (Texture.cu:16-31).
// Out of line on the device: the MIP/EWA filter is large and would otherwise
// be inlined at every BSDF call site (instruction-cache footprint).
// The differential geometry's uv and partials come by value (an argument
// passed by reference to an out-of-line call lives in scratch for the call).
CTL_TEX_FN spec image_texture_eval(TexView T, f2 duv, float dudx, float dudy, float dvdx, float dvdy,
                                   bool has_partials) {
    const ctl_texture& t = *T.tex;
    spec r;
    if (has_partials) {
        const f2 uv = mk2(t.m11 * duv.x + t.m12 * duv.y, t.m21 * duv.x + t.m22 * duv.y) + mk2(t.m13, t.m23);
        const float dsdx = t.m11 * dudx + t.m12 * dvdx, dsdy = t.m11 * dudy + t.m12 * dvdy;
        const float dtdx = t.m21 * dudx + t.m22 * dvdx, dtdy = t.m21 * dudy + t.m22 * dvdy;
        r = tex_eval(T, uv, mk2(dsdx, dtdx), mk2(dsdy, dtdy));
    } else {   // Evaluate(uv) -> Sample(uv)
        const f2 uv = mk2(t.m11 * duv.x + t.m12 * duv.y, t.m21 * duv.x + t.m22 * duv.y) + mk2(t.m13, t.m23);
        r = t.filter == CTL_TEX_POINT ? tex_texel(T, 0, uv) : tex_triangle(T, 0, uv);
    }
    return r * mk3(t.scale[0], t.scale[1], t.scale[2]);
}

// KernelMIPMap::SampleAlpha (MIPMap.cu:123-139): level-0 texel alpha, no
// filtering.  The reference indexes without clamping; the index is clamped
// here (it can only differ where the reference would read out of bounds).
CTL_HD float tex_sample_alpha(TexView T, f2 uv) {
    const ctl_texture& t = *T.tex;
    f2 l;
    if (!tex_wrap(uv, mk2((float)t.width, (float)t.height), t.wrap, l)) return 0.0f;
    const uint32_t x = tmin((uint32_t)l.x, t.width - 1), y = tmin((uint32_t)l.y, t.height - 1);
    const uint32_t c = T.data[t.offsets[0] + y * t.width + x];
    return unorm8(c >> 24);
}

CTL_HD f2 tex_map(const ctl_texture& t, f2 uv) {   // TextureMapping2D::TransformPoint
    return mk2(t.m11 * uv.x + t.m12 * uv.y, t.m21 * uv.x + t.m22 * uv.y) + mk2(t.m13, t.m23);
}

// Material::AlphaTest (Engine/Material.cu:160-189) for image / constant
// textures (sample_fast, :140-158), states without the Color compare.
CTL_HD bool material_alpha_test(const ctl_material& m, TexView tex, f2 uv) {
    if (!m.alpha_state) return true;
    const bool reflImg = m.texture != 0xffffffffu;
    const bool alphaImg = m.alpha_texture != 0xffffffffu;
    if ((m.alpha_state == 2 && alphaImg) || (m.alpha_state == 6 && reflImg)) {
        const ctl_texture& t = tex.tex[m.alpha_state == 2 ? m.alpha_texture : m.texture];
        const TexView T{&t, tex.data};
        return tex_sample_alpha(T, tex_map(t, uv)) >= m.alpha_threshold;
    }
    spec val;
    const uint32_t src = (m.alpha_state & 4) ? m.texture : m.alpha_texture;
    if (src != 0xffffffffu) {   // ImageTexture::Evaluate(uv) -> Sample
        const ctl_texture& t = tex.tex[src];
        const TexView T{&t, tex.data};
        const f2 u2 = tex_map(t, uv);
        val = (t.filter == CTL_TEX_POINT ? tex_texel(T, 0, u2) : tex_triangle_compact(T, 0, u2)) *
              mk3(t.scale[0], t.scale[1], t.scale[2]);
    } else {                    // ConstantTexture (the diffuse reflectance)
        val = refl(m);
    }
    if ((m.alpha_state & 3) == 1) return val.x * 0.212671f + val.y * 0.715160f + val.z * 0.072169f >= m.alpha_threshold;
    return true;
}

// ---------------------------------------------------------------------------
// MicrofacetDistribution (Beckmann / GGX; isotropic or anisotropic alpha)
struct Microfacet {
    uint32_t type;
    float alphaU, alphaV;
    bool sampleVisible;
};

CTL_HD bool mf_isotropic(const Microfacet& d) { return d.alphaU == d.alphaV; }

CTL_HD float mf_eval(const Microfacet& d, f3 m) {                                     // .cu:6-45
    if (m.z <= 0) return 0.0f;
    const float cosTheta2 = m.z * m.z;
    const float beckmannExponent = ((m.x * m.x) / (d.alphaU * d.alphaU) + (m.y * m.y) / (d.alphaV * d.alphaV)) / cosTheta2;
    float result;
    if (d.type == CTL_MICROFACET_BECKMANN) {
        result = cr_exp(-beckmannExponent) / (CTL_PI * d.alphaU * d.alphaV * cosTheta2 * cosTheta2);
    } else {
        const float root = (1 + beckmannExponent) * cosTheta2;
        result = 1.0f / (CTL_PI * d.alphaU * d.alphaV * root * root);
    }
    if (result < 1e-20f) result = 0;
    return result;
}

CTL_HD float mf_project_roughness(const Microfacet& d, f3 v) {                        // .h:128-137
    const float invSinTheta2 = 1 / (1.0f - v.z * v.z);
    if (mf_isotropic(d) || invSinTheta2 <= 0) return d.alphaU;
    const float cosPhi2 = v.x * v.x * invSinTheta2, sinPhi2 = v.y * v.y * invSinTheta2;
    return sqrtf(cosPhi2 * d.alphaU * d.alphaU + sinPhi2 * d.alphaV * d.alphaV);
}

CTL_HD float mf_smithG1(const Microfacet& d, f3 v, f3 m) {                            // .cu:304-336
    if (dot(v, m) * v.z <= 0) return 0.0f;
    float tanTheta;
    {   // math::abs(Frame::tanTheta(v))
        const float temp = 1 - v.z * v.z;
        tanTheta = temp <= 0.0f ? 0.0f : fabsf(sqrtf(temp) / v.z);
    }
    if (tanTheta == 0.0f) return 1.0f;
    const float alpha = mf_project_roughness(d, v);
    if (d.type == CTL_MICROFACET_BECKMANN) {
        const float a = 1.0f / (alpha * tanTheta);
        if (a >= 1.6f) return 1.0f;
        const float aSqr = a * a;
        return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
    }
    const float root = alpha * tanTheta;
    return 2.0f / (1.0f + hypot2_ref(1.0f, root));
}

CTL_HD float mf_G(const Microfacet& d, f3 wi, f3 wo, f3 m) { return mf_smithG1(d, wi, m) * mf_smithG1(d, wo, m); }

CTL_HD float mf_pdf_visible(const Microfacet& d, f3 wi, f3 m) {                      // .h:112-117
    if (wi.z == 0) return 0.0f;
    return mf_smithG1(d, wi, m) * absdot(wi, m) * mf_eval(d, m) / fabsf(wi.z);
}

CTL_HD f2 mf_sample_visible11(const Microfacet& d, float thetaI, f2 sample) {        // .cu:183-302
    const float SQRT_PI_INV = 1 / sqrtf(CTL_PI);
    f2 slope;
    if (d.type == CTL_MICROFACET_BECKMANN) {
        if (thetaI < 1e-4f) {
            const float r = sqrtf(-cr_log(1.0f - sample.x));
            const float sinPhi = cr_sin(2 * CTL_PI * sample.y), cosPhi = cr_cos(2 * CTL_PI * sample.y);
            return mk2(r * cosPhi, r * sinPhi);
        }
        const float tanThetaI = cr_tan(thetaI);
        const float cotThetaI = 1 / tanThetaI;
        float a = -1, c = erf_ref(cotThetaI);
        const float sample_x = tmax(sample.x, 1e-6f);
        const float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
        float b = c - (1 + c) * cr_pow(1 - sample_x, fit);
        const float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * cr_exp(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            const float invErf = erfinv_ref(b);
            const float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * cr_exp(-invErf * invErf)) - sample_x;
            const float derivative = normalization * (1 - invErf * tanThetaI);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0) c = b;
            else a = b;
            b -= value / derivative;
        }
        slope.x = erfinv_ref(b);
        slope.y = erfinv_ref(2.0f * tmax(sample.y, 1e-6f) - 1.0f);
        return slope;
    }
    // GGX
    if (thetaI < 1e-4f) {
        const float r = safe_sqrt_ref(sample.x / (1 - sample.x));
        const float sinPhi = cr_sin(2 * CTL_PI * sample.y), cosPhi = cr_cos(2 * CTL_PI * sample.y);
        return mk2(r * cosPhi, r * sinPhi);
    }
    const float tanThetaI = cr_tan(thetaI);
    const float a = 1 / tanThetaI;
    const float G1 = 2.0f / (1.0f + safe_sqrt_ref(1.0f + 1.0f / (a * a)));
    float A = 2.0f * sample.x / G1 - 1.0f;
    if (fabsf(A) == 1) A -= signum_ref(A) * 1e-7f;
    const float tmp = 1.0f / (A * A - 1.0f);
    const float B = tanThetaI;
    const float D = safe_sqrt_ref(B * B * tmp * tmp - (A * A - B * B) * tmp);
    const float slope_x_1 = B * tmp - D;
    const float slope_x_2 = B * tmp + D;
    slope.x = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
    float S;
    if (sample.y > 0.5f) {
        S = 1.0f;
        sample.y = 2.0f * (sample.y - 0.5f);
    } else {
        S = -1.0f;
        sample.y = 2.0f * (0.5f - sample.y);
    }
    const float z = (sample.y * (sample.y * (sample.y * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) +
                     0.000152998850436920f) /
                    (sample.y * (sample.y * (sample.y * (sample.y * 0.169507819808272f - 0.397203533833404f) -
                                             0.232500544458471f) + 1.0f) - 0.539825872510702f);
    slope.y = S * z * sqrtf(1.0f + slope.x * slope.x);
    return slope;
}

CTL_HD f3 mf_sample_visible(const Microfacet& d, f3 wi_, f2 sample) {               // .cu:146-181
    const f3 wi = normalize(mk3(d.alphaU * wi_.x, d.alphaV * wi_.y, wi_.z));
    float theta = 0, phi = 0;
    if (wi.z < 0.99999f) {
        theta = cr_acos(wi.z);
        phi = cr_atan2(wi.y, wi.x);
    }
    const float sinPhi = cr_sin(phi), cosPhi = cr_cos(phi);
    f2 slope = mf_sample_visible11(d, theta, sample);
    slope = mk2(cosPhi * slope.x - sinPhi * slope.y, sinPhi * slope.x + cosPhi * slope.y);
    slope.x *= d.alphaU;
    slope.y *= d.alphaV;
    const float normalization = 1.0f / sqrtf(slope.x * slope.x + slope.y * slope.y + (float)1.0);
    return mk3(-slope.x * normalization, -slope.y * normalization, normalization);
}

// sample(wi, sample, pdf) with m_sampleVisible (.h:71-81); sampleAll is not
// on the path (getSampleVisible is true for Beckmann and GGX).
CTL_HD f3 mf_sample(const Microfacet& d, f3 wi, f2 sample, float& pdf) {
    const f3 m = mf_sample_visible(d, wi, sample);
    pdf = mf_pdf_visible(d, wi, m);
    return m;
}

// ---------------------------------------------------------------------------
// FresnelHelper
CTL_HD float fresnel_dielectric_ext(float cosThetaI_, float& cosThetaT_, float eta) {   // :27-57
    if (eta == 1) {
        cosThetaT_ = -cosThetaI_;
        return 0.0f;
    }
    const float scale = (cosThetaI_ > 0) ? 1.0f / eta : eta,
                cosThetaTSqr = 1.0f - (1.0f - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) {
        cosThetaT_ = 0.0f;
        return 1.0f;
    }
    const float cosThetaI = fabsf(cosThetaI_);
    const float cosThetaT = safe_sqrt_ref(cosThetaTSqr);
    const float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    const float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
CTL_HD float fresnel_dielectric_ext(float cosThetaI, float eta) {                     // :191-195
    float cosThetaT;
    return fresnel_dielectric_ext(cosThetaI, cosThetaT, eta);
}
CTL_HD f3 reflect_ref(f3 wi, f3 n) { return normalize((2 * dot(wi, n)) * n - wi); }   // :144-147
CTL_HD f3 refract_ref(f3 wi, f3 n, float eta, float cosThetaT) {                    // :149-155
    if (cosThetaT < 0) eta = 1.0f / eta;
    return n * (dot(wi, n) * eta + cosThetaT) - wi * eta;
}

// ---------------------------------------------------------------------------
// roughdielectric (BSDF_Simple.cu:373-615), constant textures: alpha =
// ConstantTexture::Evaluate().avg() = (0 + a + a + a) * (1/3) (Spectrum.h:180-189)
CTL_HD float avg3_ref(float a) { float s = 0.0f; s += a; s += a; s += a; return s * (1.0f / 3); }

CTL_HD Microfacet rough_distr(const ctl_material& m) {
    Microfacet d;
    d.type = m.distribution;
    d.alphaU = avg3_ref(m.alpha_u);
    d.alphaV = avg3_ref(m.alpha_v);
    d.sampleVisible = m.sample_visible != 0;
    return d;
}

// The rough-dielectric entry points are out of line on the device; the BSDF
// record's fields travel by value and the material as a global pointer, so no
// argument needs a scratch copy around the call.
CTL_TEX_FN float rough_pdf(const ctl_material* matp, bsdf_rec b) {
    const ctl_material& mat = *matp;
    const bool hasReflection = (b.type_mask & CTL_EGLOSSY_REFLECTION) != 0,
               hasTransmission = (b.type_mask & CTL_EGLOSSY_TRANSMISSION) != 0,
               reflect = b.wi.z * b.wo.z > 0;
    f3 H;
    float dwh_dwo;
    if (reflect) {
        if (!(b.type_mask & CTL_EGLOSSY_REFLECTION)) return 0.0f;
        H = normalize(b.wo + b.wi);
        dwh_dwo = 1.0f / (4.0f * dot(b.wo, H));
    } else {
        if (!(b.type_mask & CTL_EGLOSSY_TRANSMISSION)) return 0.0f;
        const float eta = b.wi.z > 0 ? mat.eta : mat.inv_eta;
        H = normalize(b.wi + b.wo * eta);
        const float sqrtDenom = dot(b.wi, H) + eta * dot(b.wo, H);
        dwh_dwo = (eta * eta * dot(b.wo, H)) / (sqrtDenom * sqrtDenom);
    }
    H = H * signum_ref(H.z);
    Microfacet sampleDistr = rough_distr(mat);
    if (!sampleDistr.sampleVisible) {
        const float sc = 1.2f - 0.2f * sqrtf(fabsf(b.wi.z));
        sampleDistr.alphaU *= sc;
        sampleDistr.alphaV *= sc;
    }
    const float sign = signum_ref(b.wi.z);
    float prob = sampleDistr.sampleVisible ? mf_pdf_visible(sampleDistr, sign < 0 ? -b.wi : b.wi, H)
                                           : mf_eval(sampleDistr, H) * H.z;
    if (hasTransmission && hasReflection) {
        const float F = fresnel_dielectric_ext(dot(b.wi, H), mat.eta);
        prob *= reflect ? F : (1 - F);
    }
    return fabsf(prob * dwh_dwo);
}

CTL_TEX_FN spec rough_f(const ctl_material* matp, bsdf_rec b) {
    const ctl_material& mat = *matp;
    const bool reflect = b.wi.z * b.wo.z > 0;
    f3 H;
    if (reflect) {
        if (!(b.type_mask & CTL_EGLOSSY_REFLECTION)) return mk3s(0.0f);
        H = normalize(b.wo + b.wi);
    } else {
        if (!(b.type_mask & CTL_EGLOSSY_TRANSMISSION)) return mk3s(0.0f);
        const float eta = b.wi.z > 0 ? mat.eta : mat.inv_eta;
        H = normalize(b.wi + b.wo * eta);
    }
    H = H * signum_ref(H.z);
    const Microfacet distr = rough_distr(mat);
    const float D = mf_eval(distr, H);
    if (D == 0) return mk3s(0.0f);
    const float F = fresnel_dielectric_ext(dot(b.wi, H), mat.eta);
    const float G = mf_G(distr, b.wi, b.wo, H);
    if (reflect) {
        const float value = F * D * G / (4.0f * fabsf(b.wi.z));
        return mk3(mat.reflectance[0], mat.reflectance[1], mat.reflectance[2]) * value;
    }
    const float eta = b.wi.z > 0.0f ? mat.eta : mat.inv_eta;
    const float sqrtDenom = dot(b.wi, H) + eta * dot(b.wo, H);
    const float value = ((1 - F) * D * G * eta * eta * dot(b.wi, H) * dot(b.wo, H)) / (b.wi.z * sqrtDenom * sqrtDenom);
    const float factor = b.wi.z > 0 ? mat.inv_eta : mat.eta;   // ERadiance
    return mk3(mat.transmittance[0], mat.transmittance[1], mat.transmittance[2]) * fabsf(value * factor * factor);
}

// roughdielectric::sample: returns the weight; `b` and `pdf` come back in
// the result, changed only where the reference's sample writes them.
struct RoughSample { spec w; f3 wo; float pdf; uint32_t sampled_type; };
CTL_HD spec rough_sample_impl(const ctl_material& mat, bsdf_rec& b, float& pdf, f2 sample);
CTL_TEX_FN RoughSample rough_sample(const ctl_material* matp, bsdf_rec b, float pdf, f2 sample) {
    RoughSample r;
    r.w = rough_sample_impl(*matp, b, pdf, sample);
    r.wo = b.wo; r.pdf = pdf; r.sampled_type = b.sampled_type;
    return r;
}
CTL_HD spec rough_sample_impl(const ctl_material& mat, bsdf_rec& b, float& pdf, f2 sample) {
    const bool hasReflection = (b.type_mask & CTL_EGLOSSY_REFLECTION) != 0,
               hasTransmission = (b.type_mask & CTL_EGLOSSY_TRANSMISSION) != 0;
    bool sampleReflection = hasReflection;
    if (!hasReflection && !hasTransmission) return mk3s(0.0f);
    const Microfacet distr = rough_distr(mat);
    Microfacet sampleDistr = distr;
    if (!sampleDistr.sampleVisible) {
        const float sc = 1.2f - 0.2f * sqrtf(fabsf(b.wi.z));
        sampleDistr.alphaU *= sc;
        sampleDistr.alphaV *= sc;
    }
    float microfacetPDF;
    const float sign = signum_ref(b.wi.z);
    const f3 m = mf_sample(sampleDistr, sign < 0 ? -b.wi : b.wi, sample, microfacetPDF);
    if (microfacetPDF == 0) return mk3s(0.0f);
    pdf = microfacetPDF;
    float cosThetaT;
    const float F = fresnel_dielectric_ext(dot(b.wi, m), cosThetaT, mat.eta);
    spec weight = mk3s(1.0f);
    // MonteCarlo::sampleReuse(N_REUSE = 10, sample.x, slot) (MonteCarlo.cu:16-20)
    const uint32_t N_REUSE = 10;
    const uint32_t slot = (uint32_t)(int)(sample.x * N_REUSE);
    sample.x = sample.x * N_REUSE - slot;
    const float sample_z = slot / (float)N_REUSE;
    if (hasReflection && hasTransmission) {
        if (sample_z > F) {
            sampleReflection = false;
            pdf *= 1 - F;
        } else {
            pdf *= F;
        }
    } else {
        weight = weight * (hasReflection ? F : (1 - F));
    }
    float dwh_dwo;
    if (sampleReflection) {
        b.wo = reflect_ref(b.wi, m);
        b.sampled_type = CTL_EGLOSSY_REFLECTION;
        if (b.wi.z * b.wo.z <= 0) return mk3s(0.0f);
        weight = weight * mk3(mat.reflectance[0], mat.reflectance[1], mat.reflectance[2]);
        dwh_dwo = 1.0f / (4.0f * dot(b.wo, m));
    } else {
        if (cosThetaT == 0) return mk3s(0.0f);
        b.wo = normalize(refract_ref(b.wi, m, mat.eta, cosThetaT));
        const float beta = cosThetaT < 0 ? mat.eta : mat.inv_eta;   // bRec.eta
        b.sampled_type = CTL_EGLOSSY_TRANSMISSION;
        if (b.wi.z * b.wo.z >= 0) return mk3s(0.0f);
        const float factor = cosThetaT < 0 ? mat.inv_eta : mat.eta;   // ERadiance
        weight = weight * (mk3(mat.transmittance[0], mat.transmittance[1], mat.transmittance[2]) * (factor * factor));
        const float sqrtDenom = dot(b.wi, m) + beta * dot(b.wo, m);
        dwh_dwo = (beta * beta * dot(b.wo, m)) / (sqrtDenom * sqrtDenom);
    }
    if (distr.sampleVisible) weight = weight * mf_smithG1(distr, b.wo, m);
    else weight = weight * fabsf(mf_eval(distr, m) * mf_G(distr, b.wi, b.wo, m) * dot(b.wi, m) / (microfacetPDF * b.wi.z));
    pdf *= fabsf(dwh_dwo);
    return weight;
}

// ---------------------------------------------------------------------------
// diffuse with an optional image texture for m_reflectance
CTL_HD spec diffuse_reflectance(const ctl_material& m, const dgeom& dg, const TexView* tex) {
    if (m.texture != 0xffffffffu && tex) {
        return image_texture_eval(TexView{tex->tex + m.texture, tex->data}, dg.uv, dg.dudx, dg.dudy, dg.dvdx, dg.dvdy,
                                  dg.has_partials);
    }
    return refl(m);
}

// BSDFALL::sample/f/pdf (BSDF.h:140-208): two-sided flip of wi around the
// lobe, then the type switch.  `tex` = the scene's texture table.  `R`: the
// diffuse reflectance at dg when the caller already evaluated it (a textured
// diffuse hit samples and evaluates the same texture at the same dg for the
// BSDF sample and for next-event estimation: one lookup serves both).
// gm: the same material in global memory (the scene's array element; required
// for rough dielectrics), handed to the out-of-line rough-dielectric calls so
// the caller's register copy of the 80-B record need not be written to scratch
// for them.
CTL_HD spec bsdf_sample(const ctl_material& m, bsdf_rec& b, float& pdf, f2 sample, const dgeom& dg, const TexView* tex,
                        const spec* R, const ctl_material* gm) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) {
        if (!diffuse_sample_dir(m, b, pdf, sample)) return mk3s(0.0f);
        return (R ? *R : diffuse_reflectance(m, dg, tex)) * 1.0f;
    }
    const bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    const RoughSample rs = rough_sample(gm, b, pdf, sample);
    b.wo = rs.wo; b.sampled_type = rs.sampled_type; pdf = rs.pdf;
    const spec res = rs.w;
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

CTL_HD spec bsdf_f(const ctl_material& m, bsdf_rec& b, const dgeom& dg, const TexView* tex, const spec* R,
                   const ctl_material* gm) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) {
        if (!(b.type_mask & m.combined_type)) return mk3s(0.0f);
        return diffuse_f_refl(m, b, R ? *R : diffuse_reflectance(m, dg, tex));
    }
    const bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    spec res = rough_f(gm, b);
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

CTL_HD float bsdf_pdf(const ctl_material& m, bsdf_rec& b, const ctl_material* gm) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) return diffuse_pdf(m, b);
    const bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    float res = rough_pdf(gm, b);
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

}  // namespace ctl

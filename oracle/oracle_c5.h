// oracle_c5.h — TEST INFRASTRUCTURE ONLY (part of oracle.cpp).
//
// CPU restatement of the C5 shading pieces of the reference, for checking
// the device path (cudatracerlib_amd/csrc/ctl_bsdf.h) bit for bit:
//   Math/MathFunc.h            erf (A&S 7.1.26), erfinv (Giles), hypot2, safe_sqrt, signum
//   Engine/MIPMap_device.h     WrapCoordinates                        :34-57
//   Engine/MIPMap.cu           Texel, triangle, evalEWA, eval          :15-233
//   Engine/MIPMap.cpp          KernelMIPMap::m_fDim = (w - 1, h - 1)   :108
//   SceneTypes/Texture.cu      ImageTexture::Evaluate                  :7-33
//   Engine/DifferentialGeometry.cu computePartials                     :5-84
//   Math/AlgebraHelper.h       solveLinearSystem2x2                    :11-24
//   Engine/MicrofacetDistribution.{h,cu}  eval, smithG1, pdfVisible, sampleVisible(11)
//   Math/FresnelHelper.h       fresnelDielectricExt, reflect, refract  :27-160
//   Math/MonteCarlo.cu         sampleReuse(N, pdf, slot)               :16-20
//   SceneTypes/BSDF_Simple.cu  diffuse (textured), roughdielectric     :7-75, 373-615
//   SceneTypes/BSDF.h          BSDFALL two-sided wrapper               :140-208
// Included by oracle.cpp after DG/BRec; uses the oracle's own math types.
#pragma once

namespace c5 {

using namespace oracle;

inline float signum(float v) { return o_copysign(1.0f, v); }
inline float safe_sqrt(float v) { return sqrtf(omax(0.0f, v)); }
template <class T> inline T clampv(T v, T lo, T hi) { return omin(omax(v, lo), hi); }
inline float frac(float f) { return f - floorf(f); }

inline float math_hypot2(float a, float b) {   // math::hypot2
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

inline float erfinv(float x) {
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

inline float erf(float x) {
    float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f, a5 = 1.061405429f;
    float p = 0.3275911f;
    float sign = signum(x);
    x = fabsf(x);
    float t = 1.0f / (1.0f + p * x);
    float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * cr_exp(-x * x);
    return sign * y;
}

// ---------------------------------------------------------------- MIP map
struct Mip {
    const ctl_texture* t;
    const uint32_t* data;
    V2 fdim() const { return v2((float)t->width - 1, (float)t->height - 1); }
};

inline bool wrap_coords(V2 uv, V2 dim, uint32_t w, V2* loc) {
    switch (w) {
        case CTL_WRAP_REPEAT: *loc = v2(frac(uv.x) * dim.x, frac(1.0f - uv.y) * dim.y); return true;
        case CTL_WRAP_CLAMP:
            *loc = v2(clampv(uv.x, 0.0f, 1.0f) * dim.x, clampv(1.0f - uv.y, 0.0f, 1.0f) * dim.y);
            return true;
        case CTL_WRAP_MIRROR:
            loc->x = (int)uv.x % 2 == 0 ? frac(uv.x) : 1.0f - frac(uv.x);
            loc->y = (int)uv.x % 2 == 0 ? frac(uv.y) : 1.0f - frac(uv.y);
            *loc = v2(loc->x * dim.x, loc->y * dim.y);
            return true;
        case CTL_WRAP_BLACK:
            if (uv.x < 0 || uv.x >= 1 || uv.y < 0 || uv.y >= 1) return false;
            *loc = v2(uv.x * dim.x, uv.y * dim.y);
            return true;
    }
    return false;
}

inline Spec texel(const Mip& M, unsigned int level, V2 uv) {
    V2 l;
    if (!wrap_coords(uv, v2((float)(M.t->width >> level), (float)(M.t->height >> level)), M.t->wrap, &l))
        return v3s(0.0f);
    int wl = M.t->width >> level, hl = M.t->height >> level;
    int x = clampv((int)l.x, 0, wl - 1), y = clampv((int)l.y, 0, hl - 1);
    uint32_t c = M.data[M.t->offsets[level] + y * wl + x];
    float r = float(c & 0xff) / 255.0f, g = float((c >> 8) & 0xff) / 255.0f, b = float((c >> 16) & 0xff) / 255.0f;
    return v3(r, g, b);
}

inline Spec triangle(const Mip& M, unsigned int level, V2 uv) {
    level = clampv(level, 0u, M.t->levels - 1);
    V2 s = v2((float)(M.t->width >> level), (float)(M.t->height >> level)), is = v2(1.0f / s.x, 1.0f / s.y);
    V2 l = v2(uv.x * s.x, uv.y * s.y);
    float ds = frac(l.x), dt = frac(l.y);
    return (1.f - ds) * (1.f - dt) * texel(M, level, uv) + (1.f - ds) * dt * texel(M, level, uv + v2(0, is.y)) +
           ds * (1.f - dt) * texel(M, level, uv + v2(is.x, 0)) + ds * dt * texel(M, level, uv + v2(is.x, is.y));
}

inline Spec eval_ewa(const Mip& M, unsigned int level, V2 uv, float A, float B, float C) {
    if (level >= M.t->levels) return texel(M, M.t->levels - 1, v2(0, 0));
    V2 size = v2((float)(M.t->width >> level), (float)(M.t->height >> level));
    float u = uv.x * size.x - 0.5f;
    float v = uv.y * size.y - 0.5f;
    V2 fd = M.fdim();
    V2 ratio = v2(size.x / fd.x, size.y / fd.y);
    A /= ratio.x * ratio.x;
    B /= ratio.x * ratio.y;
    C /= ratio.y * ratio.y;
    float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * sqrtf(C * invDet), deltaV = 2.0f * sqrtf(A * invDet);
    int u0 = (int)ceilf(u - deltaU), u1 = (int)floorf(u + deltaU);
    int v0 = (int)ceilf(v - deltaV), v1 = (int)floorf(v + deltaV);
    float As = A * 64, Bs = B * 64, Cs = C * 64;
    Spec result = v3s(0.0f);
    float denominator = 0.0f;
    float ddq = 2 * As, uu0 = u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = vt - v;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < 64) {
                unsigned int qi = (unsigned int)q;
                if (qi < 64) {
                    const float weight = M.t->weight_lut[(int)q];
                    result = result + texel(M, level, v2((float)ut / size.x, (float)vt / size.y)) * weight;
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return triangle(M, level, uv);
    return spec_div(result, denominator);
}

inline Spec mip_eval(const Mip& M, V2 uv, V2 d0, V2 d1) {
    V2 fd = M.fdim();
    float du0 = d0.x * fd.x, dv0 = d0.y * fd.y, du1 = d1.x * fd.x, dv1 = d1.y * fd.y, du = (du0 + du1) / 2.0f,
          dv = (dv0 + dv1) / 2.0f;
    if (M.t->filter == CTL_TEX_POINT) return texel(M, 0, uv);
    else if (M.t->filter == CTL_TEX_BILINEAR) return triangle(M, 0, uv);
    else if (M.t->filter == CTL_TEX_TRILINEAR) {
        float levela = cr_log2(fd.x / fabsf(du)), levelb = cr_log2(fd.y / fabsf(dv)),
              level = M.t->levels - clampv((levela + levelb) / 2.0f, 1.0f, (float)M.t->levels);
        int iLevel = (int)floorf(level), iLevel2 = clampv(iLevel + 1, 0, (int)M.t->levels - 1);
        float p = level - iLevel;
        Spec texelA = triangle(M, iLevel, uv), texelB = triangle(M, iLevel2, uv);
        return p * texelA + (1 - p) * texelB;
    }
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1,
          F = A * C - B * B * 0.25f;
    float root = sqrtf((A - C) * (A - C) + B * B),   // MIPMap.cu's own hypot2
        Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root),
          majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        float level = cr_log2(omax(majorRadius, 1e-4f));
        int ilevel = (int)floorf(level);
        if (ilevel < 0) return triangle(M, 0, uv);
        float a = level - ilevel;
        return triangle(M, ilevel, uv) * (1.0f - a) + triangle(M, ilevel + 1, uv) * a;
    }
    const float maxAniso = 16;
    if (minorRadius * maxAniso < majorRadius) {
        minorRadius = majorRadius / maxAniso;
        float theta = 0.5f * cr_atan(B / (A - C)), sinTheta = cr_sin(theta), cosTheta = cr_cos(theta);
        float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
              cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    float scale = 1.0f / F;
    A *= scale; B *= scale; C *= scale;
    float level = omax(0.0f, cr_log2(minorRadius));
    int ilevel = (int)level;
    float a = level - ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return triangle(M, ilevel, uv);
    return eval_ewa(M, ilevel, uv, A, B, C) * (1.0f - a) + eval_ewa(M, ilevel + 1, uv, A, B, C) * a;
}

// ImageTexture::Evaluate(DifferentialGeometry) with TextureMapping2D
inline Spec image_eval(const ctl_texture* t, const uint32_t* data, const DG& dg) {
    Mip M{t, data};
    auto xform = [&](V2 p) { return v2(t->m11 * p.x + t->m12 * p.y, t->m21 * p.x + t->m22 * p.y) + v2(t->m13, t->m23); };
    Spec r;
    if (dg.hasUVPartials) {
        V2 uv = xform(dg.uv);
        float dsdx = t->m11 * dg.dudx + t->m12 * dg.dvdx, dsdy = t->m11 * dg.dudy + t->m12 * dg.dvdy;
        float dtdx = t->m21 * dg.dudx + t->m22 * dg.dvdx, dtdy = t->m21 * dg.dudy + t->m22 * dg.dvdy;
        r = mip_eval(M, uv, v2(dsdx, dtdx), v2(dsdy, dtdy));
    } else {
        V2 uv = xform(dg.uv);
        r = t->filter == CTL_TEX_POINT ? texel(M, 0, uv) : triangle(M, 0, uv);
    }
    return r * v3(t->scale[0], t->scale[1], t->scale[2]);
}

// ---------------------------------------------------------------- partials
inline bool solve2x2(const float a[2][2], const float b[2], float x[2]) {
    float det = a[0][0] * a[1][1] - a[0][1] * a[1][0];
    if (fabsf(det) <= 2.93873587705571876e-39f) return false;
    float inverse = (float)1.0f / det;
    x[0] = (a[1][1] * b[0] - a[0][1] * b[1]) * inverse;
    x[1] = (a[0][0] * b[1] - a[1][0] * b[0]) * inverse;
    return true;
}

inline void compute_partials(DG& dg, V3 rxo, V3 rxd, V3 ryo, V3 ryd) {
    float A[2][2], Bx[2], By[2], x[2];
    int axes[2];
    dg.hasUVPartials = true;
    if (dot(dg.dpdu, dg.dpdu) == 0 && dot(dg.dpdv, dg.dpdv) == 0) {
        dg.dudx = dg.dvdx = dg.dudy = dg.dvdy = 0.0f;
        return;
    }
    const float pp = dot(dg.n, dg.P), pox = dot(dg.n, rxo), poy = dot(dg.n, ryo), prx = dot(dg.n, rxd),
                pry = dot(dg.n, ryd);
    if (prx == 0 || pry == 0) {
        dg.dudx = dg.dvdx = dg.dudy = dg.dvdy = 0.0f;
        return;
    }
    const float tx = (pp - pox) / prx, ty = (pp - poy) / pry;
    float absX = fabsf(dg.n.x), absY = fabsf(dg.n.y), absZ = fabsf(dg.n.z);
    if (absX > absY && absX > absZ) { axes[0] = 1; axes[1] = 2; }
    else if (absY > absZ) { axes[0] = 0; axes[1] = 2; }
    else { axes[0] = 0; axes[1] = 1; }
    float dpduA[] = {dg.dpdu.x, dg.dpdu.y, dg.dpdu.z};
    float dpdvA[] = {dg.dpdv.x, dg.dpdv.y, dg.dpdv.z};
    A[0][0] = dpduA[axes[0]];
    A[0][1] = dpdvA[axes[0]];
    A[1][0] = dpduA[axes[1]];
    A[1][1] = dpdvA[axes[1]];
    V3 px = rxo + rxd * tx, py = ryo + ryd * ty;
    float pA[] = {dg.P.x, dg.P.y, dg.P.z};
    float pxA[] = {px.x, px.y, px.z};
    float pyA[] = {py.x, py.y, py.z};
    Bx[0] = pxA[axes[0]] - pA[axes[0]];
    Bx[1] = pxA[axes[1]] - pA[axes[1]];
    By[0] = pyA[axes[0]] - pA[axes[0]];
    By[1] = pyA[axes[1]] - pA[axes[1]];
    if (solve2x2(A, Bx, x)) { dg.dudx = x[0]; dg.dvdx = x[1]; }
    else { dg.dudx = 1; dg.dvdx = 0; }
    if (solve2x2(A, By, x)) { dg.dudy = x[0]; dg.dvdy = x[1]; }
    else { dg.dudy = 0; dg.dvdy = 1; }
}

// ---------------------------------------------------------------- microfacet
struct Distr {
    uint32_t type;
    float au, av;
    bool visible;
    bool isotropic() const { return au == av; }
};

inline float d_eval(const Distr& d, V3 m) {
    if (m.z <= 0) return 0.0f;
    float cosTheta2 = m.z * m.z;
    float e = ((m.x * m.x) / (d.au * d.au) + (m.y * m.y) / (d.av * d.av)) / cosTheta2;
    float result;
    if (d.type == CTL_MICROFACET_BECKMANN) result = cr_exp(-e) / (O_PI * d.au * d.av * cosTheta2 * cosTheta2);
    else {
        float root = (1 + e) * cosTheta2;
        result = 1.0f / (O_PI * d.au * d.av * root * root);
    }
    if (result < 1e-20f) result = 0;
    return result;
}

inline float d_project(const Distr& d, V3 v) {
    float invSinTheta2 = 1 / (1.0f - v.z * v.z);
    if (d.isotropic() || invSinTheta2 <= 0) return d.au;
    float cosPhi2 = v.x * v.x * invSinTheta2, sinPhi2 = v.y * v.y * invSinTheta2;
    return sqrtf(cosPhi2 * d.au * d.au + sinPhi2 * d.av * d.av);
}

inline float d_G1(const Distr& d, V3 v, V3 m) {
    if (dot(v, m) * v.z <= 0) return 0.0f;
    float tt = 1 - v.z * v.z;
    const float tanTheta = fabsf(tt <= 0.0f ? 0.0f : sqrtf(tt) / v.z);
    if (tanTheta == 0.0f) return 1.0f;
    float alpha = d_project(d, v);
    if (d.type == CTL_MICROFACET_BECKMANN) {
        float a = 1.0f / (alpha * tanTheta);
        if (a >= 1.6f) return 1.0f;
        float aSqr = a * a;
        return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
    }
    const float root = alpha * tanTheta;
    return 2.0f / (1.0f + math_hypot2(1.0f, root));
}

inline float d_G(const Distr& d, V3 wi, V3 wo, V3 m) { return d_G1(d, wi, m) * d_G1(d, wo, m); }

inline float d_pdf_visible(const Distr& d, V3 wi, V3 m) {
    if (wi.z == 0) return 0.0f;
    return d_G1(d, wi, m) * fabsf(dot(wi, m)) * d_eval(d, m) / fabsf(wi.z);
}

inline V2 d_visible11(const Distr& d, float thetaI, V2 sample) {
    const float SQRT_PI_INV = 1 / sqrtf(O_PI);
    V2 slope;
    if (d.type == CTL_MICROFACET_BECKMANN) {
        if (thetaI < 1e-4f) {
            float r = sqrtf(-cr_log(1.0f - sample.x));
            float sinPhi = cr_sin(2 * O_PI * sample.y), cosPhi = cr_cos(2 * O_PI * sample.y);
            return v2(r * cosPhi, r * sinPhi);
        }
        float tanThetaI = cr_tan(thetaI);
        float cotThetaI = 1 / tanThetaI;
        float a = -1, c = erf(cotThetaI);
        float sample_x = omax(sample.x, 1e-6f);
        float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
        float b = c - (1 + c) * cr_pow(1 - sample_x, fit);
        float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * cr_exp(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            float invErf = erfinv(b);
            float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * cr_exp(-invErf * invErf)) - sample_x;
            float derivative = normalization * (1 - invErf * tanThetaI);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0) c = b;
            else a = b;
            b -= value / derivative;
        }
        slope.x = erfinv(b);
        slope.y = erfinv(2.0f * omax(sample.y, 1e-6f) - 1.0f);
        return slope;
    }
    if (thetaI < 1e-4f) {
        float r = safe_sqrt(sample.x / (1 - sample.x));
        float sinPhi = cr_sin(2 * O_PI * sample.y), cosPhi = cr_cos(2 * O_PI * sample.y);
        return v2(r * cosPhi, r * sinPhi);
    }
    float tanThetaI = cr_tan(thetaI);
    float a = 1 / tanThetaI;
    float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
    float A = 2.0f * sample.x / G1 - 1.0f;
    if (fabsf(A) == 1) A -= signum(A) * 1e-7f;
    float tmp = 1.0f / (A * A - 1.0f);
    float B = tanThetaI;
    float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
    float slope_x_1 = B * tmp - D;
    float slope_x_2 = B * tmp + D;
    slope.x = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
    float S;
    if (sample.y > 0.5f) { S = 1.0f; sample.y = 2.0f * (sample.y - 0.5f); }
    else { S = -1.0f; sample.y = 2.0f * (0.5f - sample.y); }
    float z = (sample.y * (sample.y * (sample.y * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) +
               0.000152998850436920f) /
              (sample.y * (sample.y * (sample.y * (sample.y * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) +
                           1.0f) - 0.539825872510702f);
    slope.y = S * z * sqrtf(1.0f + slope.x * slope.x);
    return slope;
}

inline V3 d_sample_visible(const Distr& d, V3 _wi, V2 sample) {
    V3 wi = normalize(v3(d.au * _wi.x, d.av * _wi.y, _wi.z));
    float theta = 0, phi = 0;
    if (wi.z < 0.99999f) {
        theta = cr_acos(wi.z);
        phi = cr_atan2(wi.y, wi.x);
    }
    float sinPhi = cr_sin(phi), cosPhi = cr_cos(phi);
    V2 slope = d_visible11(d, theta, sample);
    slope = v2(cosPhi * slope.x - sinPhi * slope.y, sinPhi * slope.x + cosPhi * slope.y);
    slope.x *= d.au;
    slope.y *= d.av;
    float normalization = 1.0f / sqrtf(slope.x * slope.x + slope.y * slope.y + (float)1.0);
    return v3(-slope.x * normalization, -slope.y * normalization, normalization);
}

// ---------------------------------------------------------------- Fresnel
inline float fresnel_ext(float cosThetaI_, float& cosThetaT_, float eta) {
    if (eta == 1) { cosThetaT_ = -cosThetaI_; return 0.0f; }
    float scale = (cosThetaI_ > 0) ? 1.0f / eta : eta,
          cosThetaTSqr = 1.0f - (1.0f - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) { cosThetaT_ = 0.0f; return 1.0f; }
    float cosThetaI = fabsf(cosThetaI_);
    float cosThetaT = safe_sqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
inline float fresnel_ext(float cosThetaI, float eta) { float c; return fresnel_ext(cosThetaI, c, eta); }
inline V3 reflect(V3 wi, V3 n) { return normalize(2 * dot(wi, n) * n - wi); }
inline V3 refract(V3 wi, V3 n, float eta, float cosThetaT) {
    if (cosThetaT < 0) eta = 1.0f / eta;
    return n * (dot(wi, n) * eta + cosThetaT) - wi * eta;
}

// ---------------------------------------------------------------- roughdielectric
inline float const_avg(float a) {   // ConstantTexture(Spectrum(a)).avg() = sum() * (1.0f / 3)
    float s = 0.0f;
    s += a; s += a; s += a;
    return s * (1.0f / 3);
}
inline Distr distr_of(const ctl_material& m) {
    return Distr{m.distribution, const_avg(m.alpha_u), const_avg(m.alpha_v), m.sample_visible != 0};
}
inline Spec spec_refl(const ctl_material& m) { return v3(m.reflectance[0], m.reflectance[1], m.reflectance[2]); }
inline Spec spec_trans(const ctl_material& m) { return v3(m.transmittance[0], m.transmittance[1], m.transmittance[2]); }

inline float rough_pdf(const ctl_material& mt, const BRec& b) {
    bool hasR = (b.typeMask & CTL_EGLOSSY_REFLECTION) != 0, hasT = (b.typeMask & CTL_EGLOSSY_TRANSMISSION) != 0,
         reflect_ = b.wi.z * b.wo.z > 0;
    V3 H;
    float dwh_dwo;
    if (reflect_) {
        if (!(b.typeMask & CTL_EGLOSSY_REFLECTION)) return 0.0f;
        H = normalize(b.wo + b.wi);
        dwh_dwo = 1.0f / (4.0f * dot(b.wo, H));
    } else {
        if (!(b.typeMask & CTL_EGLOSSY_TRANSMISSION)) return 0.0f;
        float eta = b.wi.z > 0 ? mt.eta : mt.inv_eta;
        H = normalize(b.wi + b.wo * eta);
        float sqrtDenom = dot(b.wi, H) + eta * dot(b.wo, H);
        dwh_dwo = (eta * eta * dot(b.wo, H)) / (sqrtDenom * sqrtDenom);
    }
    H = H * signum(H.z);
    Distr sd = distr_of(mt);
    if (!sd.visible) {
        float sc = 1.2f - 0.2f * sqrtf(fabsf(b.wi.z));
        sd.au *= sc; sd.av *= sc;
    }
    float sign = signum(b.wi.z);
    float prob = sd.visible ? d_pdf_visible(sd, sign < 0 ? -b.wi : b.wi, H) : d_eval(sd, H) * H.z;
    if (hasT && hasR) {
        float F = fresnel_ext(dot(b.wi, H), mt.eta);
        prob *= reflect_ ? F : (1 - F);
    }
    return fabsf(prob * dwh_dwo);
}

inline Spec rough_f(const ctl_material& mt, const BRec& b) {
    bool reflect_ = b.wi.z * b.wo.z > 0;
    V3 H;
    if (reflect_) {
        if (!(b.typeMask & CTL_EGLOSSY_REFLECTION)) return v3s(0.0f);
        H = normalize(b.wo + b.wi);
    } else {
        if (!(b.typeMask & CTL_EGLOSSY_TRANSMISSION)) return v3s(0.0f);
        float eta = b.wi.z > 0 ? mt.eta : mt.inv_eta;
        H = normalize(b.wi + b.wo * eta);
    }
    H = H * signum(H.z);
    Distr d = distr_of(mt);
    const float D = d_eval(d, H);
    if (D == 0) return v3s(0.0f);
    const float F = fresnel_ext(dot(b.wi, H), mt.eta);
    const float G = d_G(d, b.wi, b.wo, H);
    if (reflect_) {
        float value = F * D * G / (4.0f * fabsf(b.wi.z));
        return spec_refl(mt) * value;
    }
    float eta = b.wi.z > 0.0f ? mt.eta : mt.inv_eta;
    float sqrtDenom = dot(b.wi, H) + eta * dot(b.wo, H);
    float value = ((1 - F) * D * G * eta * eta * dot(b.wi, H) * dot(b.wo, H)) / (b.wi.z * sqrtDenom * sqrtDenom);
    float factor = b.wi.z > 0 ? mt.inv_eta : mt.eta;
    return spec_trans(mt) * fabsf(value * factor * factor);
}

inline Spec rough_sample(const ctl_material& mt, BRec& b, float& pdf, V2 sample) {
    bool hasR = (b.typeMask & CTL_EGLOSSY_REFLECTION) != 0, hasT = (b.typeMask & CTL_EGLOSSY_TRANSMISSION) != 0,
         sampleReflection = hasR;
    if (!hasR && !hasT) return v3s(0.0f);
    Distr d = distr_of(mt);
    Distr sd = d;
    if (!sd.visible) {
        float sc = 1.2f - 0.2f * sqrtf(fabsf(b.wi.z));
        sd.au *= sc; sd.av *= sc;
    }
    float microfacetPDF;
    float sign = signum(b.wi.z);
    V3 wis = sign < 0 ? -b.wi : b.wi;
    V3 m = d_sample_visible(sd, wis, sample);   // sample() with m_sampleVisible
    microfacetPDF = d_pdf_visible(sd, wis, m);
    if (microfacetPDF == 0) return v3s(0.0f);
    pdf = microfacetPDF;
    float cosThetaT;
    float F = fresnel_ext(dot(b.wi, m), cosThetaT, mt.eta);
    Spec weight = v3s(1.0f);
    unsigned int N_REUSE = 10, slot;
    slot = int(sample.x * N_REUSE);        // MonteCarlo::sampleReuse(N_REUSE, sample.x, slot)
    sample.x = sample.x * N_REUSE - slot;
    float sample_z = slot / (float)N_REUSE;
    if (hasR && hasT) {
        if (sample_z > F) { sampleReflection = false; pdf *= 1 - F; }
        else pdf *= F;
    } else {
        weight = weight * (hasR ? F : (1 - F));
    }
    float dwh_dwo;
    if (sampleReflection) {
        b.wo = reflect(b.wi, m);
        b.sampledType = CTL_EGLOSSY_REFLECTION;
        if (b.wi.z * b.wo.z <= 0) return v3s(0.0f);
        weight = weight * spec_refl(mt);
        dwh_dwo = 1.0f / (4.0f * dot(b.wo, m));
    } else {
        if (cosThetaT == 0) return v3s(0.0f);
        b.wo = normalize(refract(b.wi, m, mt.eta, cosThetaT));
        float eta_s = cosThetaT < 0 ? mt.eta : mt.inv_eta;
        b.sampledType = CTL_EGLOSSY_TRANSMISSION;
        if (b.wi.z * b.wo.z >= 0) return v3s(0.0f);
        float factor = cosThetaT < 0 ? mt.inv_eta : mt.eta;
        weight = weight * (spec_trans(mt) * (factor * factor));
        float sqrtDenom = dot(b.wi, m) + eta_s * dot(b.wo, m);
        dwh_dwo = (eta_s * eta_s * dot(b.wo, m)) / (sqrtDenom * sqrtDenom);
    }
    if (d.visible) weight = weight * d_G1(d, b.wo, m);
    else weight = weight * fabsf(d_eval(d, m) * d_G(d, b.wi, b.wo, m) * dot(b.wi, m) / (microfacetPDF * b.wi.z));
    pdf *= fabsf(dwh_dwo);
    return weight;
}

}  // namespace c5

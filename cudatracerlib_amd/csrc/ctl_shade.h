// ctl_shade.h — the PathTracer shading stage (fp32, reference operation order)
// compiled for gfx950 and, where the host scene compiler needs it (ShapeSet
// precompute), for the host.
//
//   fill_dg            TriangleData::fillDG        Engine/TriangleData.cu:75-103
//   diffuse_*          diffuse::sample/f/pdf       SceneTypes/BSDF_Simple.cu:7-75
//                      + BSDFALL two-sided wrapper SceneTypes/BSDF.h:147-208
//   light_sample_direct DiffuseLight::sampleDirect SceneTypes/Light.cu:84-135
//                      + ShapeSet::SamplePosition  Engine/ShapeSet.cu:51-69
//   light_pdf_direct   DiffuseLight::pdfDirect     SceneTypes/Light.cu:137-155
//   power_heuristic    MonteCarlo::PowerHeuristic  Math/MonteCarlo.h:29-33
#pragma once
#include "ctl_math.h"
#include "../../include/ctl_trace.h"

namespace ctl {

typedef f3 spec;   // RGB Spectrum (SPECTRUM_SAMPLES 3, Math/Spectrum.h:10)
CTL_HD float spec_max(spec s) { float r = s.x; r = tmax(r, s.y); r = tmax(r, s.z); return r; }
CTL_HD bool spec_zero(spec s) { return s.x == 0.0f && s.y == 0.0f && s.z == 0.0f; }
CTL_HD spec spec_div(spec s, float f) { float recip = 1.0f / f; return s * recip; }   // Spectrum.h:122-128

struct dgeom {   // DifferentialGeometry subset used by the path (Engine/DifferentialGeometry.h)
    f3 P;
    frame sys;
    f3 n;
    f3 dpdu, dpdv;                   // world space
    f2 uv;                           // uv[0] (TriangleData holds one UV set)
    float dudx, dudy, dvdx, dvdy;    // computePartials; live for the whole path
    bool has_partials;
};

// NDEC: callable uint32 (16-bit code) -> f3 normal (the device passes a LUT).
template <class NDEC>
CTL_HD void fill_dg(const ctl_triangle_data& td, const m44& L2W, f2 bary, bool half_quirk, const NDEC& ndec,
                    dgeom& dg) {
    const uint32_t* w = td.w;
    f3 na = ndec(w[0] & 0xffffu), nb = ndec(w[0] >> 16), nc = ndec(w[1] & 0xffffu);
    float ww = 1.0f - bary.x - bary.y, u = bary.x, v = bary.y;
    f3 n = normalize(u * na + v * nb + ww * nc);
    f3 dpdu = mk3(half_to_float(w[2] & 0xffffu, half_quirk), half_to_float(w[2] >> 16, half_quirk),
                  half_to_float(w[3] & 0xffffu, half_quirk));
    f3 dpdv = mk3(half_to_float(w[3] >> 16, half_quirk), half_to_float(w[4] & 0xffffu, half_quirk),
                  half_to_float(w[4] >> 16, half_quirk));
    f3 s = dpdu - n * dot(n, dpdu);
    f3 t = cross(s, n);
    s = xform_dir(L2W, s);
    t = xform_dir(L2W, t);
    dg.sys.s = normalize(s);
    dg.sys.t = normalize(t);
    dg.sys.n = normalize(cross(t, s));
    dg.dpdu = xform_dir(L2W, dpdu);
    dg.dpdv = xform_dir(L2W, dpdv);
    dg.n = normalize(cross(dg.dpdu, dg.dpdv));
    {   // UV set 0: three half2 (TriangleData.cu:91-98)
        f2 ta = mk2(half_to_float(w[5] & 0xffffu, half_quirk), half_to_float(w[5] >> 16, half_quirk));
        f2 tb = mk2(half_to_float(w[6] & 0xffffu, half_quirk), half_to_float(w[6] >> 16, half_quirk));
        f2 tc = mk2(half_to_float(w[7] & 0xffffu, half_quirk), half_to_float(w[7] >> 16, half_quirk));
        dg.uv = u * ta + v * tb + ww * tc;
    }
    if (dot(dg.n, dg.sys.n) < 0.0f) dg.n = -dg.n;
}

// The spherical-normal decode without a table (Uchar2ToNormalizedFloat3,
// Compression.h:20-31); the device LUT holds the same values.
struct NormalDecodeRef {
#if defined(__HIP__)
    __host__ __device__
#endif
    f3 operator()(uint32_t c) const { return normal_decode16(c); }
};

// TriIntersectorData::getData (Engine/TriIntersectorData.cu:20-32): the three
// vertices back from the Woop record (inverse of the unit-triangle transform).
CTL_HD void woop_get_hd(const float v[12], f3& v0, f3& v1, f3& v2) {
    m44 m = m44_identity();
    m.set_row(0, mk4(v[4], v[5], v[6], v[7]));
    m.set_row(1, mk4(v[8], v[9], v[10], v[11]));
    m.set_row(2, mk4(v[0], v[1], v[2], v[3]));
    m.at(2, 3) *= -1.0f;
    m = inverse(m);
    f3 e02 = xyz(m.col(0)), e12 = xyz(m.col(1));
    v2 = xyz(m.col(3));
    v0 = v2 + e02;
    v1 = v2 + e12;
}

// ShapeSet::triData::Recalculate (Engine/ShapeSet.cu:11-22) for a light triangle
// whose i_dat / t_dat are set: world-space vertices under the node transform, the
// shading normal at the centroid (fillDG on the host: the half quirk decode) and
// the area.  Shared by the scene compile (DynamicScene::CreateShape) and the
// device update of a moved node (DynamicScene::SetNodeTransform -> RecomputeShape,
// DynamicScene.cpp:433-443).
CTL_HD void light_tri_recalc(const float woop[12], const ctl_triangle_data& td, const m44& mxf, ctl_light_tri& lt) {
    f3 p[3];
    woop_get_hd(woop, p[0], p[1], p[2]);
    dgeom dg;
    fill_dg(td, mxf, mk2(1.0f / 3.0f, 1.0f / 3.0f), true, NormalDecodeRef{}, dg);
    for (int i = 0; i < 3; i++) p[i] = xform_point(mxf, p[i]);
    const float area = 0.5f * length(cross(p[2] - p[0], p[1] - p[0]));
    for (int i = 0; i < 3; i++) { lt.p[i][0] = p[i].x; lt.p[i][1] = p[i].y; lt.p[i][2] = p[i].z; }
    lt.n[0] = dg.sys.n.x; lt.n[1] = dg.sys.n.y; lt.n[2] = dg.sys.n.z;
    lt.area = area;
}

// ShapeSet::Recalculate's area distribution (Engine/ShapeSet.cpp:39-57): the CDF
// over the light's triangles in order, normalised by the summed area.
CTL_HD float shapeset_cdf(const ctl_light_tri* tris, uint32_t n, float* cdf) {
    float sumArea = 0;
    cdf[0] = 0.0f;
    for (uint32_t i = 0; i < n; i++) { sumArea += tris[i].area; cdf[i + 1] = cdf[i] + tris[i].area; }
    for (uint32_t i = 0; i <= n; i++) cdf[i] = cdf[i] / sumArea;
    return sumArea;
}

// DifferentialGeometry::computePartials (Engine/DifferentialGeometry.cu:5-84)
// with AlgebraHelper::solveLinearSystem2x2 (Math/AlgebraHelper.h:11-24).
CTL_HD bool solve2x2_ref(const float a[2][2], const float b[2], float x[2]) {
    const float det = a[0][0] * a[1][1] - a[0][1] * a[1][0];
    if (fabsf(det) <= 2.93873587705571876e-39f) return false;   // RCPOVERFLOW
    const float inverse = (float)1.0f / det;
    x[0] = (a[1][1] * b[0] - a[0][1] * b[1]) * inverse;
    x[1] = (a[0][0] * b[1] - a[1][0] * b[0]) * inverse;
    return true;
}
CTL_HD void compute_partials(dgeom& dg, f3 rxo, f3 rxd, f3 ryo, f3 ryd) {
    // One exit, the four partials stored once in a fixed order: stores in the
    // early-return branches made the compiler keep them in scratch, addressed
    // through a selected offset.
    float dudx = 0.0f, dvdx = 0.0f, dudy = 0.0f, dvdy = 0.0f;
    dg.has_partials = true;
    const float pp = dot(dg.n, dg.P), pox = dot(dg.n, rxo), poy = dot(dg.n, ryo), prx = dot(dg.n, rxd),
                pry = dot(dg.n, ryd);
    if (!(dot(dg.dpdu, dg.dpdu) == 0 && dot(dg.dpdv, dg.dpdv) == 0) && !(prx == 0 || pry == 0)) {
        float A[2][2], Bx[2], By[2], x[2];
        int axes[2];
        const float tx = (pp - pox) / prx, ty = (pp - poy) / pry;
        const float absX = fabsf(dg.n.x), absY = fabsf(dg.n.y), absZ = fabsf(dg.n.z);
        if (absX > absY && absX > absZ) { axes[0] = 1; axes[1] = 2; }
        else if (absY > absZ) { axes[0] = 0; axes[1] = 2; }
        else { axes[0] = 0; axes[1] = 1; }
        A[0][0] = comp(dg.dpdu, axes[0]);
        A[0][1] = comp(dg.dpdv, axes[0]);
        A[1][0] = comp(dg.dpdu, axes[1]);
        A[1][1] = comp(dg.dpdv, axes[1]);
        const f3 px = rxo + rxd * tx, py = ryo + ryd * ty;
        Bx[0] = comp(px, axes[0]) - comp(dg.P, axes[0]);
        Bx[1] = comp(px, axes[1]) - comp(dg.P, axes[1]);
        By[0] = comp(py, axes[0]) - comp(dg.P, axes[0]);
        By[1] = comp(py, axes[1]) - comp(dg.P, axes[1]);
        const bool okx = solve2x2_ref(A, Bx, x);
        dudx = okx ? x[0] : 1.0f; dvdx = okx ? x[1] : 0.0f;
        const bool oky = solve2x2_ref(A, By, x);
        dudy = oky ? x[0] : 0.0f; dvdy = oky ? x[1] : 1.0f;
    }
    dg.dudx = dudx; dg.dudy = dudy; dg.dvdx = dvdx; dg.dvdy = dvdy;
}

struct bsdf_rec { f3 wi, wo; uint32_t sampled_type, type_mask; };

enum : uint32_t { kEAll = 0x1ffu, kEDelta = 0x61u, kESmooth = 0x1eu };

CTL_HD spec refl(const ctl_material& m) { return mk3(m.reflectance[0], m.reflectance[1], m.reflectance[2]); }

// diffuse::sample up to its return value (BSDF_Simple.cu:7-24, pure
// EDiffuseReflection): false = the reference returns 0.
CTL_HD bool diffuse_sample_dir(const ctl_material& m, bsdf_rec& b, float& pdf, f2 sample) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    bool ok;
    if (!(b.type_mask & m.combined_type) || (m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z <= 0)) {
        ok = false;
    } else {
        b.sampled_type = m.combined_type;
        // Warp::squareToCosineHemisphere + squareToUniformDiskConcentric (Math/Warp.h:61-125)
        float r1 = 2.0f * sample.x - 1.0f, r2 = 2.0f * sample.y - 1.0f;
        float phi, r;
        if (r1 == 0 && r2 == 0) { r = phi = 0; }
        else if (r1 * r1 > r2 * r2) { r = r1; phi = (CTL_PI / 4.0f) * (r2 / r1); }
        else { r = r2; phi = (CTL_PI / 2.0f) - (r1 / r2) * (CTL_PI / 4.0f); }
        float sinPhi = cr_sin(phi), cosPhi = cr_cos(phi);
        f2 p = mk2(r * cosPhi, r * sinPhi);
        float z = sqrtf(1.0f - p.x * p.x - p.y * p.y);
        b.wo = mk3(p.x, p.y, z);
        pdf = fabsf(CTL_INV_PI * b.wo.z) * 1.0f;
        ok = true;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return ok;
}

CTL_HD spec diffuse_sample(const ctl_material& m, bsdf_rec& b, float& pdf, f2 sample) {
    return diffuse_sample_dir(m, b, pdf, sample) ? refl(m) * 1.0f : mk3s(0.0f);
}

// diffuse::f (BSDF_Simple.cu:31-43) with the evaluated reflectance R
CTL_HD spec diffuse_f_refl(const ctl_material& m, bsdf_rec& b, spec R) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    spec res = mk3s(0.0f);
    if (b.type_mask & m.combined_type) {
        bool validRefl = m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z > 0 && b.wo.z > 0;
        bool validTrans = m.combined_type == CTL_EDIFFUSE_TRANSMISSION && b.wi.z * b.wo.z < 0;
        spec s = R * (CTL_INV_PI * fabsf(b.wo.z));
        if (validRefl || validTrans) res = s;
        else if (m.combined_type == (CTL_EDIFFUSE_REFLECTION | CTL_EDIFFUSE_TRANSMISSION)) res = s * 0.5f;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

CTL_HD spec diffuse_f(const ctl_material& m, bsdf_rec& b) { return diffuse_f_refl(m, b, refl(m)); }

CTL_HD float diffuse_pdf(const ctl_material& m, bsdf_rec& b) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    float res = 0.0f;
    if (b.type_mask & m.combined_type) {
        bool validRefl = m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z > 0 && b.wo.z > 0;
        bool validTrans = m.combined_type == CTL_EDIFFUSE_TRANSMISSION && b.wi.z * b.wo.z < 0;
        float f = fabsf(CTL_INV_PI * b.wo.z);
        if (validRefl || validTrans) res = f;
        else if (m.combined_type == (CTL_EDIFFUSE_REFLECTION | CTL_EDIFFUSE_TRANSMISSION)) res = f * 0.5f;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

enum : int { kESolidAngle = 1, kEArea = 3, kEDiscrete = 4 };

struct direct_rec {   // DirectSamplingRecord subset
    f3 p, n; float pdf; int measure; f3 ref, refN, d; float dist;
};

// MonteCarlo::sampleReuse (Math/MonteCarlo.cu:7-14), STL_lower_bound (Base/STL.h:39-56)
CTL_HD uint32_t sample_reuse(const float* cdf, uint32_t size, float& sample, float& pdf) {
    const float* first = cdf;
    uint32_t count = size + 1;
    while (count > 0) {
        uint32_t c2 = count / 2;
        const float* mid = first + c2;
        if (*mid < sample) { first = ++mid; count -= c2 + 1; }
        else count = c2;
    }
    uint32_t index = (uint32_t)tmin(tmax(0, int(first - cdf) - 1), int(size - 1));
    pdf = cdf[index + 1] - cdf[index];
    sample = (sample - cdf[index]) / pdf;
    return index;
}

CTL_HD spec light_sample_direct(const ctl_light& L, const ctl_light_tri* tris, const float* cdfs, direct_rec& dRec,
                                f2 s_in) {
    f2 sample = s_in;
    float pdf;
    uint32_t index = sample_reuse(cdfs + L.cdf_first, L.tri_count, sample.y, pdf);
    const ctl_light_tri& sn = tris[L.tri_first + index];
    float a = sqrtf(1.0f - sample.x);
    f2 bary = mk2(1 - a, a * sample.y);
    f3 p0 = mk3(sn.p[0][0], sn.p[0][1], sn.p[0][2]), p1 = mk3(sn.p[1][0], sn.p[1][1], sn.p[1][2]),
       p2 = mk3(sn.p[2][0], sn.p[2][1], sn.p[2][2]);
    dRec.p = bary.x * p0 + bary.y * p1 + (1.f - bary.x - bary.y) * p2;
    dRec.n = mk3(sn.n[0], sn.n[1], sn.n[2]);
    dRec.pdf = 1.0f / L.sum_area;
    dRec.measure = kEArea;
    f3 dir = dRec.p - dRec.ref;
    float distSquared = lenSqr(dir);
    dRec.dist = sqrtf(distSquared);
    dRec.d = dir / dRec.dist;
    float dp = absdot(dRec.d, dRec.n);
    dRec.pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
    dRec.measure = kESolidAngle;
    if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0 && dRec.pdf != 0)
        return spec_div(mk3(L.radiance[0], L.radiance[1], L.radiance[2]), dRec.pdf) * 1.0f;
    dRec.pdf = 0.0f;
    return mk3s(0.0f);
}

CTL_HD float light_pdf_direct(const ctl_light& L, const direct_rec& dRec) {
    if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0) {
        float pdfPos = 1.0f / L.sum_area;
        if (dRec.measure == kESolidAngle) return pdfPos * (dRec.dist * dRec.dist) / absdot(dRec.d, dRec.n);
        else if (dRec.measure == kEArea) return pdfPos;
        return 0.0f;
    }
    return 0.0f;
}

CTL_HD float power_heuristic(float fPdf, float gPdf) {
    float f = 1 * fPdf, g = 1 * gPdf;
    return (f * f) / (f * f + g * g);
}

// m44 from the ABI's row-major float[16]
CTL_HD m44 to_m44(const ctl_float4x4& a) { m44 m; for (int i = 0; i < 16; i++) m.d[i] = a.m[i]; return m; }

}  // namespace ctl

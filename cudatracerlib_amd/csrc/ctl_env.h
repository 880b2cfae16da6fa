// ctl_env.h — the environment light (InfiniteLight, SceneTypes/Light.h:294-367,
// Light.cu:350-511, Light.cpp:10-58) for the host compile and the device
// kernels: importance sampling of the latitude-longitude radiance map through
// its row / column CDFs with a tent offset, the matching solid-angle pdf, and
// the radiance seen along a ray (bilinear at level 0, or filtered with ray
// differentials for the PrimTracer), under m_worldTransform's rotation.
//
//   env_sample_direct  InfiniteLight::sampleDirect + internalSampleDirection (Light.cu:350-365, 420-457)
//   env_pdf_direct     InfiniteLight::pdfDirect + internalPdfDirection      (Light.cu:367-377, 459-479)
//   env_eval           InfiniteLight::evalEnvironment(ray)                  (Light.cu:481-494)
//   env_eval_diff      InfiniteLight::evalEnvironment(ray, rX, rY)          (Light.cu:496-511)
//   env_build_tables   the constructor's CDF / row-weight tables            (Light.cpp:10-58)
#pragma once
#include "ctl_bsdf.h"

namespace ctl {

#define CTL_EPSILON 0.000001f                   // MathFunc.h:21
#define CTL_INV_TWOPI (1.0f / (2.0f * CTL_PI))  // MathFunc.h:14

struct EnvView {
    const ctl_env_light* e;
    const float* data;         // env_data (sampling tables)
    const ctl_texture* tex;    // the scene's texture records
    const uint32_t* texels;    // the scene's texel data
    CTL_HD TexView map() const { return TexView{tex + e->texture, texels}; }
};


// m_worldTransform (Light.h:307, an OrthogonalAffineMap with zero translation):
// TransformDirection = float4x4::TransformDirection (float4x4.h:404-408),
// TransformDirectionTranspose = (dot(d, col0), dot(d, col1), dot(d, col2)) (float4x4.h:424-427)
CTL_HD m44 env_world(const ctl_env_light& L) {
    m44 m = m44_zero();
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m.at(i, j) = L.world[i][j];
    m.at(3, 3) = 1.0f;
    return m;
}
CTL_HD f3 env_to_world(const ctl_env_light& L, f3 d) { return xform_dir(env_world(L), d); }
CTL_HD f3 env_to_local(const ctl_env_light& L, f3 d) {
    const m44 m = env_world(L);
    return mk3(dot(d, xyz(m.col(0))), dot(d, xyz(m.col(1))), dot(d, xyz(m.col(2))));
}

CTL_HD float luminance(spec s) { return s.x * 0.212671f + s.y * 0.715160f + s.z * 0.072169f; }   // Spectrum.cu:174-177

// KernelMIPMap::Sample(float width = 0, int x, int y) (MIPMap.cu:155-172): level 0, clamped texel
CTL_HD spec env_texel(const EnvView& E, int x, int y) {
    const ctl_texture& t = E.tex[E.e->texture];
    const int w = (int)t.width, h = (int)t.height;
    x = clampi_ref(x, 0, w - 1);
    y = clampi_ref(y, 0, h - 1);
    const uint32_t c = E.texels[t.offsets[0] + (uint32_t)y * (uint32_t)w + (uint32_t)x];
    return mk3(unorm8(c & 0xffu), unorm8((c >> 8) & 0xffu), unorm8((c >> 16) & 0xffu));
}

CTL_HD float interval_to_tent(float sample) {   // Warp::intervalToTent (Math/Warp.h:13-27)
    float sign;
    if (sample < 0.5f) {
        sign = 1;
        sample *= 2;
    } else {
        sign = -1;
        sample = 2 * (sample - 0.5f);
    }
    return sign * (1 - sqrtf(sample));
}

CTL_HD void env_internal_sample(const EnvView& E, f2 sample, f3& d, spec& value, float& pdf) {
    const ctl_env_light& L = *E.e;
    const float* cdfRows = E.data + L.cdf_rows;
    const float* cdfCols = E.data + L.cdf_cols;
    const float* rowWeights = E.data + L.row_weights;
    float qpdf;
    const uint32_t row = sample_reuse(cdfRows, (uint32_t)L.size[1], sample.y, qpdf);
    const uint32_t col = sample_reuse(cdfCols + row * (uint32_t)(L.size[0] + 1), (uint32_t)L.size[0], sample.x, qpdf);
    const f2 pos = mk2((float)col, (float)row) + mk2(interval_to_tent(sample.x), interval_to_tent(sample.y));
    const int xPos = clampi_ref((int)floorf(pos.x), 0, (int)(L.size[0] - 1));
    const int yPos = clampi_ref((int)floorf(pos.y), 0, (int)(L.size[1] - 1));
    const float dx1 = pos.x - xPos, dx2 = 1.0f - dx1, dy1 = pos.y - yPos, dy2 = 1.0f - dy1;
    const spec value1 = env_texel(E, xPos, yPos) * dx2 * dy2 + env_texel(E, xPos + 1, yPos) * dx1 * dy2;
    const spec value2 = env_texel(E, xPos, yPos + 1) * dx2 * dy1 + env_texel(E, xPos + 1, yPos + 1) * dx1 * dy1;
    value = (value1 + value2) * mk3(L.scale[0], L.scale[1], L.scale[2]);
    pdf = (luminance(value1) * rowWeights[(int)clampf_ref((float)yPos, 0.0f, L.size[1] - 1.0f)] +
           luminance(value2) * rowWeights[(int)clampf_ref((float)(yPos + 1), 0.0f, L.size[1] - 1.0f)]) *
          L.normalization;
    const float phi = L.pixel_size[0] * (pos.x + 0.5f), theta = L.pixel_size[1] * (pos.y + 0.5f);
    const float sinPhi = cr_sin(phi), cosPhi = cr_cos(phi), sinTheta = cr_sin(theta), cosTheta = cr_cos(theta);
    d = mk3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= tmax(fabsf(sinTheta), CTL_EPSILON);
}

CTL_HD float env_internal_pdf(const EnvView& E, f3 d) {
    const ctl_env_light& L = *E.e;
    const float* rowWeights = E.data + L.row_weights;
    const f2 uv = mk2(cr_atan2(d.x, -d.z) * CTL_INV_TWOPI, cr_acos(tmin(1.0f, tmax(-1.0f, d.y))) * CTL_INV_PI);
    const float u = uv.x * L.size[0] - 0.5f, v = uv.y * L.size[1] - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    const spec value1 = env_texel(E, xPos, yPos) * dx2 * dy2 + env_texel(E, xPos + 1, yPos) * dx1 * dy2;
    const spec value2 = env_texel(E, xPos, yPos + 1) * dx2 * dy1 + env_texel(E, xPos + 1, yPos + 1) * dx1 * dy1;
    const float sinTheta = sqrtf(tmax(0.0f, 1 - d.y * d.y));
    return (luminance(value1) * rowWeights[clampi_ref(yPos, 0, (int)L.size[1] - 1)] +
            luminance(value2) * rowWeights[clampi_ref(yPos + 1, 0, (int)L.size[1] - 1)]) *
           L.normalization / tmax(fabsf(sinTheta), CTL_EPSILON);
}

CTL_HD spec env_sample_direct(const EnvView& E, direct_rec& dRec, f2 sample) {
    const ctl_env_light& L = *E.e;
    spec value;
    f3 d;
    float pdf;
    env_internal_sample(E, sample, d, value, pdf);
    d = env_to_world(L, d);   // d = m_worldTransform.TransformDirection(d) (Light.cu:355)
    dRec.pdf = pdf;
    dRec.p = mk3(L.scene_center[0], L.scene_center[1], L.scene_center[2]) + d * L.scene_radius;
    dRec.n = -normalize(d);
    dRec.dist = L.scene_radius;
    dRec.d = normalize(d);
    dRec.measure = kESolidAngle;
    return spec_div(value, pdf);
}

CTL_HD float env_pdf_direct(const EnvView& E, const direct_rec& dRec) {
    const float pdfSA = env_internal_pdf(E, env_to_local(*E.e, dRec.d));   // Light.cu:369
    if (dRec.measure == kESolidAngle) return pdfSA;
    if (dRec.measure == kEArea) return pdfSA * absdot(dRec.d, dRec.n) / (dRec.dist * dRec.dist);
    return 0.0f;
}

CTL_HD f2 env_uv(f3 v) {
    return mk2(cr_atan2(v.x, -v.z) * CTL_INV_TWOPI, cr_acos(tmin(1.0f, tmax(-1.0f, v.y))) * CTL_INV_PI);
}

// evalEnvironment(ray): KernelMIPMap::Sample(uv, 0) = the bilinear lookup of level 0 (MIPMap.cu:140-153)
CTL_HD spec env_eval(const EnvView& E, f3 dir) {
    const spec value = tex_triangle(E.map(), 0, env_uv(env_to_local(*E.e, dir)));   // Light.cu:483
    return value * mk3(E.e->scale[0], E.e->scale[1], E.e->scale[2]);
}

// evalEnvironment(ray, rX, rY): the map filtered over the ray differentials' footprint
// (rd, rxd, ryd: the world directions of ray, rX, rY; Light.cu:496-511)
CTL_HD spec env_eval_diff(const EnvView& E, f3 rd, f3 rxd, f3 ryd) {
    const f3 v = env_to_local(*E.e, rd);
    const f2 uv = env_uv(v);
    const f3 dvdx = env_to_local(*E.e, rxd) - v, dvdy = env_to_local(*E.e, ryd) - v;
    const float t1 = CTL_INV_TWOPI / (v.x * v.x + v.z * v.z);
    const float t2 = -CTL_INV_PI / tmax(sqrtf(tmax(0.0f, 1.0f - v.y * v.y)), 1e-4f);
    const f2 dudx = mk2(t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y);
    const f2 dudy = mk2(t1 * (dvdy.z * v.x - dvdy.x * v.z), t2 * dvdy.y);
    const spec value = tex_eval(E.map(), uv, dudx, dudy);
    return value * mk3(E.e->scale[0], E.e->scale[1], E.e->scale[2]);
}

// InfiniteLight::InfiniteLight (Light.cpp:10-58): per row the luminance CDF over
// the columns, over the rows the CDF of row sums weighted by sin(theta); fills
// L.size / pixel_size / normalization and writes the three tables into `out`
// (cdf_cols, cdf_rows, row_weights offsets relative to out's start).
inline void env_build_tables(const EnvView& E, ctl_env_light& L, float* out) {
    const ctl_texture& t = E.tex[L.texture];
    const uint32_t w = t.width, h = t.height;
    L.size[0] = (float)w;
    L.size[1] = (float)h;
    L.cdf_cols = 0;
    L.cdf_rows = (w + 1) * h;
    L.row_weights = L.cdf_rows + h + 1;
    float* cdfCols = out + L.cdf_cols;
    float* cdfRows = out + L.cdf_rows;
    float* rowWeights = out + L.row_weights;
    uint32_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    cdfRows[rowPos++] = 0;
    for (uint32_t y = 0; y < h; ++y) {
        float colSum = 0;
        cdfCols[colPos++] = 0;
        for (uint32_t x = 0; x < w; ++x) {
            const spec value = env_texel(E, (int)x, (int)y);
            colSum += luminance(value);
            cdfCols[colPos++] = (float)colSum;
        }
        const float normalization = 1.0f / (float)colSum;
        for (uint32_t x = 1; x < w; ++x) cdfCols[colPos - x - 1] *= normalization;
        cdfCols[colPos - 1] = 1.0f;
        const float weight = cr_sin((y + 0.5f) * CTL_PI / L.size[1]);
        rowWeights[y] = weight;
        rowSum += colSum * weight;
        cdfRows[rowPos++] = (float)rowSum;
    }
    const float normalization = 1.0f / (float)rowSum;
    for (uint32_t y = 1; y < h; ++y) cdfRows[rowPos - y - 1] *= normalization;
    cdfRows[rowPos - 1] = 1.0f;
    L.normalization = 1.0f / (rowSum * (2 * CTL_PI / L.size[0]) * (CTL_PI / L.size[1]));
    L.pixel_size[0] = 2 * CTL_PI / L.size[0];
    L.pixel_size[1] = CTL_PI / L.size[1];
}
inline size_t env_table_floats(uint32_t w, uint32_t h) { return (size_t)(w + 1) * h + (h + 1) + h; }

}  // namespace ctl

// common.h — device pieces shared by the megakernel (ctl_trace.hip) and the
// wavefront pipeline (wavefront.hip): pass parameters, the SequenceSampler,
// sensor rays, AddSample, and the context structure of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "traverse.h"
#include "../ctl_env.h"

namespace ctl {

constexpr int kBlock = 256;

struct PathParams {
    uint32_t width, height;
    int32_t max_path_length, rr_start_depth;
    uint32_t tile_size, tiles_x, num_tiles, num_ranks, rank;
    uint32_t nseq, len;
    int32_t shadow_any_hit;
    int32_t direct;   // KEY_Direct: PathTrace<true> (NEE + MIS) or PathTrace<false>
    bool half_quirk;
    // N > 1 ranks: work items [0, owned_items) are this rank's pixels; then, per
    // owned tile, apron (2 ts + 1 items: left column, top row, corner) -- the
    // other ranks' pixels whose jittered sample can land in the tile (ApronItem)
    uint32_t owned_items;
    uint32_t apron;   // 2 * tile_size + 1 when num_ranks > 1, else 0
};

// d1 / d2: the 1D / 2D draw counters reduced modulo len -- the reference only
// ever uses counter % len (the table row), and (d + 1) % len follows from
// d % len with a compare, so no division (and no loop-held reciprocal) per draw.
struct SamplerDev {   // SequenceSampler (Kernel/Sampler_device.h:59-113)
    const float* s1;
    const float2* s2;
    uint32_t nseq, len, a, b;   // a = idx % nseq, b = (idx / nseq) % nseq
    uint32_t d1, d2;            // draw counters mod len
    __device__ __forceinline__ void init(const float* t1, const float2* t2, const PathParams& P, uint32_t idx,
                                         uint32_t c1, uint32_t c2) {
        s1 = t1; s2 = t2; nseq = P.nseq; len = P.len;
        a = idx % P.nseq; b = (idx / P.nseq) % P.nseq;
        d1 = c1 % len; d2 = c2 % len;
    }
    __device__ __forceinline__ float next1() {
        const uint32_t k = d1;
        float val = 0.0f;
        val += s1[k * nseq + a];
        val += s1[k * nseq + b];
        d1 = d1 + 1 == len ? 0u : d1 + 1;
        return fracf_ref(val);
    }
    __device__ __forceinline__ f2 next2() {
        const uint32_t k = d2;
        float2 p = s2[k * nseq + a], q = s2[k * nseq + b];
        float x = 0.0f, y = 0.0f;
        x += p.x; y += p.y;
        x += q.x; y += q.y;
        d2 = d2 + 1 == len ? 0u : d2 + 1;
        return mk2(fracf_ref(x), fracf_ref(y));
    }
};

struct LutDecode {
    const float4* lut;
    __device__ __forceinline__ f3 operator()(uint32_t c) const { float4 q = lut[c]; return mk3(q.x, q.y, q.z); }
};

__device__ __forceinline__ m44 load_m44(const float4* M) {
    float4 r0 = M[0], r1 = M[1], r2 = M[2], r3 = M[3];
    m44 m;
    m.d[0] = r0.x; m.d[1] = r0.y; m.d[2] = r0.z; m.d[3] = r0.w;
    m.d[4] = r1.x; m.d[5] = r1.y; m.d[6] = r1.z; m.d[7] = r1.w;
    m.d[8] = r2.x; m.d[9] = r2.y; m.d[10] = r2.z; m.d[11] = r2.w;
    m.d[12] = r3.x; m.d[13] = r3.y; m.d[14] = r3.z; m.d[15] = r3.w;
    return m;
}

// Number of set bits of `mask` below the calling lane (mbcnt: no per-lane
// mask register held for the kernel's lifetime).
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// The same pointer, opaque to the optimiser: reads through it (and the
// integer-division reciprocals of the fields read) stay where they are used
// instead of being hoisted out of a loop into registers held for its lifetime.
template <class T>
__device__ __forceinline__ const T* opaque_ptr(const T* p) {
    asm volatile("" : "+s"(p));
    return p;
}

__device__ __forceinline__ void wave_add_u64(unsigned long long* dst, uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

// work item g -> pixel of the owned tiles (tile_id % num_ranks == rank); each
// wave covers an 8x8 pixel block so primary rays in a wave are coherent.
// Work items of one pass: the rank's pixels, then the apron items.
__host__ __device__ inline uint32_t owned_tiles_of(const PathParams& P) {
    return P.num_tiles > P.rank ? (P.num_tiles - P.rank + P.num_ranks - 1) / P.num_ranks : 0u;
}
__host__ __device__ inline uint64_t pass_items_of(const PathParams& P) {
    return (uint64_t)P.owned_items + (uint64_t)owned_tiles_of(P) * P.apron;
}

// Apron items (N > 1 ranks).  A sample lands on floor(pX): its own pixel or,
// when the jitter rounds up, the right / lower / lower-right neighbour, which
// may belong to another rank's tile.  So that every pixel's samples are summed
// by one rank in the 1-GPU order (fold_samples_kernel), the owner of the
// target tile traces such a foreign pixel's path itself: apron item (tile, i)
// is the pixel left of / above / above-left of the tile; it is traced only
// when its sample lands inside that tile (apron_keep), which needs just the
// first sampler draw, so the duplicated work is a few paths per image.
__device__ __forceinline__ bool apron_pixel(const PathParams& P, uint64_t a, uint32_t& px, uint32_t& py,
                                            uint32_t& x0, uint32_t& y0) {
    const uint32_t ts = P.tile_size;
    const uint32_t j = (uint32_t)(a / P.apron), i = (uint32_t)(a % P.apron);
    const uint32_t tile = j * P.num_ranks + P.rank;
    if (tile >= P.num_tiles) return false;
    x0 = (tile % P.tiles_x) * ts;
    y0 = (tile / P.tiles_x) * ts;
    if (i < ts) { if (x0 == 0) return false; px = x0 - 1; py = y0 + i; }
    else if (i < 2 * ts) { if (y0 == 0) return false; px = x0 + (i - ts); py = y0 - 1; }
    else { if (x0 == 0 || y0 == 0) return false; px = x0 - 1; py = y0 - 1; }
    if (px >= P.width || py >= P.height) return false;
    const uint32_t t2 = (py / ts) * P.tiles_x + px / ts;
    return t2 % P.num_ranks != P.rank;   // a pixel of this rank is covered by its own item
}

__device__ __forceinline__ bool work_pixel(const PathParams& P, uint64_t g, uint32_t& px, uint32_t& py) {
    if (P.apron && g >= P.owned_items) {
        uint32_t x0, y0;
        return apron_pixel(P, g - P.owned_items, px, py, x0, y0);
    }
    const uint32_t perTile = P.tile_size * P.tile_size;
    const uint32_t j = (uint32_t)(g / perTile), w = (uint32_t)(g % perTile);
    const uint32_t tile = j * P.num_ranks + P.rank;
    if (tile >= P.num_tiles) return false;
    const uint32_t groupsPerRow = P.tile_size / 8;
    const uint32_t grp = w / 64, lane = w % 64;
    px = (tile % P.tiles_x) * P.tile_size + (grp % groupsPerRow) * 8 + lane % 8;
    py = (tile / P.tiles_x) * P.tile_size + (grp / groupsPerRow) * 8 + lane / 8;
    return px < P.width && py < P.height;
}

// PerspectiveSensor::sampleRayDifferential (SceneTypes/Sensor.cu:130-144), primary ray only
__device__ __forceinline__ void sensor_ray(const DevScene& S, f2 pX, f3& o, f3& d) {
    m44 s2c = to_m44(S.camera.sample_to_camera), tw = to_m44(S.camera.to_world);
    f3 nearP = xform_point(s2c, mk3(pX.x * S.camera.inv_resolution[0], pX.y * S.camera.inv_resolution[1], 0.0f));
    f3 dd = normalize(nearP);
    o = xform_point(tw, mk3s(0.0f));
    d = xform_dir(tw, dd);
}

// Image::AddSample (Engine/Image.cu:22-44); one owner per pixel per pass -> plain RMW
__device__ __forceinline__ void add_sample(ctl_pixel* fb, const PathParams& P, f2 pX, spec col) {
    col.x = tmax(0.0f, col.x); col.y = tmax(0.0f, col.y); col.z = tmax(0.0f, col.z);
    int x = (int)floorf(pX.x), y = (int)floorf(pX.y);
    bool valid = !(isnan(col.x) || isnan(col.y) || isnan(col.z)) && isfinite(col.x) && isfinite(col.y) &&
                 isfinite(col.z) && col.x >= 0.0f && col.y >= 0.0f && col.z >= 0.0f;
    if (x >= 0 && x < (int)P.width && y >= 0 && y < (int)P.height && valid) {
        ctl_pixel* pp = fb + (size_t)y * P.width + x;
        pp->rgb[0] += col.x;
        pp->rgb[1] += col.y;
        pp->rgb[2] += col.z;
        pp->weight_sum += 1.0f;
    }
}

// Work item k of a pass covers pixel work_pixel(k).  Its finished sample lands
// on floor(pX) (Image::AddSample, Engine/Image.cu:22-44), which is the pixel
// itself or, when the jitter rounds up, its right / lower / lower-right
// neighbour, so two samples of one pass can meet on a pixel.  The path kernels
// therefore never add into the framebuffer: each work item stores its sample
// in its own slot (rgb, code), and fold_samples_kernel adds, per target pixel,
// the samples that landed there in work-item order, pass by pass -- the
// additions and their order of one sequential AddSample per work item.
// code: 0 = no sample (dropped as AddSample drops it), 1 + dx + 2 dy = landed
// on (px + dx, py + dy).
// A kernel's by-value record argument read in place from the kernel-argument
// segment (device pass; `arg` itself on the host pass, which never runs it).
// off = the argument's byte offset among the explicit arguments, laid out in
// order at their natural alignment (kernarg_next).
template <class T>
__device__ __forceinline__ const T& kernarg_ref(const T& arg, size_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
    (void)arg;
    return *reinterpret_cast<const T*>((const char*)__builtin_amdgcn_kernarg_segment_ptr() + off);
#else
    (void)off;
    return arg;
#endif
}
// offset of the argument of type B that follows an argument of type A at offset off
template <class A, class B>
constexpr size_t kernarg_next(size_t off) {
    return (off + sizeof(A) + alignof(B) - 1) / alignof(B) * alignof(B);
}

struct SampleSlots {
    float4* s;            // [pass slot][work item]
    uint32_t per_pass;    // work items of one pass
    uint32_t inv;         // min(floor(2^32 / per_pass), 2^32 - 1): k / per_pass in one mul_hi (split)
    // k -> (pass slot, work item of the pass): the mul_hi quotient is exact or
    // one short (k < 2^32), fixed by one compare
    __device__ __forceinline__ void split(uint32_t k, uint32_t& ps, uint32_t& kk) const {
        ps = __umulhi(k, inv);
        kk = k - ps * per_pass;
        if (kk >= per_pass) { kk -= per_pass; ps++; }
    }
};
inline SampleSlots make_slots(float4* s, uint32_t per_pass) {
    const uint64_t q = per_pass ? (1ull << 32) / per_pass : 0;
    return SampleSlots{s, per_pass, (uint32_t)(q > 0xffffffffull ? 0xffffffffull : q)};
}
__device__ __forceinline__ void store_sample(const PathParams& P, const SampleSlots& S, uint32_t ps, uint32_t kk,
                                             uint32_t px, uint32_t py, f2 pX, spec col) {
    col.x = tmax(0.0f, col.x); col.y = tmax(0.0f, col.y); col.z = tmax(0.0f, col.z);
    const int x = (int)floorf(pX.x), y = (int)floorf(pX.y);
    const bool valid = !(isnan(col.x) || isnan(col.y) || isnan(col.z)) && isfinite(col.x) && isfinite(col.y) &&
                       isfinite(col.z) && col.x >= 0.0f && col.y >= 0.0f && col.z >= 0.0f;
    const int dx = x - (int)px, dy = y - (int)py;
    float code = 0.0f;
    if (x >= 0 && x < (int)P.width && y >= 0 && y < (int)P.height && valid && (dx | dy) >= 0 && dx <= 1 && dy <= 1)
        code = (float)(1 + dx + 2 * dy);
    S.s[(size_t)ps * S.per_pass + kk] = make_float4(col.x, col.y, col.z, code);
}

// Apron item g keeps its path only when the sample lands inside its tile.
__device__ __forceinline__ bool apron_keep(const PathParams& P, uint64_t g, f2 pX) {
    if (!P.apron || g < P.owned_items) return true;
    uint32_t px, py, x0, y0;
    apron_pixel(P, g - P.owned_items, px, py, x0, y0);
    const float lx = floorf(pX.x), ly = floorf(pX.y);
    return lx >= (float)x0 && lx < (float)(x0 + P.tile_size) && ly >= (float)y0 && ly < (float)(y0 + P.tile_size);
}

// Work item of source pixel (sx, sy) for a target pixel of tile (x0, y0) owned
// by this rank: its own item, or the tile's apron item when another rank owns it.
__device__ __forceinline__ bool source_item(const PathParams& P, uint32_t sx, uint32_t sy, uint32_t x0, uint32_t y0,
                                            uint32_t& k);

// inverse of work_pixel: owned pixel -> work item (false when another rank owns it)
__device__ __forceinline__ bool pixel_work(const PathParams& P, uint32_t x, uint32_t y, uint32_t& k) {
    const uint32_t ts = P.tile_size;
    const uint32_t tile = (y / ts) * P.tiles_x + x / ts;
    if (tile % P.num_ranks != P.rank) return false;
    const uint32_t xx = x % ts, yy = y % ts;
    k = (tile / P.num_ranks) * ts * ts + ((yy / 8) * (ts / 8) + xx / 8) * 64 + (yy % 8) * 8 + xx % 8;
    return true;
}

__device__ __forceinline__ bool source_item(const PathParams& P, uint32_t sx, uint32_t sy, uint32_t x0, uint32_t y0,
                                            uint32_t& k) {
    if (pixel_work(P, sx, sy, k)) return true;
    if (!P.apron) return false;
    const uint32_t ts = P.tile_size;
    const uint32_t tile = (y0 / ts) * P.tiles_x + x0 / ts;
    uint32_t i;
    if (sx + 1 == x0 && sy + 1 == y0) i = 2 * ts;
    else if (sx + 1 == x0) i = sy - y0;
    else i = ts + (sx - x0);
    k = P.owned_items + (tile / P.num_ranks) * P.apron + i;
    return true;
}

// Loop-carried variables of PathTrace<true> (PathTracer.cu:10-33).  wo and
// brdf_pdf persist: diffuse_sample leaves them untouched when it rejects a
// sample, and the reference then continues with the previous values.
struct PathVars {
    spec cl, cf;
    f3 rori, rdir, last_nor, wo;
    f2 pX;
    float brdf_pdf;
    int depth;
    bool specular;
    // DifferentialGeometry partials: computed at the first hit and kept for the
    // rest of the path (PathTrace's bRec lives across bounces, PathTracer.cu:16,60-61)
    float dudx, dudy, dvdx, dvdy;
    bool has_partials;
    __device__ __forceinline__ void begin(f2 px, f3 o, f3 d) {
        dudx = dudy = dvdx = dvdy = 0.0f;
        has_partials = false;
        cl = mk3s(0.0f); cf = mk3s(1.0f);
        rori = o; rdir = d;
        last_nor = mk3s(0.0f);
        wo = mk3(0.0f, 0.0f, 1.0f);
        pX = px;
        brdf_pdf = 0.0f;
        depth = 0;
        specular = false;
    }
};

// NEE shadow ray of one bounce: origin = the new rori, unoccluded -> cl += add.
// Skipping the add for occluded / absent shadow rays is exact: the reference
// adds cf * (0 / lightPdf) = +0 there (cf is finite and >= 0).
struct ShadowReq {
    f3 d;
    float dist;
    spec add;
    bool valid;
};

// Ray-differential directions of PerspectiveSensor::sampleRayDifferential
// (Sensor.cu:130-144): rX/rY start at the camera and point through nearP + m_dx / m_dy.
__device__ __forceinline__ void sensor_diff(const DevScene& S, f2 pX, f3& o, f3& dX, f3& dY) {
    m44 s2c = to_m44(S.camera.sample_to_camera), tw = to_m44(S.camera.to_world);
    f3 nearP = xform_point(s2c, mk3(pX.x * S.camera.inv_resolution[0], pX.y * S.camera.inv_resolution[1], 0.0f));
    o = xform_point(tw, mk3s(0.0f));
    dX = xform_dir(tw, normalize(nearP + mk3(S.camera.dx[0], S.camera.dx[1], S.camera.dx[2])));
    dY = xform_dir(tw, normalize(nearP + mk3(S.camera.dy[0], S.camera.dy[1], S.camera.dy[2])));
}

// Sensor sample + primary ray of pixel (px, py) (pathKernel2, PathTracer.cu:182-194;
// PerspectiveSensor::sampleRayDifferential, Sensor.cu:130-144).
__device__ __forceinline__ f2 primary_ray(const DevScene& S, SamplerDev& rng, uint32_t px, uint32_t py, f3& o,
                                          f3& dw) {
    f2 pX = mk2((float)px, (float)py) + rng.next2();
    (void)rng.next2();   // aperture sample (unused by PerspectiveSensor)
    sensor_ray(S, pX, o, dw);
    return pX;
}

// Shading level of the path kernels (template FULL, DevScene::full_shading):
// lean = constant diffuse materials only; full = C5 materials (ray
// differentials, partials, the BSDF type switch); alpha = full plus
// alpha-tested traversal (scenes with alpha maps); env = alpha plus the
// environment light.  The alpha test stays out of scenes without alpha maps:
// its code in the leaf loop costs the full kernel 2 % on C5.  The environment
// code lives only in the env instantiation: inlined into the others it costs
// the hot kernel ~80 spilled VGPRs.  A scene with an environment map always
// runs the env level (full shading of constant diffuse materials is exact, see
// shade_hit).
enum : int { kShadeLean = 0, kShadeFull = 1, kShadeEnv = 2, kShadeAlpha = 3 };
// the traversal's ALPHA flag of a shading level
#define CTL_ALPHA_OF(F) ((F) == kShadeEnv || (F) == kShadeAlpha)
// kernels that never trace (wavefront shade, WPT iterate) share the full instantiation
#define CTL_NO_TRACE_LEVEL(F) ((F) == kShadeAlpha ? kShadeFull : (F))

__device__ __forceinline__ EnvView env_view(const DevScene& S) { return EnvView{S.env, S.env_data, S.textures, S.tex_data}; }

// KernelDynamicScene::pdfEmitter (KernelDynamicScene.cu:42-46)
__device__ __forceinline__ float pdf_emitter(const DevScene& S, uint32_t li) {
    return S.light_cdf[li] - (li == 0 ? 0.0f : S.light_cdf[li - 1]);
}

// The escaped-path term of PathTrace (PathTracer.cu:98-111):
// misWeight * cf * EvalEnvironment(r), with r the last traced ray.  Without an
// environment map EvalEnvironment is 0 and the sum stays as it was.
template <int FULL>
__device__ __forceinline__ spec env_miss(const DevScene& S, const PathParams& P, const PathVars& v) {
    if (FULL != kShadeEnv || S.env_index == 0xffffffffu) return (v.cf * 1.0f) * mk3s(0.0f);
    const EnvView E = env_view(S);
    float misWeight = 1.0f;
    if (!(!P.direct || v.depth == 1 || v.specular)) {
        direct_rec dRec;   // DirectSamplingRecFromRay: d = r.dir, solid-angle measure
        dRec.d = v.rdir; dRec.measure = kESolidAngle;
        dRec.ref = v.rori; dRec.refN = v.last_nor; dRec.p = mk3s(0.0f); dRec.n = mk3s(0.0f); dRec.dist = 0.0f;
        const float direct_pdf = env_pdf_direct(E, dRec) * pdf_emitter(S, S.env_index);
        misWeight = power_heuristic(v.brdf_pdf, direct_pdf);
    }
    return (v.cf * misWeight) * env_eval(E, v.rdir);
}

// UniformSampleOneLight up to its occlusion test (TraceAlgorithms.cu:44-73,
// 92-101; sampleEmitter KernelDynamicScene.cu:25-39; needs S.n_lights > 0):
// draws the light choice and the light position, and when both the light
// sample and the BSDF value are non-zero fills the shadow ray and, in sh.add,
// EstimateDirect(...) / pdf -- the value UniformSampleOneLight returns when the
// shadow ray is unoccluded (it returns +0 otherwise).  gm: the material's
// record in the scene array (the rough-dielectric calls read it there; required
// for FULL), R: the diffuse reflectance when already evaluated (or null).
template <int FULL>
__device__ __forceinline__ void nee_sample(const DevScene& S, SamplerDev& rng, const ctl_material& mat,
                                           const bsdf_rec& b, const dgeom& dg, const TexView& tex, ShadowReq& sh,
                                           const spec* R, const ctl_material* gm) {
    f2 sample = rng.next2();
    const uint32_t nl = S.n_lights < CTL_MAX_NUM_LIGHTS ? S.n_lights : CTL_MAX_NUM_LIGHTS;
    uint32_t first = 0, cnt = nl;   // STL_upper_bound
    while (cnt > 0) {
        uint32_t c2 = cnt / 2, mid = first + c2;
        if (!(sample.x < S.light_cdf[mid])) { first = mid + 1; cnt -= c2 + 1; }
        else cnt = c2;
    }
    const uint32_t lidx = first < nl ? first : nl - 1;
    const float fU = S.light_cdf[lidx], fL = lidx > 0 ? S.light_cdf[lidx - 1] : 0.0f;
    sample.x = (sample.x - fL) / (fU - fL);
    const float lpdf = fU - fL;
    direct_rec dRec;
    dRec.p = dg.P; dRec.n = dg.sys.n; dRec.measure = kEArea;
    dRec.ref = dg.P; dRec.refN = dg.sys.n;
    // Light::sampleDirect dispatch: the environment map or a diffuse area light
    const f2 lsample = rng.next2();
    spec value = FULL == kShadeEnv && S.lights[lidx].kind == CTL_LIGHT_INFINITE
                     ? env_sample_direct(env_view(S), dRec, lsample)
                     : light_sample_direct(S.lights[lidx], S.light_tris, S.light_tri_cdf, dRec, lsample);
    if (!spec_zero(value)) {
        bsdf_rec b2 = b;
        b2.wo = to_local(dg.sys, dRec.d);
        b2.type_mask = kEAll & ~kEDelta;
        spec bsdfVal = FULL ? bsdf_f(mat, b2, dg, &tex, R, gm) : diffuse_f(mat, b2);
        if (!spec_zero(bsdfVal)) {
            float weight = 1.0f;
            if (dRec.measure != kEDiscrete)
                weight = power_heuristic(dRec.pdf * lpdf, FULL ? bsdf_pdf(mat, b2, gm) : diffuse_pdf(mat, b2));
            spec ret = value * bsdfVal * weight;
            ret = ret * mk3s(1.0f);
            sh.valid = true;
            sh.d = dRec.d;
            sh.dist = dRec.dist;
            sh.add = spec_div(ret, lpdf);
        }
    }
}

// One closest hit of PathTrace<DIRECT> (PathTracer.cu:35-96; DIRECT = P.direct): emission with MIS,
// BSDF sample, UniformSampleOneLight up to its occlusion test
// (TraceAlgorithms.cu:44-73, 92-101; sampleEmitter KernelDynamicScene.cu:25-39),
// throughput update and Russian roulette.  Returns false when RR ends the path.
// Sampler draws are in the reference order: BSDF 2D, light choice 2D, light
// position 2D, RR 1D.
// FULL = the scene has C5 materials (roughdielectric or image textures): ray
// differentials, partials and the BSDF type switch.  Scenes with constant
// diffuse materials only take the lean instantiation — the partials are only
// observable through textures, so both give identical results there.
// SINGLE: one-instance scene, so the hit's node is ~start_node for every
// lane; indexing with that kernel-uniform value turns the node record and its
// transform into scalar loads.
// part: when non-null (persistent kernel), the path's first-hit partials live in
// this memory slot instead of PathVars, so they hold no VGPRs across the traces;
// they are read back only for a textured material, the one consumer of the
// partials.  has_partials is then `depth > 1` (the first hit always computes them).
// pk: when non-null (persistent kernel, PK = its LDS park), the path variables
// other than the ray, depth / specular and the sampler state are still parked
// in LDS on entry and are read where they are used: pX for the first-hit
// partials, brdf_pdf and last_nor for an emitter's MIS weight, wo and brdf_pdf
// just before the BSDF sample, cl and cf at the end.  So they hold no VGPRs
// across the out-of-line texture and microfacet calls.  The arithmetic is the
// same either way.
struct NoPark {};
template <int FULL, bool SINGLE = false, class PK = NoPark>
__device__ __forceinline__ bool shade_hit(const DevScene& S, const PathParams& P, SamplerDev& rng, PathVars& v,
                                          const HitRec& r, ShadowReq& sh, float4* part = nullptr,
                                          const PK* pk = nullptr) {
    constexpr bool kLazy = !std::is_same<PK, NoPark>::value;
    const uint32_t node = SINGLE ? ~(uint32_t)S.start_node : r.node;
    sh.valid = false;
    bsdf_rec b;
    b.sampled_type = 0;
    b.type_mask = kEAll;
    dgeom dg;
    dg.P = v.rori + r.t * v.rdir;
    const ctl_triangle_data td = S.tri_data[r.tri];
    // Node fields read in place: a local copy of the struct would be indexed
    // dynamically (lights[]) and so live in scratch.
    const ctl_node* N = S.nodes + node;
    fill_dg(td, load_m44(S.xf + 4 * node), mk2(r.u, r.v), P.half_quirk, LutDecode{S.normal_lut}, dg);
    b.wi = to_local(dg.sys, -v.rdir);
    const ctl_material* gmat = S.mats + (((td.w[1] >> 16) & 0xffu) + N->material_offset);
    const ctl_material mat = *gmat;
    if (mat.two_sided && b.wi.z < 0) {
        dg.n = -dg.n;
        dg.sys.n = -dg.sys.n;
        b.wi.z *= -1.0f;
    }
    if (FULL) {
        if (v.depth == 1) {   // bRec.dg.computePartials(r, rX, rY) (PathTracer.cu:60-61)
            if constexpr (kLazy) pk->load_px(v);
            f3 co, dX, dY;
            sensor_diff(S, v.pX, co, dX, dY);
            compute_partials(dg, co, dX, co, dY);
            if (part) {
                *part = make_float4(dg.dudx, dg.dudy, dg.dvdx, dg.dvdy);
            } else {
                v.dudx = dg.dudx; v.dudy = dg.dudy; v.dvdx = dg.dvdx; v.dvdy = dg.dvdy;
                v.has_partials = true;
            }
        } else if (part) {
            dg.has_partials = true;
            float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (mat.texture != 0xffffffffu) q = *part;
            dg.dudx = q.x; dg.dudy = q.y; dg.dvdx = q.z; dg.dvdy = q.w;
        } else {
            dg.dudx = v.dudx; dg.dudy = v.dudy; dg.dvdx = v.dvdx; dg.dvdy = v.dvdy;
            dg.has_partials = v.has_partials;
        }
    }
    const TexView tex{S.textures, S.tex_data};
    if (mat.node_light_index != 0xffffffffu) {
        const uint32_t li = N->lights[mat.node_light_index];
        const ctl_light L = S.lights[li];
        float misWeight = 1.0f;
        if (!(!P.direct || v.depth == 1 || v.specular)) {   // PathTracer.cu:66-67
            if constexpr (kLazy) pk->load_mis(v);
            direct_rec dRec;
            dRec.ref = v.rori; dRec.refN = v.last_nor; dRec.p = dg.P; dRec.n = dg.n;
            dRec.d = v.rdir; dRec.dist = r.t; dRec.measure = kESolidAngle;
            float direct_pdf = light_pdf_direct(L, dRec) * pdf_emitter(S, li);
            misWeight = power_heuristic(v.brdf_pdf, direct_pdf);
        }
        f3 w = -v.rdir;
        spec Le = (dot(dg.sys.n, w) <= 0) ? mk3s(0.0f) : mk3(L.radiance[0], L.radiance[1], L.radiance[2]);
        if constexpr (kLazy) pk->load_cl_cf(v);
        v.cl = v.cl + (v.cf * misWeight) * Le;
        if constexpr (kLazy) pk->store_cl(v);
    }
    // a textured diffuse hit: one texture lookup for the BSDF sample and the NEE evaluation
    // The diffuse reflectance is evaluated here for every diffuse hit (refl(mat)
    // when untextured, the value diffuse_reflectance returns) and handed to the
    // BSDF sample and the NEE evaluation, so the full kernel has one texture
    // call site instead of three (C5 kernel VGPR spills 27 -> 24).
    const bool texd = FULL && mat.bsdf_type == CTL_BSDF_DIFFUSE && mat.texture != 0xffffffffu;
    spec Rtex = refl(mat);
    if (texd) Rtex = diffuse_reflectance(mat, dg, &tex);
    const spec* Rp = FULL ? &Rtex : nullptr;
    if constexpr (kLazy) pk->load_sample_state(v);
    b.wo = v.wo;
    spec f = FULL ? bsdf_sample(mat, b, v.brdf_pdf, rng.next2(), dg, &tex, Rp, gmat)
                  : diffuse_sample(mat, b, v.brdf_pdf, rng.next2());
    v.last_nor = dg.sys.n;
    if (P.direct && (mat.combined_type & kESmooth) != 0 && S.n_lights) {   // PathTracer.cu:82-83
        nee_sample<FULL>(S, rng, mat, b, dg, tex, sh, Rp, gmat);
    }
    if constexpr (kLazy) pk->load_cl_cf(v);
    if (sh.valid) sh.add = v.cf * sh.add;
    v.specular = (b.sampled_type & kEDelta) != 0;
    v.cf = v.cf * f;
    v.rori = dg.P;
    v.rdir = to_world(dg.sys, b.wo);
    v.wo = b.wo;
    if (v.depth > P.rr_start_depth && !v.specular) {
        if (rng.next1() >= spec_max(v.cf)) return false;
        v.cf = spec_div(v.cf, spec_max(v.cf));
    }
    return true;
}

// KernelDynamicScene::Occluded(ray, 0, dist) decided from a finished shadow
// traversal (KernelDynamicScene.cu:70-80): any-hit over (eps, dist - eps), or
// the reference's closest hit tested against (eps, dist - eps), where a miss
// with an infinite dist is not occluded (:77-78).
__device__ __forceinline__ bool shadow_occluded(const DevScene& S, bool any_hit, const HitRec& h, float dist) {
    if (any_hit) return h.tri != 0xffffffffu;
    bool end = h.t < dist - S.ray_eps;
    if (isinf(dist) && h.tri == 0xffffffffu) end = false;
    return h.t > 0 + S.ray_eps && end;
}
// The any-hit shadow query over (eps, dist - eps) culls boxes at
// dist + slab_slack(ray) (traverse.h), not at its acceptance bound: a box whose
// rounded slab entry lands past dist - eps, or past dist (the slab cancels two
// products of size |o| |idir|), can hold a hit below dist - eps, which the
// reference's closest-hit query finds (it culls nothing before its first hit).
// tests/test_shadow_query.py measures the rules against the reference's form.

// Wavefront path state, structure of arrays (capacity = paths per pass).
struct WfState {
    float4* o;        // ray origin xyz | w: brdf_pdf
    float4* d;        // ray direction xyz | w: unused
    float4* cl;       // accumulated radiance xyz | w: pX.x
    float4* cf;       // throughput xyz | w: pX.y
    float4* wo;       // persistent BSDF wo xyz | w: last_nor.x
    float2* ln;       // last_nor.yz
    uint4* meta;      // x: pixel idx, y: d1 | d2 << 16, z: depth | specular << 16, w: has_partials
    float4* part;     // dudx, dudy, dvdx, dvdy (first-hit partials, kept for the path)
    float4* hit;      // t, u, v, tri bits
    uint32_t* hit_node;
    uint32_t* q[2];   // extension-ray queues (path indices), ping-pong
    uint32_t* sq;     // shadow queue (path indices)
    float4* sh_o;     // shadow ray origin | w: tmax (any-hit: dist - eps)
    float4* sh_d;     // shadow ray direction | w: dist
    float4* sh_val;   // contribution to add if unoccluded | w: terminated flag
    uint32_t* sh_occ; // occlusion result
    uint32_t* counts; // [2 * bounce + {0: ext queue, 1: shadow queue}]
    size_t capacity;
};

struct WptBuffers;
struct AnimState;

// Device arrays of an uploaded scene (scene_dev.hip): one allocation per
// KernelDynamicScene stream, reused by ctl_scene_update while it fits.
enum SceneArr : int {
    SA_BVH, SA_WOOP, SA_IDX, SA_TRI, SA_MATS, SA_MESHES, SA_NODES, SA_SBVH, SA_XF, SA_IXF, SA_LIGHTS, SA_LTRIS,
    SA_LCDF, SA_LUT, SA_TEX, SA_TEXDATA, SA_ENV, SA_ENVDATA, SA_WBVH, SA_SWBVH, SA_WBASE,
    SA_COUNT
};
struct SceneArray {
    void* p = nullptr;
    size_t bytes = 0;   // bytes of the current contents
    size_t cap = 0;     // allocated
};

}  // namespace ctl

struct ctl_ctx {
    int device = 0;
    std::string err;
    ctl::SceneArray sarr[ctl::SA_COUNT];
    std::vector<uint32_t> h_wbase;              // host copy of the mesh wide-tree bases
    int stack_mesh_bin = 0, stack_mesh_wide = 0;// worst-case mesh-level stacks (bvh_wide.h)
    int stack_top_bin = -1, stack_top_wide = -1;// top level (-1: no instance tree)
    uint32_t tree_flags = 0;                    // CTL_SCENE_BINARY_BVH / WIDE_QUANT the trees were built for
    uint32_t n_anim_meshes = 0;
    bool device_eps = false;                    // ray_eps derived on the device (set_transform / animate)
    bool device_edited = false;                 // set_transform / animate rewrote device arrays since the upload
    ctl::DevScene scene{};
    bool has_scene = false;
    bool half_quirk = false;
    uint32_t nseq = 4096, len = 30;
    float* d_s1[2] = {nullptr, nullptr};
    float2* d_s2[2] = {nullptr, nullptr};
    // ctl_render_passes: sampler tables of every pass of one launch, and the
    // per-pass sample slices of the owned tiles (folded into the caller's
    // framebuffer in pass order)
    float* d_mt1 = nullptr;
    float2* d_mt2 = nullptr;
    uint32_t mt_cap = 0;        // tables allocated
    float4* d_slices = nullptr; // SampleSlots of the path kernels (common.h)
    uint64_t slices_cap = 0;    // float4 elements allocated
    float* h_s1[2] = {nullptr, nullptr};
    float* h_s2[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    int next_buf = 0, active = -1;
    unsigned long long* d_counters = nullptr;   // [0] rays [1] overflow [2..4] stats
    unsigned long long* h_overflow = nullptr;   // pinned host copy of d_counters[1], read at ctl_sync
    bool overflow_seen = false;                 // sticky: a traversal stack overflowed since the last reset
    // 64-bit work cursors ([0] batch intersect [1] path pass [2] prim pass): resident
    // lanes fetch once more after the work runs out, which a 32-bit cursor
    // near 2^32 items would wrap
    unsigned long long* d_cursors = nullptr;
    std::vector<std::pair<const void*, std::pair<size_t, int>>> resident;   // resident_blocks cache
    hipEvent_t pass_ev[2] = {nullptr, nullptr}; // bracket the last render pass (ctl_last_pass_ms)
    bool pass_timed = false;
    size_t wide_nodes = 0;
    int stack_bound = 0;                        // worst-case traversal stack of the uploaded scene
    uint8_t* d_tile_flags = nullptr;            // PixelVarianceBuffer block flags
    size_t tile_flags_cap = 0;
    uint32_t* d_powers = nullptr;               // XORWOW step powers for sampler_kernel
    ctl::WfState wf{};
    std::vector<void*> wf_allocs;
    ctl::WptBuffers* wpt = nullptr;             // WavefrontPathTracer queues (wpt.hip)
    ctl::AnimState* anim = nullptr;             // animated meshes, refit plans (anim.hip)
    uint64_t n_tri_data = 0, n_woop = 0, n_bvh_nodes = 0, n_scene_bvh = 0;   // uploaded array lengths
    int cu_count = 256;
    // Speculative DoPass windows (ctl_render_pass): the reference's host loop
    // renders one pass per call (Tracer.h:209-248); once the calls follow each
    // other with consecutive sampler passes and nothing else changing, one call
    // renders the next passes too in one launch (their samples wait in the sample
    // slots) and the following calls only fold them.  Anything that changes the
    // scene, the tables, the parameters, the framebuffer or the stream, or uses
    // the slots, drops the pending passes.
    uint64_t scene_epoch = 0;                   // bumped by every scene / table change
    int64_t tables_pass = -1;                   // pass of the active sampler tables (-1: uploaded tables)
    struct Spec {
        bool pending = false;                   // slots hold passes [next, end) of the window
        int64_t first = 0, next = 0, end = 0;
        bool last_valid = false;                // the previous ctl_render_pass call, for the pattern
        int64_t last_pass = 0;
        ctl_pt_params params{};
        const void* fb = nullptr;
        const void* stream = nullptr;
        uint64_t epoch = 0;
        uint32_t streak = 0;                    // windows consumed in a row: their length doubles up to 8
        uint64_t per_pass = 0;
    } spec;
};

namespace ctl {
// Persistent grids = exactly the co-resident blocks (occupancy from the
// compiled register/LDS footprint x CU count): no block waits for a slot and
// the atomic work cursor spreads the pass evenly over all CUs.  Cached per
// context (a context is bound to one device and one host thread at a time).
template <class K>
int resident_blocks(ctl_ctx* c, K kernel, size_t lds) {
    const void* key = reinterpret_cast<const void*>(kernel);
    for (const auto& e : c->resident) if (e.first == key && e.second.first == lds) return e.second.second;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds) != hipSuccess || per_cu <= 0)
        per_cu = 2;
    const int nb = per_cu * c->cu_count;
    c->resident.push_back({key, {lds, nb}});
    return nb;
}

// scene_dev.hip: drops the device scene
void free_scene(ctl_ctx* c);
// wavefront.hip
int wavefront_pass(ctl_ctx* c, const PathParams& P, const SampleSlots& SS, bool stats, hipStream_t s);
void wavefront_free(ctl_ctx* c);
// anim.hip
struct WideNode;
int anim_setup(ctl_ctx* c, const ctl_scene_desc* d, const std::vector<WideNode>& wn, const std::vector<uint32_t>& wbase,
               const std::vector<WideNode>& sw);
void anim_free(ctl_ctx* c);
// wpt.hip
int wpt_pass(ctl_ctx* c, const ctl_wpt_params* p, ctl_pixel* fb, hipStream_t s);
void wpt_free(ctl_ctx* c);
// ctl_trace.hip: the batch traversal launch and the ray counter, for wpt.hip
// (rays, hits)[0, n) and, in the same launch, (rays2, hits2)[0, n2)
int intersect_launch(ctl_ctx* c, int64_t n, const ctl_ray* rays, ctl_hit* hits, int32_t any_hit, hipStream_t s,
                     int64_t n2 = 0, const ctl_ray* rays2 = nullptr, ctl_hit* hits2 = nullptr,
                     const uint32_t* dcount = nullptr, uint32_t band_w = 0);
int count_rays(ctl_ctx* c, uint64_t n, hipStream_t s);
}

// wpt.hip — WavefrontPathTracer (Integrators/PseudoRealtime/WavefrontPathTracer.cu:17-189)
// over a DoubleRayBuffer (Kernel/DoubleRayBuffer.h:13-231): the second caller of
// the batch traversal (ctl_intersect's kernel).
//
// Per bounce:
//   traverse   payload rays, closest hit; last bounce's shadow rays, closest hit
//              (DoubleRayBuffer::FinishIteration, DoubleRayBuffer.h:84-112)
//   iterate    one thread per payload element: pathIterateKernel's body
//              (WavefrontPathTracer.cu:51-150) -> continuation ray, shadow ray,
//              flags; AddSample of finished paths
//   scan       block totals -> exclusive offsets (one block)
//   scatter    stable compaction of continuations and shadow rays
//
// The reference assigns queue slots with atomicInc (insertPayloadElement /
// insertSecondaryRay) and a path's random numbers come from its slot
// (g_SamplerData(rayIdx), WavefrontPathTracer.cu:58), so its image depends on
// the order the atomics resolve.  The stable compaction here reproduces the
// sequential order of those atomics — element j's shadow ray and continuation
// get the slots a one-thread run would give them — which makes the pass
// deterministic and lets the CPU oracle follow it bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "common.h"

namespace ctl {

// WavefrontPTRayData (WavefrontPathTracer.h:11-22), 64 B
struct WptPay {
    float4 a;   // throughput xyz | bsdf_pdf
    float4 b;   // L xyz | dDist
    float4 c;   // directF xyz | bits: half x (pixel) | half y << 16, stored as the rounded floats' integers
    uint4 d;    // dIdx | specular_bounce | prev_normal (16-bit spherical code) | source pixel (ours)
};
static_assert(sizeof(WptPay) == 64, "payload is 64 B");

struct WptBuffers {
    size_t capacity = 0;
    WptPay* pay[2] = {nullptr, nullptr};
    ctl_ray* rays[2] = {nullptr, nullptr};
    ctl_hit* hits = nullptr;
    ctl_ray* sec_tmp = nullptr;    // shadow ray of element j (uncompacted)
    ctl_ray* sec = nullptr;        // compacted shadow rays of the last bounce
    ctl_hit* sec_hits = nullptr;
    uint8_t* flags = nullptr;      // bit 0: continues, bit 1: shadow ray
    uint2* blocks = nullptr;       // per-block counts -> exclusive offsets
    float4* samples = nullptr;     // images over 2048 px: a finished path's sample per source pixel (L, bounce + 1)
    size_t sample_capacity = 0;
    // queue counts per bounce: slot b = {payload rays, shadow rays} traced by bounce
    // b, written by bounce b-1's scan; kernels read them on the device, the host
    // reads them back a few bounces late only to stop issuing bounces
    uint32_t* counts = nullptr;
    uint32_t count_slots = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // h_counts is double-buffered over passes: done[b] is recorded after the last
    // count copy of the pass that used buffer b, and the pass two later waits on it
    // before it writes that buffer, so a late copy of a pass issued on another
    // stream cannot overwrite the counts a later pass reads
    uint32_t* h_cnt[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    bool done_pending[2] = {false, false};
    int cur_buf = 0;
    std::vector<void*> allocs;
};
constexpr int kWptLag = 2;   // bounces the host check trails the device by

namespace {

struct WptArgs {
    uint32_t width, height, nseq, len;
    int32_t depth, max_path_length, rr_start_depth;
    uint32_t skip;       // rng.skip(iterationIdx + 2), iterationIdx = m_uPassesDone
    bool half_quirk;
    bool shadow_any;     // CTL_WPT_SHADOW_ANY_HIT: shadow rays as the any-hit query to dist (1 - eps)
    float4* samples;     // non-null: samples go to per-source slots, folded by wpt_fold_kernel
};

__device__ __forceinline__ SamplerDev wpt_rng(const float* s1, const float2* s2, const WptArgs& A, uint32_t idx,
                                              uint32_t skip) {
    SamplerDev r;
    r.s1 = s1; r.s2 = s2; r.nseq = A.nseq; r.len = A.len;
    r.a = idx % A.nseq; r.b = (idx / A.nseq) % A.nseq;
    r.d1 = skip % A.len; r.d2 = skip % A.len;   // draw counters mod len (SamplerDev)
    return r;
}

// pathCreateKernelWPT (WavefrontPathTracer.cu:17-49) with one sample per pixel:
// the payload slot of pixel i is i (rayidx order).
__global__ __launch_bounds__(kBlock) void wpt_create_kernel(DevScene S_arg, WptArgs A, const float* s1, const float2* s2,
                                                            uint32_t n, ctl_ray* rays, WptPay* pay, uint32_t* count0) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) { count0[0] = n; count0[1] = 0u; }   // bounce 0: every pixel, no shadow rays
    if (i >= n) return;
    const uint32_t x = i % A.width, y = i / A.width;
    SamplerDev rng = wpt_rng(s1, s2, A, i, 0);
    // sampleSensorRay(r, Vec2f(x, y) + rng.randomFloat2(), rng.randomFloat2()): arguments left to right
    const f2 pX = mk2((float)x, (float)y) + rng.next2();
    (void)rng.next2();
    f3 o, d;
    sensor_ray(S, pX, o, d);
    ctl_ray r;
    r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z; r.tmin = S.ray_eps;
    r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z; r.tmax = FLT_MAX;
    rays[i] = r;
    WptPay p;
    p.a = make_float4(1.0f, 1.0f, 1.0f, 0.0f);   // throughput = W = Spectrum(1) (Sensor.cu:117)
    p.b = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    p.c = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float((uint32_t)half_round_int(x) | ((uint32_t)half_round_int(y) << 16)));
    p.d = make_uint4(0xffffffffu, 1u, 0u, i);
    pay[i] = p;
}

// KernelDynamicScene::sampleEmitter (KernelDynamicScene.cu:25-39)
__device__ __forceinline__ uint32_t sample_emitter(const DevScene& S, f2& sample, float& emPdf) {
    const uint32_t nl = S.n_lights < CTL_MAX_NUM_LIGHTS ? S.n_lights : CTL_MAX_NUM_LIGHTS;
    uint32_t first = 0, cnt = nl;   // STL_upper_bound
    while (cnt > 0) {
        uint32_t c2 = cnt / 2, mid = first + c2;
        if (!(sample.x < S.light_cdf[mid])) { first = mid + 1; cnt -= c2 + 1; }
        else cnt = c2;
    }
    const uint32_t idx = first < nl ? first : nl - 1;
    const float fU = S.light_cdf[idx], fL = idx > 0 ? S.light_cdf[idx - 1] : 0.0f;
    sample.x = (sample.x - fL) / (fU - fL);
    emPdf = fU - fL;
    return idx;
}

// pathIterateKernel<NEXT_EVENT_EST> body for payload element j (WavefrontPathTracer.cu:56-148).
template <bool NEE, int FULL>
__global__ __launch_bounds__(kBlock) void wpt_iterate_kernel(DevScene S_arg, WptArgs A, const float* s1, const float2* s2,
                                                             const uint32_t* __restrict__ cnt, WptPay* pay, ctl_ray* rays,
                                                             const ctl_hit* __restrict__ hits,
                                                             const ctl_hit* __restrict__ sec_hits, ctl_ray* sec_tmp,
                                                             uint8_t* flags, uint2* blocks, ctl_pixel* fb) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n = cnt[0];
    if (blockIdx.x * kBlock >= n) return;   // grid sized for the largest queue
    bool cont = false, shadow = false;
    if (j < n) {
        WptPay p = pay[j];
        const ctl_ray ray = rays[j];
        const ctl_hit h = hits[j];
        SamplerDev rng = wpt_rng(s1, s2, A, j, A.skip);   // rng.skip(iterationIdx + 2): plus the camera sample
        spec tp = mk3(p.a.x, p.a.y, p.a.z), L = mk3(p.b.x, p.b.y, p.b.z);
        float bpdf = p.a.w;
        bool specular = p.d.y != 0;
        if (NEE && A.depth > 0 && p.d.x != 0xffffffffu) {
            // accessSecondaryRay: closest hit of the shadow ray against the light distance
            if (sec_hits[p.d.x].dist >= p.b.w * (1 - S.ray_eps)) L = L + mk3(p.c.x, p.c.y, p.c.z);
            p.d.x = 0xffffffffu;
            p.c.x = p.c.y = p.c.z = 0.0f;
        }
        bool terminated = A.depth + 1 == A.max_path_length;
        const f3 ro = mk3(ray.o[0], ray.o[1], ray.o[2]), rd = mk3(ray.d[0], ray.d[1], ray.d[2]);
        ctl_ray next;
        if ((uint32_t)h.tri_idx != 0xffffffffu) {
            // traversalResult::toResult (TraceHelper.cu:44-51): 16-bit barycentrics
            const uint32_t bc = (uint32_t)h.bary;
            const f2 bary = mk2((float)(bc & 0xffffu) / 65535.0f, (float)(bc >> 16) / 65535.0f);
            // TraceResult::getBsdfSample (TraceResult.cu:16-45); wo has no value yet -> (0,0,1)
            bsdf_rec b;
            b.wo = mk3(0.0f, 0.0f, 1.0f);
            b.sampled_type = 0;
            b.type_mask = kEAll;
            dgeom dg;
            dg.P = ro + h.dist * rd;
            const uint32_t tri = (uint32_t)h.tri_idx, node = (uint32_t)h.node_idx;
            const ctl_triangle_data td = S.tri_data[tri];
            const ctl_node* N = S.nodes + node;
            fill_dg(td, load_m44(S.xf + 4 * node), bary, A.half_quirk, LutDecode{S.normal_lut}, dg);
            dg.dudx = dg.dudy = dg.dvdx = dg.dvdy = 0.0f;
            dg.has_partials = false;   // no ray differentials in the wavefront tracer
            b.wi = to_local(dg.sys, -rd);
            const ctl_material* gmat = S.mats + (((td.w[1] >> 16) & 0xffu) + N->material_offset);
            const ctl_material mat = *gmat;
            if (mat.two_sided && b.wi.z < 0) {
                dg.n = -dg.n;
                dg.sys.n = -dg.sys.n;
                b.wi.z *= -1.0f;
            }
            const TexView tex{S.textures, S.tex_data};
            if (mat.node_light_index != 0xffffffffu) {
                const uint32_t li = N->lights[mat.node_light_index];
                const ctl_light Lt = S.lights[li];
                float misWeight = 1.0f;
                if (NEE && !(A.depth == 0 || specular)) {
                    direct_rec dRec;   // DirectSamplingRecFromRay with the stored previous normal
                    dRec.ref = ro; dRec.refN = LutDecode{S.normal_lut}(p.d.z); dRec.p = dg.P; dRec.n = dg.n;
                    dRec.d = rd; dRec.dist = h.dist; dRec.measure = kESolidAngle;
                    float direct_pdf = light_pdf_direct(Lt, dRec) * pdf_emitter(S, li);
                    misWeight = power_heuristic(bpdf, direct_pdf);
                }
                f3 w = -rd;
                spec Le = (dot(dg.sys.n, w) <= 0) ? mk3s(0.0f) : mk3(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
                L = L + (misWeight * Le) * tp;
            }
            bool surviveRR = true;
            if (A.depth >= A.rr_start_depth) {
                if (rng.next1() < spec_max(tp)) tp = spec_div(tp, spec_max(tp));
                else surviveRR = false;
            }
            if (A.depth + 1 != A.max_path_length && surviveRR) {
                // textured diffuse: one texture lookup for the BSDF sample and the NEE evaluation
                const bool texd = FULL && mat.bsdf_type == CTL_BSDF_DIFFUSE && mat.texture != 0xffffffffu;
                spec Rtex = mk3s(0.0f);
                if (texd) Rtex = diffuse_reflectance(mat, dg, &tex);
                const spec* Rp = texd ? &Rtex : nullptr;
                spec f = FULL ? bsdf_sample(mat, b, bpdf, rng.next2(), dg, &tex, Rp, gmat)
                              : diffuse_sample(mat, b, bpdf, rng.next2());
                specular = (b.sampled_type & kEDelta) != 0;
                const f3 out = to_world(dg.sys, b.wo);
                p.d.x = 0xffffffffu;
                if (NEE && (mat.combined_type & kESmooth) != 0) {
                    direct_rec dRec;   // DirectSamplingRecord(P, sys.n)
                    dRec.ref = dg.P; dRec.refN = dg.sys.n; dRec.p = dg.P; dRec.n = dg.sys.n; dRec.measure = kEArea;
                    // sampleEmitterDirect (KernelDynamicScene.cu:98-117): one 2D sample picks the
                    // light and, rescaled, the point on it; no lights -> no emitter, value 0
                    f2 sample = rng.next2();
                    float emPdf = 0.0f;
                    if (S.n_lights) {
                    const uint32_t lidx = sample_emitter(S, sample, emPdf);
                    spec value = FULL == kShadeEnv && S.lights[lidx].kind == CTL_LIGHT_INFINITE
                                     ? env_sample_direct(env_view(S), dRec, sample)
                                     : light_sample_direct(S.lights[lidx], S.light_tris, S.light_tri_cdf, dRec, sample);
                    if (dRec.pdf != 0) {
                        dRec.pdf *= emPdf;
                        value = spec_div(value, emPdf);
                    } else {
                        value = mk3s(0.0f);
                    }
                    if (!spec_zero(value)) {
                        b.type_mask = kEAll & ~kEDelta;
                        b.wo = to_local(dg.sys, dRec.d);
                        spec bsdfVal = FULL ? bsdf_f(mat, b, dg, &tex, Rp, gmat) : diffuse_f(mat, b);
                        const float bsdfPdf = FULL ? bsdf_pdf(mat, b, gmat) : diffuse_pdf(mat, b);
                        const float directPdf = dRec.pdf;   // measure is ESolidAngle after sampleDirect
                        const float weight = power_heuristic(directPdf, bsdfPdf);
                        const spec dF = tp * value * bsdfVal * weight;
                        p.c.x = dF.x; p.c.y = dF.y; p.c.z = dF.z;
                        p.b.w = dRec.dist;
                        ctl_ray sr;
                        sr.o[0] = dg.P.x; sr.o[1] = dg.P.y; sr.o[2] = dg.P.z; sr.tmin = S.ray_eps;
                        // any-hit form: accept t < dist (1 - eps), the bound the compare
                        // in the next iteration tests the closest hit against
                        sr.d[0] = dRec.d.x; sr.d[1] = dRec.d.y; sr.d[2] = dRec.d.z;
                        sr.tmax = A.shadow_any ? p.b.w * (1 - S.ray_eps) : FLT_MAX;
                        sec_tmp[j] = sr;
                        shadow = true;   // dIdx = its slot, set by the scatter
                    }
                    }
                }
                p.d.z = normal_encode16(dg.sys.n);
                tp = tp * f;
                next.o[0] = dg.P.x; next.o[1] = dg.P.y; next.o[2] = dg.P.z; next.tmin = S.ray_eps;
                next.d[0] = out.x; next.d[1] = out.y; next.d[2] = out.z; next.tmax = FLT_MAX;
                cont = true;
            } else {
                terminated = true;
            }
        } else {
            terminated = true;
            // misWeight * throughput * EvalEnvironment(ray) (WavefrontPathTracer.cu:144-157)
            if (FULL == kShadeEnv && S.env_index != 0xffffffffu) {
                const EnvView E = env_view(S);
                float misWeight = 1.0f;
                if (NEE && !(A.depth == 0 || specular)) {
                    direct_rec dRec;   // DirectSamplingRecFromRay: d = ray dir, solid-angle measure
                    dRec.ref = ro; dRec.refN = LutDecode{S.normal_lut}(p.d.z); dRec.p = mk3s(0.0f); dRec.n = mk3s(0.0f);
                    dRec.d = rd; dRec.dist = h.dist; dRec.measure = kESolidAngle;
                    misWeight = power_heuristic(bpdf, env_pdf_direct(E, dRec) * pdf_emitter(S, S.env_index));
                }
                L = L + (misWeight * tp) * env_eval(E, rd);
            } else {
                L = L + (1.0f * tp) * mk3s(0.0f);
            }
        }
        if (terminated) {
            if (A.samples) {
                // the pixel coordinates travel as half: above 2048 several source
                // pixels share a target, so the sample waits for the ordered fold
                A.samples[p.d.w] = make_float4(L.x, L.y, L.z, __int_as_float(A.depth + 1));
            } else {
                const uint32_t hx = __float_as_uint(p.c.w) & 0xffffu, hy = __float_as_uint(p.c.w) >> 16;
                PathParams P{};
                P.width = A.width; P.height = A.height;
                add_sample(fb, P, mk2((float)hx, (float)hy), L);
            }
        }
        if (cont) {
            p.a = make_float4(tp.x, tp.y, tp.z, bpdf);
            p.b.x = L.x; p.b.y = L.y; p.b.z = L.z;
            p.d.y = specular ? 1u : 0u;
            pay[j] = p;
            rays[j] = next;
        }
        flags[j] = (uint8_t)((cont ? 1u : 0u) | (shadow ? 2u : 0u));
    }
    const int nc = __syncthreads_count(cont), ns = __syncthreads_count(shadow);
    if (threadIdx.x == 0) blocks[blockIdx.x] = make_uint2((uint32_t)nc, (uint32_t)ns);
}

// Source range [lo, hi] of pixel coordinate q under the half rounding of the
// payload (__float2half_rn, round to nearest even): {q} below 2048, up to 33
// coordinates near 65504; empty when q is not representable.
__device__ __forceinline__ void half_preimage(uint32_t q, uint32_t n, uint32_t& lo, uint32_t& hi) {
    lo = 1u; hi = 0u;
    if (q < 2048u) { lo = hi = q; return; }
    const uint32_t a = q > 16u ? q - 16u : 0u, b = min(q + 16u, n - 1u);
    for (uint32_t x = a; x <= b; x++) {
        if ((uint32_t)half_round_int(x) == q) {
            if (lo > hi) lo = x;
            hi = x;
        }
    }
}

// AddSample of the finished paths of a pass on images over 2048 px: per target
// pixel, its source pixels' samples in (bounce, image order) -- the sequential
// order of the reference's atomicAdds that the oracle follows -- into PixelData.
__global__ __launch_bounds__(kBlock) void wpt_fold_kernel(WptArgs A, const float4* __restrict__ samples, ctl_pixel* fb) {
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= (uint64_t)A.width * A.height) return;
    const uint32_t qx = (uint32_t)(q % A.width), qy = (uint32_t)(q / A.width);
    uint32_t x0, x1, y0, y1;
    half_preimage(qx, A.width, x0, x1);
    half_preimage(qy, A.height, y0, y1);
    if (x0 > x1 || y0 > y1) return;
    PathParams P{};
    P.width = A.width; P.height = A.height;
    int last = 0;   // bounces are visited in increasing order; sources in image order within one
    for (;;) {
        int next = 0x7fffffff;
        for (uint32_t y = y0; y <= y1; y++)
            for (uint32_t x = x0; x <= x1; x++) {
                const int b = __float_as_int(samples[(size_t)y * A.width + x].w);
                if (b > last && b < next) next = b;
            }
        if (next == 0x7fffffff) break;
        for (uint32_t y = y0; y <= y1; y++)
            for (uint32_t x = x0; x <= x1; x++) {
                const float4 v = samples[(size_t)y * A.width + x];
                if (__float_as_int(v.w) == next) add_sample(fb, P, mk2((float)qx, (float)qy), mk3(v.x, v.y, v.z));
            }
        last = next;
    }
}

// Exclusive scan of the per-block counts in one 1024-thread block.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void wpt_scan_kernel(uint2* blocks, const uint32_t* cnt, uint32_t* totals) {
    __shared__ uint32_t sc[kScanThreads], ss[kScanThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t nb = (cnt[0] + kBlock - 1) / kBlock;
    const uint32_t per = (nb + kScanThreads - 1) / kScanThreads;
    const uint32_t b0 = std::min(nb, t * per), b1 = std::min(nb, b0 + per);
    uint32_t c = 0, s = 0;
    for (uint32_t i = b0; i < b1; i++) { uint2 v = blocks[i]; c += v.x; s += v.y; }
    sc[t] = c; ss[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < kScanThreads; off <<= 1) {   // Hillis-Steele inclusive scan
        uint32_t ac = t >= off ? sc[t - off] : 0u, as = t >= off ? ss[t - off] : 0u;
        __syncthreads();
        sc[t] += ac; ss[t] += as;
        __syncthreads();
    }
    uint32_t oc = sc[t] - c, os = ss[t] - s;
    for (uint32_t i = b0; i < b1; i++) {
        uint2 v = blocks[i];
        blocks[i] = make_uint2(oc, os);
        oc += v.x; os += v.y;
    }
    if (t == kScanThreads - 1) { totals[0] = sc[t]; totals[1] = ss[t]; }
}

// Stable compaction: slot = block offset + preceding waves + preceding lanes.
__global__ __launch_bounds__(kBlock) void wpt_scatter_kernel(const uint32_t* __restrict__ cnt, const uint8_t* __restrict__ flags,
                                                             const uint2* __restrict__ blocks,
                                                             const WptPay* __restrict__ pay_in,
                                                             const ctl_ray* __restrict__ rays_in,
                                                             const ctl_ray* __restrict__ sec_tmp, WptPay* pay_out,
                                                             ctl_ray* rays_out, ctl_ray* sec_out) {
    __shared__ uint32_t wc[kBlock / 64], ws[kBlock / 64];
    const uint32_t n = cnt[0];
    if (blockIdx.x * kBlock >= n) return;
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t f = j < n ? flags[j] : 0u;
    const bool cont = f & 1u, sh = f & 2u;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t mc = __ballot(cont), ms = __ballot(sh);
    if (lane == 0) { wc[wave] = (uint32_t)__popcll(mc); ws[wave] = (uint32_t)__popcll(ms); }
    __syncthreads();
    uint32_t pc = blocks[blockIdx.x].x + (uint32_t)__popcll(mc & lt), ps = blocks[blockIdx.x].y + (uint32_t)__popcll(ms & lt);
    for (uint32_t w = 0; w < wave; w++) { pc += wc[w]; ps += ws[w]; }
    if (cont) {
        WptPay p = pay_in[j];
        p.d.x = sh ? ps : 0xffffffffu;   // insertSecondaryRay's index
        pay_out[pc] = p;
        rays_out[pc] = rays_in[j];
    }
    if (sh) sec_out[ps] = sec_tmp[j];
}

template <class T>
bool wpt_alloc(WptBuffers* B, T** p, size_t n) {
    if (hipMalloc((void**)p, n * sizeof(T) + 64) != hipSuccess) return false;
    B->allocs.push_back((void*)*p);
    return true;
}

#define WPT_HIP(call)                                                          \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) {                                                \
            c->err = std::string("wpt: ") + #call + ": " + hipGetErrorString(e_); \
            return CTL_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

}  // namespace

void wpt_free(ctl_ctx* c) {
    WptBuffers* B = c->wpt;
    if (!B) return;
    for (void* p : B->allocs) (void)hipFree(p);
    for (int b = 0; b < 2; b++) {
        if (B->h_cnt[b]) (void)hipHostFree(B->h_cnt[b]);
        if (B->done[b]) (void)hipEventDestroy(B->done[b]);
    }
    for (hipEvent_t e : B->ev)
        if (e) (void)hipEventDestroy(e);
    delete B;
    c->wpt = nullptr;
}

int wpt_pass(ctl_ctx* c, const ctl_wpt_params* prm, ctl_pixel* fb, hipStream_t s) {
    const ctl_camera& cam = c->scene.camera;
    const uint64_t items = (uint64_t)cam.width * cam.height;
    if (items == 0) return CTL_OK;
    if (cam.width > 65504u || cam.height > 65504u) {   // pixel coordinates travel as half
        c->err = "wpt: image larger than the half-precision pixel coordinates allow";
        return CTL_ERR_INVALID;
    }
    if (items > 0x7fffffffull) { c->err = "wpt: too many pixels"; return CTL_ERR_INVALID; }
    if (!c->wpt) c->wpt = new WptBuffers();
    WptBuffers* B = c->wpt;
    const uint32_t nb_max = (uint32_t)((items + kBlock - 1) / kBlock);
    if (B->capacity < items) {
        WPT_HIP(hipStreamSynchronize(s));
        wpt_free(c);
        c->wpt = B = new WptBuffers();
        const size_t n = items;
        bool ok = wpt_alloc(B, &B->pay[0], n) && wpt_alloc(B, &B->pay[1], n) && wpt_alloc(B, &B->rays[0], n) &&
                  wpt_alloc(B, &B->rays[1], n) && wpt_alloc(B, &B->hits, n) && wpt_alloc(B, &B->sec_tmp, n) &&
                  wpt_alloc(B, &B->sec, n) && wpt_alloc(B, &B->sec_hits, n) && wpt_alloc(B, &B->flags, n) &&
                  wpt_alloc(B, &B->blocks, nb_max);
        for (hipEvent_t& e : B->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
        for (hipEvent_t& e : B->done) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
        if (!ok) { wpt_free(c); c->err = "wpt: buffer allocation failed"; return CTL_ERR_NOMEM; }
        B->capacity = items;
    }
    WptArgs A;
    A.width = cam.width; A.height = cam.height;
    A.nseq = c->nseq; A.len = c->len;
    A.max_path_length = prm->max_path_length;
    A.rr_start_depth = prm->rr_start_depth;
    A.skip = prm->passes_done + 2u;
    A.half_quirk = c->half_quirk;
    A.shadow_any = (prm->flags & CTL_WPT_SHADOW_ANY_HIT) != 0;
    A.depth = 0;
    A.samples = nullptr;
    if (cam.width > 2048u || cam.height > 2048u) {
        if (B->sample_capacity < items) {
            float4* sm = nullptr;
            if (!wpt_alloc(B, &sm, items)) { c->err = "wpt: sample slot allocation failed"; return CTL_ERR_NOMEM; }
            B->samples = sm;
            B->sample_capacity = items;
        }
        A.samples = B->samples;
        WPT_HIP(hipMemsetAsync(A.samples, 0, items * sizeof(float4), s));   // bounce tag 0: no sample
    }
    const float* s1 = c->d_s1[c->active];
    const float2* s2 = c->d_s2[c->active];
    const bool nee = prm->direct != 0;
    const uint32_t full = CTL_NO_TRACE_LEVEL(c->scene.full_shading);

    // count slots for every bounce of the pass (+1 for the last scan's output)
    const uint32_t slots = (uint32_t)prm->max_path_length + 1u;
    if (B->count_slots < slots) {
        WPT_HIP(hipDeviceSynchronize());   // no count copy of an earlier pass in flight
        uint32_t* dc = nullptr;
        if (!wpt_alloc(B, &dc, 2 * (size_t)slots)) { c->err = "wpt: count allocation failed"; return CTL_ERR_NOMEM; }
        for (int b = 0; b < 2; b++) {
            if (B->h_cnt[b]) (void)hipHostFree(B->h_cnt[b]);
            B->h_cnt[b] = nullptr;
            B->done_pending[b] = false;
            if (hipHostMalloc((void**)&B->h_cnt[b], 2 * (size_t)slots * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
                c->err = "wpt: count allocation failed";
                return CTL_ERR_NOMEM;
            }
        }
        B->counts = dc;
        B->count_slots = slots;
    }
    // this pass's host count buffer: the pass that used it last (two passes ago)
    // may still have copies in flight on its stream
    const int hb = B->cur_buf;
    B->cur_buf = 1 - hb;
    if (B->done_pending[hb]) {
        WPT_HIP(hipEventSynchronize(B->done[hb]));
        B->done_pending[hb] = false;
    }
    uint32_t* const h_counts = B->h_cnt[hb];
    const uint32_t n0 = (uint32_t)items;
    int cur = 0;
    hipLaunchKernelGGL(wpt_create_kernel, dim3(nb_max), dim3(kBlock), 0, s, c->scene, A, s1, s2, n0, B->rays[0],
                       B->pay[0], B->counts);
    WPT_HIP(hipGetLastError());
    // The queue sizes stay on the device: every kernel of bounce b reads slot b,
    // the grids are sized for the largest queue (the pass's pixels) and idle
    // blocks exit at once.  The host copies each bounce's totals back and waits
    // only on bounce b - kWptLag's copy, to stop issuing bounces once a queue is
    // empty (the at most kWptLag bounces already issued after it run empty).
    // Queues only shrink (a bounce's continuations and shadow rays are at most its
    // payload), so the last count the host has read back bounds the grids.
    uint32_t ub = n0;
    h_counts[0] = n0;   // slot 0 is written by wpt_create_kernel; its host copy is known
    h_counts[1] = 0u;
    for (int depth = 0;; depth++) {
        const uint32_t* cnt = B->counts + 2 * depth;
        if (depth >= kWptLag) ub = std::min(ub, h_counts[2 * (depth - kWptLag)]);
        const uint32_t nb = (ub + kBlock - 1) / kBlock;
        // FinishIteration: payload rays, then the secondary buffer (closest
        // hit), as one launch over both batches (one resident grid, one tail);
        // the kernel counts the rays it traces
        // bounce 0: the camera rays, one per pixel in row order, traced in 8 x 8 blocks
        int r = intersect_launch(c, ub, B->rays[cur], B->hits, A.shadow_any ? 2 : 0, s, depth ? ub : 0, B->sec, B->sec_hits, cnt,
                                 depth == 0 && (uint64_t)n0 == (uint64_t)A.width * A.height ? A.width : 0u);
        if (r != CTL_OK) return r;
        A.depth = depth;
#define WPT_IT(NE, FU)                                                                                             \
    hipLaunchKernelGGL((wpt_iterate_kernel<NE, FU>), dim3(nb), dim3(kBlock), 0, s, c->scene, A, s1, s2, cnt,      \
                       B->pay[cur], B->rays[cur], B->hits, B->sec_hits, B->sec_tmp, B->flags, B->blocks, fb)
        if (nee) { if (full == kShadeEnv) WPT_IT(true, kShadeEnv); else if (full) WPT_IT(true, kShadeFull); else WPT_IT(true, kShadeLean); }
        else { if (full == kShadeEnv) WPT_IT(false, kShadeEnv); else if (full) WPT_IT(false, kShadeFull); else WPT_IT(false, kShadeLean); }
#undef WPT_IT
        hipLaunchKernelGGL(wpt_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, B->blocks, cnt, B->counts + 2 * (depth + 1));
        hipLaunchKernelGGL(wpt_scatter_kernel, dim3(nb), dim3(kBlock), 0, s, cnt, B->flags, B->blocks, B->pay[cur],
                           B->rays[cur], B->sec_tmp, B->pay[1 - cur], B->rays[1 - cur], B->sec);
        WPT_HIP(hipGetLastError());
        WPT_HIP(hipMemcpyAsync(h_counts + 2 * (depth + 1), B->counts + 2 * (depth + 1), 2 * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, s));
        WPT_HIP(hipEventRecord(B->ev[depth % 4], s));
        cur = 1 - cur;
        // while (!m_ray_buf->isEmpty() && ++pass < maxPathLength)
        if (depth + 1 >= prm->max_path_length) break;
        if (depth >= kWptLag) {
            const int d = depth - kWptLag;
            WPT_HIP(hipEventSynchronize(B->ev[d % 4]));
            if (h_counts[2 * (d + 1)] == 0) break;   // bounce d left no paths: the later ones are empty
        }
    }
    if (A.samples) {
        hipLaunchKernelGGL(wpt_fold_kernel, dim3(nb_max), dim3(kBlock), 0, s, A, (const float4*)A.samples, fb);
        WPT_HIP(hipGetLastError());
    }
    WPT_HIP(hipEventRecord(B->done[hb], s));
    B->done_pending[hb] = true;
    return CTL_OK;
}

}  // namespace ctl

using namespace ctl;

extern "C" {

CTL_API ctl_status ctl_wpt_render_pass(ctl_ctx* c, const ctl_wpt_params* p, ctl_pixel* d_fb, void* stream) {
    if (!c || !p || !d_fb) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "wpt_render_pass: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->active < 0) { c->err = "wpt_render_pass: no sampler tables (call ctl_sampler_generate)"; return CTL_ERR_STATE; }
    if (p->max_path_length < 1) { c->err = "wpt_render_pass: MaxPathLength must be >= 1"; return CTL_ERR_INVALID; }
    if (p->rr_start_depth < 1) { c->err = "wpt_render_pass: RRStartDepth must be >= 1"; return CTL_ERR_INVALID; }
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "wpt_render_pass: hipSetDevice failed"; return CTL_ERR_HIP; }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hipEventRecord(c->pass_ev[0], s) != hipSuccess) { c->err = "wpt_render_pass: event record failed"; return CTL_ERR_HIP; }
    int r = wpt_pass(c, p, d_fb, s);
    if (r != CTL_OK) return (ctl_status)r;
    if (hipEventRecord(c->pass_ev[1], s) != hipSuccess) { c->err = "wpt_render_pass: event record failed"; return CTL_ERR_HIP; }
    c->pass_timed = true;
    return CTL_OK;
}

}  // extern "C"

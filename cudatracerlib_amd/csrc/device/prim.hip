// prim.hip — PrimTracer (Integrators/PrimTracer.cu): one primary ray per pixel
// and a first-hit draw mode, the reference's CPU-runnable BASELINE config C1.
//
//   prim_kernel   persistent grid; a wave takes 64 pixels (an 8x8 block) at a
//                 time from a 64-bit atomic cursor (primaryKernel's per-warp
//                 g_NextRayCounter2 fetch, PrimTracer.cu:181-209), traces the
//                 primary ray (and, for the *_direct modes, the NEE shadow ray)
//                 and writes the pixel (computePixel, PrimTracer.cu:19-106)
//
// The pixel sample is the pixel corner (x, y) itself, without jitter
// (PrimTracer.cu:22); the sampler's first 2-D draw is the (unused) aperture
// sample.  AddSample at integer coordinates lands on the pixel's own entry,
// so every PixelData entry has exactly one writer.
#include <hip/hip_runtime.h>

#include <string>

#include "../../../include/ctl_trace.h"
#include "common.h"

using namespace ctl;

namespace {

struct PrimParams {
    int32_t mode;
    float near_d, far_d;
    uint32_t write_depth;
};

// DeviceDepthImage::NormalizeDepthD3D (Kernel/Tracer.h:26-31)
__device__ __forceinline__ float depth_d3d(float d, float n, float f) {
    const float z = tmin(tmax(d, n), f);   // math::clamp
    return (f / (f - n) * z - f * n / (f - n)) / z;
}

#ifndef CTL_PRIM_WAVES
#define CTL_PRIM_WAVES 0   // waves/SIMD hint for prim_kernel (0: the compiler's choice)
#endif
template <bool SINGLE, int WIDE, int FULL>
__global__ __launch_bounds__(kBlock)
#if CTL_PRIM_WAVES
__attribute__((amdgpu_waves_per_eu(CTL_PRIM_WAVES)))
#endif
void prim_kernel(DevScene S_arg, PathParams P_arg, PrimParams Q, const float* s1,
                                                      const float2* s2, uint64_t items, unsigned long long* cursor,
                                                      unsigned long long* counters, ctl_pixel* fb, float* depth) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    CTL_LANE_STACK(st);
    const int lane = threadIdx.x & 63;
    uint32_t rays = 0;
    bool ok = true;
    TraceStats ts{0, 0, 0};
    while (true) {
        // every lane of the wave is done with its pixel: fetch 64 more
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(cursor, 64ull);
        base = __shfl(base, 0);
        if (base >= items) break;   // wave-uniform
        const uint64_t k = base + (uint64_t)lane;
        uint32_t px, py;
        if (k >= items || !work_pixel(P, k, px, py)) continue;
        const uint32_t idx = py * P.width + px;   // g_SamplerData(rayidx), rayidx = y * w + x
        SamplerDev rng{s1, s2, P.nseq, P.len, idx % P.nseq, (idx / P.nseq) % P.nseq, 0, 0};
        const f2 pX = mk2((float)px, (float)py);
        (void)rng.next2();   // aperture sample of sampleRayDifferential (unused by PerspectiveSensor)
        f3 o, d;
        sensor_ray(S, pX, o, d);
        HitRec h;
        h.t = FLT_MAX; h.u = h.v = 0.0f; h.tri = 0xffffffffu; h.node = 0xffffffffu;
        rays++;
        if (S.n_nodes != 0) ok &= trace_one<0, false, SINGLE, WIDE, CTL_ALPHA_OF(FULL)>(S, o, d, 0.0f, S.ray_eps, h, st, &ts);
        spec L = mk3s(0.0f);
        if (h.tri != 0xffffffffu) {
            if (Q.mode == CTL_PRIM_LINEAR_DEPTH) {
                L = mk3s((h.t - Q.near_d) / (Q.far_d - Q.near_d));
            } else if (Q.mode == CTL_PRIM_D3D_DEPTH) {
                L = mk3s(depth_d3d(h.t, Q.near_d, Q.far_d));
            } else {
                // TraceResult::getBsdfSample (TraceResult.cu:16-45) + computePartials
                const uint32_t node = SINGLE ? ~(uint32_t)S.start_node : h.node;
                const ctl_triangle_data td = S.tri_data[h.tri];
                const ctl_node* N = S.nodes + node;
                dgeom dg;
                dg.P = o + h.t * d;
                fill_dg(td, load_m44(S.xf + 4 * node), mk2(h.u, h.v), P.half_quirk, LutDecode{S.normal_lut}, dg);
                bsdf_rec b;
                b.sampled_type = 0;
                b.type_mask = kEAll;
                b.wi = to_local(dg.sys, -d);
                const ctl_material* gmat = S.mats + (((td.w[1] >> 16) & 0xffu) + N->material_offset);
                const ctl_material mat = *gmat;
                if (mat.two_sided && b.wi.z < 0) {
                    dg.n = -dg.n;
                    dg.sys.n = -dg.sys.n;
                    b.wi.z *= -1.0f;
                }
                if (FULL) {
                    f3 co, dX, dY;
                    sensor_diff(S, pX, co, dX, dY);
                    compute_partials(dg, co, dX, co, dY);
                } else {
                    dg.dudx = dg.dudy = dg.dvdx = dg.dvdy = 0.0f;
                    dg.has_partials = false;
                }
                const f3 w = -d;
                switch (Q.mode) {
                case CTL_PRIM_V_ABSDOT_N_GEO: L = mk3s(absdot(w, dg.n)); break;
                case CTL_PRIM_V_DOT_N_GEO: L = mk3s(dot(w, dg.n)); break;
                case CTL_PRIM_V_DOT_N_SHADE: L = mk3s(dot(w, dg.sys.n)); break;
                case CTL_PRIM_N_GEO_COLORED: { const f3 n = (dg.n + mk3s(1.0f)) / 2.0f; L = n; break; }
                case CTL_PRIM_N_SHADE_COLORED: { const f3 n = (dg.sys.n + mk3s(1.0f)) / 2.0f; L = n; break; }
                case CTL_PRIM_UV: L = mk3(dg.uv.x, dg.uv.y, 0.0f); break;
                case CTL_PRIM_BARY_COORDS: L = mk3(h.u, h.v, 0.0f); break;
                default: {
                    // first_* modes; the supported BSDFs (diffuse, roughdielectric)
                    // have no delta component, so first_non_delta_X == first_X
                    // (PrimTracer.cu:61-67: isDelta is false)
                    b.wo = mk3(0.0f, 0.0f, 1.0f);
                    const TexView tex{S.textures, S.tex_data};
                    const spec f_avg = FULL ? bsdf_f(mat, b, dg, &tex, nullptr, gmat) : diffuse_f(mat, b);
                    spec Le = mk3s(0.0f);   // TraceResult::Le -> DiffuseLight::eval (Light.cu:67-82)
                    if (mat.node_light_index != 0xffffffffu) {
                        const ctl_light Lt = S.lights[N->lights[mat.node_light_index]];
                        Le = (dot(dg.sys.n, w) <= 0) ? mk3s(0.0f) : mk3(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
                    }
                    const spec through = mk3s(1.0f);   // Transmittance without media
                    if (Q.mode == CTL_PRIM_FIRST_LE || Q.mode == CTL_PRIM_FIRST_NON_DELTA_LE) {
                        L = through * Le;
                    } else if (Q.mode == CTL_PRIM_FIRST_F || Q.mode == CTL_PRIM_FIRST_NON_DELTA_F) {
                        L = through * f_avg;
                    } else {   // first_f_direct: Le + through * (UniformSampleOneLight + f_avg * 0.5)
                        spec direct = mk3s(0.0f);
                        if (S.n_lights) {
                            ShadowReq sh;
                            sh.valid = false;
                            nee_sample<FULL>(S, rng, mat, b, dg, tex, sh, nullptr, gmat);
                            if (sh.valid) {
                                // KernelDynamicScene::Occluded (KernelDynamicScene.cu:70-80)
                                HitRec hs;
                                hs.t = sh.dist - S.ray_eps; hs.u = hs.v = 0.0f;
                                hs.tri = 0xffffffffu; hs.node = 0xffffffffu;
                                rays++;
                                ok &= trace_one<1, false, SINGLE, WIDE, CTL_ALPHA_OF(FULL)>(S, dg.P, sh.d, 0.0f, S.ray_eps, hs, st, &ts,
                                                                                             sh.dist);
                                if (!shadow_occluded(S, true, hs, sh.dist)) direct = sh.add;
                            }
                        }
                        L = Le + through * (direct + f_avg * 0.5f);
                    }
                }
                }
            }
        }
        else if (FULL == kShadeEnv && S.env_index != 0xffffffffu) {
            // L = EvalEnvironment(r, rX, rY) (PrimTracer.cu:102): the map filtered
            // over the primary ray's differential footprint
            f3 co, dX, dY;
            sensor_diff(S, pX, co, dX, dY);
            L = env_eval_diff(env_view(S), d, dX, dY);
        }
        add_sample(fb, P, pX, L);   // Image::AddSample((float)x, (float)y, L): the pixel's own entry
        if (Q.write_depth) depth[idx] = depth_d3d(h.t, Q.near_d, Q.far_d);   // g_DepthImage2.Store
    }
    wave_add_u64(&counters[0], rays);
    if (!ok) atomicAdd(&counters[1], 1ull);
}

}  // namespace

#define CTL_HIP(ctx, call)                                                                 \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                \
            return CTL_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

extern "C" {

CTL_API ctl_status ctl_prim_pass(ctl_ctx* c, const ctl_prim_params* p, ctl_pixel* d_fb, float* d_depth,
                                 void* stream) {
    if (!c || !p || !d_fb) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "prim_pass: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->overflow_seen) return CTL_ERR_STATE;
    if (c->active < 0) { c->err = "prim_pass: no sampler tables (call ctl_sampler_generate)"; return CTL_ERR_STATE; }
    if (p->draw_mode < CTL_PRIM_LINEAR_DEPTH || p->draw_mode > CTL_PRIM_FIRST_NON_DELTA_F_DIRECT) {
        c->err = "prim_pass: unknown draw mode";
        return CTL_ERR_INVALID;
    }
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const ctl_camera& cam = c->scene.camera;
    PathParams P{};
    P.width = cam.width; P.height = cam.height;
    P.tile_size = 64;
    P.tiles_x = (cam.width + 63) / 64;
    P.num_tiles = P.tiles_x * ((cam.height + 63) / 64);
    P.num_ranks = 1; P.rank = 0;
    P.nseq = c->nseq; P.len = c->len;
    P.half_quirk = c->half_quirk;
    P.direct = 1;
    const uint64_t items = (uint64_t)P.num_tiles * 64 * 64;
    PrimParams Q{p->draw_mode, p->near_depth, p->far_depth, d_depth ? 1u : 0u};
    CTL_HIP(c, hipEventRecord(c->pass_ev[0], s));
    // Tracer<false>::DoPass clears the image before every pass (Tracer.h:214-224)
    CTL_HIP(c, hipMemsetAsync(d_fb, 0, sizeof(ctl_pixel) * (size_t)cam.width * cam.height, s));
    unsigned long long* cursor = c->d_cursors + 2;
    CTL_HIP(c, hipMemsetAsync(cursor, 0, sizeof(unsigned long long), s));
    const bool single = c->scene.single != 0, wide = c->scene.wide != 0;
    const uint32_t full = c->scene.full_shading;
    const uint64_t want = (items + kBlock - 1) / kBlock;
#define PRK(SG, WD, FU)                                                                                          \
    do {                                                                                                         \
        const int nb = resident_blocks(c, prim_kernel<SG, WD, FU>, kStackLdsBytes);                              \
        hipLaunchKernelGGL((prim_kernel<SG, WD, FU>), dim3((unsigned)std::min<uint64_t>(nb, want)), dim3(kBlock), \
                           kStackLdsBytes, s, c->scene, P, Q, c->d_s1[c->active], c->d_s2[c->active], items,     \
                           cursor, c->d_counters, d_fb, d_depth);                                                \
    } while (0)
#define PRK2(SG, WD) do { if (full == kShadeEnv) PRK(SG, WD, kShadeEnv); else if (full == kShadeAlpha) PRK(SG, WD, kShadeAlpha); \
                           else if (full) PRK(SG, WD, kShadeFull); else PRK(SG, WD, kShadeLean); } while (0)
    if (wide) { if (single) PRK2(true, 1); else PRK2(false, 1); }
    else { if (single) PRK2(true, 0); else PRK2(false, 0); }
#undef PRK2
#undef PRK
    CTL_HIP(c, hipGetLastError());
    CTL_HIP(c, hipEventRecord(c->pass_ev[1], s));
    c->pass_timed = true;
    return CTL_OK;
}

}  // extern "C"

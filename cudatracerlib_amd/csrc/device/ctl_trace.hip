// ctl_trace.hip — gfx950 kernels and the device half of the C ABI
// (include/ctl_trace.h).
//
//   intersect_kernel   batch closest/any hit over ctl_ray -> ctl_hit
//                      (intersectKernel<ANY_HIT> + __internal__IntersectBuffers,
//                       Kernel/TraceHelper.cu:326-746)
//   path_kernel        one PathTracer pass: sensor ray + PathTrace<true> + AddSample
//                      (pathKernel2 / PathTrace, Integrators/PathTracer.cu:10-113,182-194;
//                       Image::AddSample, Engine/Image.cu:22-44)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/ctl_trace.h"
#include "common.h"

namespace ctl {
void sampler_tables(uint64_t pass, uint32_t nseq, uint32_t len, float* seq1d, float* seq2d);
void sampler_pass_state(uint64_t pass, uint32_t nseq, uint32_t len, uint32_t v[5], uint32_t* d);
void sampler_step_powers(uint32_t* out, int kmax);
}

using namespace ctl;

static_assert(sizeof(ctl_bvh_node) == 64, "BVHNodeData is 64 B");
static_assert(sizeof(ctl_woop_tri) == 48, "TriIntersectorData is 48 B");
static_assert(sizeof(ctl_triangle_data) == 32, "TriangleData is 32 B");
static_assert(sizeof(ctl_kernel_mesh) == 20, "KernelMesh is 20 B");
static_assert(sizeof(ctl_node) == 24, "Node is 24 B");
static_assert(sizeof(ctl_ray) == 32, "traversalRay is 32 B");
static_assert(sizeof(ctl_hit) == 16, "traversalResult is 16 B");
static_assert(sizeof(ctl_pixel) == 28, "PixelData is 28 B");
static_assert(sizeof(ctl_light_tri) == 64, "ShapeSet::triData is 64 B");

namespace {

template <bool STATS>
struct PathCtx {
    const DevScene& S;
    const PathParams& P;
    SamplerDev& rng;
    LaneStack& st;
    uint32_t rays;
    TraceStats ts;
    bool ok;

    __device__ void trace_closest(f3 o, f3 d, HitRec& h) {   // traceRay (TraceHelper.cu:174-180)
        rays++;
        h.t = FLT_MAX; h.tri = 0xffffffffu; h.node = 0xffffffffu; h.u = h.v = 0.0f;
        ok &= trace_ray_dev<false, STATS>(S, o, d, 0.0f, S.ray_eps, h, st, &ts);
    }
    // KernelDynamicScene::Occluded(ray, 0, tmax) (KernelDynamicScene.cu:70-80)
    __device__ bool occluded(f3 o, f3 d, float tmax) {
        if (P.shadow_any_hit) {
            rays++;
            HitRec h;
            h.t = tmax - S.ray_eps; h.tri = 0xffffffffu; h.node = 0xffffffffu; h.u = h.v = 0.0f;
            ok &= trace_ray_dev<true, STATS>(S, o, d, 0.0f, S.ray_eps, h, st, &ts);
            return h.tri != 0xffffffffu;
        }
        HitRec h;
        trace_closest(o, d, h);
        bool end = h.t < tmax - S.ray_eps;
        return h.t > 0 + S.ray_eps && end;
    }

    // EstimateDirect (Kernel/TraceAlgorithms.cu:44-73): flags EAll & ~EDelta, attenuated, MIS
    __device__ spec estimate_direct(bsdf_rec b, const dgeom& dg, const ctl_material& mat, const ctl_light& L,
                                    float light_pdf) {
        direct_rec dRec;
        dRec.p = dg.P; dRec.n = dg.sys.n; dRec.measure = kEArea;
        dRec.ref = dg.P; dRec.refN = dg.sys.n;
        spec value = light_sample_direct(L, S.light_tris, S.light_tri_cdf, dRec, rng.next2());
        spec ret = mk3s(0.0f);
        if (!spec_zero(value)) {
            b.wo = to_local(dg.sys, dRec.d);
            b.type_mask = kEAll & ~kEDelta;
            spec bsdfVal = diffuse_f(mat, b);
            if (!spec_zero(bsdfVal) && !occluded(dRec.ref, dRec.d, dRec.dist)) {
                float weight = 1.0f;
                if (dRec.measure != kEDiscrete) {
                    const float bsdfPdf = diffuse_pdf(mat, b);
                    const float directPdf = dRec.pdf * light_pdf;
                    weight = power_heuristic(directPdf, bsdfPdf);
                }
                ret = value * bsdfVal * weight;
                ret = ret * mk3s(1.0f);
            }
        }
        return ret;
    }

    // UniformSampleOneLight (TraceAlgorithms.cu:92-101) + sampleEmitter (KernelDynamicScene.cu:25-39)
    __device__ spec sample_one_light(const bsdf_rec& b, const dgeom& dg, const ctl_material& mat) {
        if (!S.n_lights) return mk3s(0.0f);
        f2 sample = rng.next2();
        uint32_t n = S.n_lights < CTL_MAX_NUM_LIGHTS ? S.n_lights : CTL_MAX_NUM_LIGHTS;
        uint32_t first = 0, count = n;   // STL_upper_bound
        while (count > 0) {
            uint32_t c2 = count / 2, mid = first + c2;
            if (!(sample.x < S.light_cdf[mid])) { first = mid + 1; count -= c2 + 1; }
            else count = c2;
        }
        uint32_t idx = first;
        if (idx >= n) idx = n - 1;
        float fU = S.light_cdf[idx], fL = idx > 0 ? S.light_cdf[idx - 1] : 0.0f;
        sample.x = (sample.x - fL) / (fU - fL);
        float pdf = fU - fL;
        return spec_div(estimate_direct(b, dg, mat, S.lights[idx], pdf), pdf);
    }

    // PathTrace<true> without media / environment (PathTracer.cu:10-113)
    __device__ spec path_trace(f3 rori, f3 rdir) {
        spec cl = mk3s(0.0f), cf = mk3s(1.0f);
        int depth = 0;
        bool specularBounce = false;
        bsdf_rec b;
        b.wo = mk3(0.0f, 0.0f, 1.0f);
        b.wi = mk3(0.0f, 0.0f, 1.0f);
        b.sampled_type = 0;
        b.type_mask = kEAll;
        float brdf_pdf = 0.0f;
        f3 last_nor = mk3s(0.0f);
        HitRec r2;
        r2.tri = 0xffffffffu;
        while (depth++ < P.max_path_length) {
            trace_closest(rori, rdir, r2);
            if (r2.tri != 0xffffffffu) {
                b.sampled_type = 0;
                b.type_mask = kEAll;
                dgeom dg;
                dg.P = rori + r2.t * rdir;
                const ctl_triangle_data td = S.tri_data[r2.tri];
                const ctl_node N = S.nodes[r2.node];
                fill_dg(td, load_m44(S.xf + 4 * r2.node), mk2(r2.u, r2.v), P.half_quirk, LutDecode{S.normal_lut}, dg);
                b.wi = to_local(dg.sys, -rdir);
                const ctl_material mat = S.mats[((td.w[1] >> 16) & 0xffu) + N.material_offset];
                if (mat.two_sided && b.wi.z < 0) {
                    dg.n = -dg.n;
                    dg.sys.n = -dg.sys.n;
                    b.wi.z *= -1.0f;
                }
                if (mat.node_light_index != 0xffffffffu) {
                    uint32_t li = N.lights[mat.node_light_index];
                    const ctl_light L = S.lights[li];
                    float misWeight = 1.0f;
                    if (!(depth == 1 || specularBounce)) {
                        direct_rec dRec;
                        dRec.ref = rori; dRec.refN = last_nor; dRec.p = dg.P; dRec.n = dg.n;
                        dRec.d = rdir; dRec.dist = r2.t; dRec.measure = kESolidAngle;
                        float direct_pdf = light_pdf_direct(L, dRec) * (S.light_cdf[li] - (li == 0 ? 0.0f : S.light_cdf[li - 1]));
                        misWeight = power_heuristic(brdf_pdf, direct_pdf);
                    }
                    f3 w = -rdir;
                    spec Le = (dot(dg.sys.n, w) <= 0) ? mk3s(0.0f) : mk3(L.radiance[0], L.radiance[1], L.radiance[2]);
                    cl = cl + (cf * misWeight) * Le;
                }
                spec f = diffuse_sample(mat, b, brdf_pdf, rng.next2());
                last_nor = dg.sys.n;
                if ((mat.combined_type & kESmooth) != 0) cl = cl + cf * sample_one_light(b, dg, mat);
                specularBounce = (b.sampled_type & kEDelta) != 0;
                cf = cf * f;
                rori = dg.P;
                rdir = to_world(dg.sys, b.wo);
            }
            if (r2.tri == 0xffffffffu) break;
            if (depth > P.rr_start_depth && !specularBounce) {
                if (rng.next1() >= spec_max(cf)) break;
                cf = spec_div(cf, spec_max(cf));
            }
        }
        if (r2.tri == 0xffffffffu) cl = cl + (cf * 1.0f) * mk3s(0.0f);
        return cl;
    }
};

// SequenceSamplerData tables of one pass generated on the device: sequence q
// starts q*len*3 draws after the pass's first state (host-computed), reached
// with the GF(2) step powers M^(2^k); then curand_uniform * (1 - 1e-5f)
// exactly as Base/CudaRandom.cu:8-17 and the CUDA toolkit's XORWOW.
constexpr int kJumpBits = 24;
struct XorwowDev { uint32_t v[5]; uint32_t d; };

__global__ __launch_bounds__(256) void sampler_kernel(const uint32_t* __restrict__ powers, XorwowDev base,
                                                      uint32_t nseq, uint32_t len, float* s1, float2* s2) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nseq) return;
    const uint32_t off = q * len * 3;
    uint32_t v[5] = {base.v[0], base.v[1], base.v[2], base.v[3], base.v[4]};
    for (int k = 0; k < kJumpBits; k++) {
        if (!((off >> k) & 1u)) continue;
        const uint32_t* M = powers + k * 800;
        uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
        for (int w = 0; w < 5; w++) {
            uint32_t bits = v[w];
            while (bits) {
                int b = __builtin_ctz(bits);
                bits &= bits - 1;
                const uint32_t* c = M + (w * 32 + b) * 5;
                r0 ^= c[0]; r1 ^= c[1]; r2 ^= c[2]; r3 ^= c[3]; r4 ^= c[4];
            }
        }
        v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
    }
    uint32_t d = base.d + 362437u * off;
    auto next = [&]() -> float {
        uint32_t t = v[0] ^ (v[0] >> 2);
        v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
        v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
        d += 362437u;
        const float kInv = 2.3283064e-10f;
        float f = (float)(v[4] + d) * kInv + (kInv / 2.0f);
        return f * (1 - 1e-5f);
    };
    for (uint32_t i = 0; i < len; i++) s1[i * nseq + q] = next();
    for (uint32_t i = 0; i < len; i++) {
        float x = next();
        float y = next();
        s2[i * nseq + q] = make_float2(x, y);
    }
}

template <bool STATS>
__global__ __launch_bounds__(kBlock) void path_kernel(DevScene S, PathParams P, const float* s1, const float2* s2,
                                                      ctl_pixel* fb, unsigned long long* counters) {
    CTL_LANE_STACK(st);
    const uint32_t perTile = P.tile_size * P.tile_size;
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t j = (uint32_t)(g / perTile), w = (uint32_t)(g % perTile);
    const uint32_t tile = j * P.num_ranks + P.rank;
    uint32_t rays = 0;
    TraceStats ts{0, 0, 0};
    bool ok = true;
    if (tile < P.num_tiles) {
        const uint32_t groupsPerRow = P.tile_size / 8;
        const uint32_t grp = w / 64, lane = w % 64;
        const uint32_t px = (tile % P.tiles_x) * P.tile_size + (grp % groupsPerRow) * 8 + lane % 8;
        const uint32_t py = (tile / P.tiles_x) * P.tile_size + (grp / groupsPerRow) * 8 + lane / 8;
        const uint32_t idx = py * P.width + px;   // TracerBase::getPixelIndex (Tracer.h:89-97)
        if (px < P.width && py < P.height) {
            SamplerDev rng{s1, s2, P.nseq, P.len, idx % P.nseq, (idx / P.nseq) % P.nseq, 0, 0};
            PathCtx<STATS> C{S, P, rng, st, 0, TraceStats{0, 0, 0}, true};
            f2 pX = mk2((float)px, (float)py) + rng.next2();
            (void)rng.next2();   // aperture sample (unused by PerspectiveSensor)
            // PerspectiveSensor::sampleRayDifferential (Sensor.cu:130-144)
            m44 s2c = to_m44(S.camera.sample_to_camera), tw = to_m44(S.camera.to_world);
            f3 nearP = xform_point(s2c, mk3(pX.x * S.camera.inv_resolution[0], pX.y * S.camera.inv_resolution[1], 0.0f));
            f3 d = normalize(nearP);
            f3 o = xform_point(tw, mk3s(0.0f));
            f3 dw = xform_dir(tw, d);
            spec col = mk3s(1.0f) * C.path_trace(o, dw);
            // Image::AddSample: single owner per pixel per pass -> plain read-modify-write
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
            rays = C.rays;
            ts = C.ts;
            ok = C.ok;
        }
    }
    wave_add_u64(&counters[0], rays);
    if (!ok) atomicAdd(&counters[1], 1ull);
    if (STATS) {
        wave_add_u64(&counters[2], ts.nodes);
        wave_add_u64(&counters[3], ts.tris);
        wave_add_u64(&counters[4], ts.inst);
    }
}

template <bool ANY, bool STATS>
__global__ __launch_bounds__(kBlock) void intersect_kernel(DevScene S, int64_t n, const ctl_ray* rays, ctl_hit* hits,
                                                           unsigned long long* counters) {
    CTL_LANE_STACK(st);
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    TraceStats ts{0, 0, 0};
    bool ok = true;
    if (i < n) {
        const float4* r4 = reinterpret_cast<const float4*>(rays + i);
        const float4 o = r4[0], d = r4[1];
        HitRec h;
        h.t = d.w; h.tri = 0xffffffffu; h.node = 0xffffffffu; h.u = h.v = 0.0f;
        if (S.n_nodes != 0) ok = trace_ray_dev<ANY, STATS>(S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), o.w, o.w, h, st, &ts);
        uint4 res = make_uint4((uint32_t)__float_as_int(h.t), 0xffffffffu, 0xffffffffu, 0u);
        if (h.tri != 0xffffffffu) {   // TraceHelper.cu:722-731
            res.y = h.node;
            res.z = h.tri;
            uint16_t xd = (uint16_t)(h.u * 65535), yd = (uint16_t)(h.v * 65535);
            res.w = ((uint32_t)yd << 16) | (uint32_t)xd;
        }
        reinterpret_cast<uint4*>(hits)[i] = res;
    }
    if (!ok) atomicAdd(&counters[1], 1ull);
    if (STATS) {
        wave_add_u64(&counters[2], ts.nodes);
        wave_add_u64(&counters[3], ts.tris);
        wave_add_u64(&counters[4], ts.inst);
    }
}

}  // namespace

// ===========================================================================
// Context + C ABI
// ===========================================================================
static std::mutex g_err_mtx;
static std::string g_create_err;

#define CTL_HIP(ctx, call)                                                                 \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                \
            return CTL_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

static void free_scene(ctl_ctx* c) {
    for (void* p : c->scene_allocs) (void)hipFree(p);
    c->scene_allocs.clear();
    c->has_scene = false;
}

template <class T>
static ctl_status upload(ctl_ctx* c, const T* src, size_t count, const T** dst) {
    size_t bytes = count * sizeof(T);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) { c->err = std::string("hipMalloc: ") + hipGetErrorString(e); return CTL_ERR_NOMEM; }
    c->scene_allocs.push_back(p);
    if (bytes) {
        e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) { c->err = std::string("hipMemcpy: ") + hipGetErrorString(e); return CTL_ERR_HIP; }
    }
    *dst = reinterpret_cast<const T*>(p);
    return CTL_OK;
}

extern "C" {

CTL_API int32_t ctl_abi_version(void) { return CTL_ABI_VERSION; }

CTL_API const char* ctl_last_error(const ctl_ctx* ctx) {
    if (ctx) return ctx->err.c_str();
    std::lock_guard<std::mutex> g(g_err_mtx);
    return g_create_err.c_str();
}

CTL_API ctl_ctx* ctl_create(int32_t device) {
    auto fail = [](const std::string& s) -> ctl_ctx* {
        std::lock_guard<std::mutex> g(g_err_mtx);
        g_create_err = s;
        return nullptr;
    };
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail("ctl_create: no HIP device");
    if (device < 0 || device >= n) return fail("ctl_create: device index out of range");
    if (hipSetDevice(device) != hipSuccess) return fail("ctl_create: hipSetDevice failed");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail("ctl_create: hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(std::string("ctl_create: device is ") + prop.gcnArchName + ", kernels are built for gfx950 only");
    ctl_ctx* c = new ctl_ctx();
    c->device = device;
    c->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (hipMalloc(&c->d_counters, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_counters, 0, 8 * sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return fail("ctl_create: counter allocation failed");
    }
    {
        std::vector<uint32_t> pw((size_t)kJumpBits * 800);
        ctl::sampler_step_powers(pw.data(), kJumpBits);
        if (hipMalloc(&c->d_powers, pw.size() * 4) != hipSuccess ||
            hipMemcpy(c->d_powers, pw.data(), pw.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            ctl_destroy(c);
            return fail("ctl_create: sampler power table allocation failed");
        }
    }
    for (int i = 0; i < 2; i++) {
        size_t n1 = (size_t)c->nseq * c->len;
        if (hipMalloc(&c->d_s1[i], n1 * sizeof(float)) != hipSuccess ||
            hipMalloc(&c->d_s2[i], n1 * sizeof(float2)) != hipSuccess ||
            hipHostMalloc(&c->h_s1[i], n1 * sizeof(float)) != hipSuccess ||
            hipHostMalloc(&c->h_s2[i], n1 * 2 * sizeof(float)) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming) != hipSuccess) {
            ctl_destroy(c);
            return fail("ctl_create: sampler buffer allocation failed");
        }
    }
    return c;
}

CTL_API void ctl_destroy(ctl_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    free_scene(c);
    ctl::wavefront_free(c);
    for (int i = 0; i < 2; i++) {
        if (c->d_s1[i]) (void)hipFree(c->d_s1[i]);
        if (c->d_s2[i]) (void)hipFree(c->d_s2[i]);
        if (c->h_s1[i]) (void)hipHostFree(c->h_s1[i]);
        if (c->h_s2[i]) (void)hipHostFree(c->h_s2[i]);
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    }
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->d_powers) (void)hipFree(c->d_powers);
    delete c;
}

CTL_API ctl_status ctl_scene_upload(ctl_ctx* c, const ctl_scene_desc* d) {
    if (!c || !d) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    if (d->env_map_index != 0xffffffffu) { c->err = "scene_upload: environment maps are not supported"; return CTL_ERR_INVALID; }
    if (d->n_lights > CTL_MAX_NUM_LIGHTS) { c->err = "scene_upload: more than 16 lights"; return CTL_ERR_INVALID; }
    for (uint32_t i = 0; i < d->n_lights; i++)
        if (d->lights[i].orthogonal) { c->err = "scene_upload: orthogonal DiffuseLight unsupported"; return CTL_ERR_INVALID; }
    for (uint32_t i = 0; i < d->n_materials; i++)
        if (d->materials[i].bsdf_type != CTL_BSDF_DIFFUSE) { c->err = "scene_upload: only diffuse BSDFs are supported"; return CTL_ERR_INVALID; }
    CTL_HIP(c, hipDeviceSynchronize());
    free_scene(c);
    DevScene S{};
    ctl_status r;
#define UP(src, cnt, dst)                                         \
    if ((r = upload(c, src, cnt, dst)) != CTL_OK) { free_scene(c); return r; }
    const ctl_bvh_node* bvh; UP(d->bvh_nodes, d->n_bvh_nodes, &bvh);
    const ctl_woop_tri* woop; UP(d->woop_tris, d->n_woop_tris, &woop);
    UP(d->tri_indices, d->n_tri_indices, &S.tri_idx);
    UP(d->tri_data, d->n_tri_data, &S.tri_data);
    UP(d->materials, d->n_materials, &S.mats);
    UP(d->meshes, d->n_meshes, &S.meshes);
    UP(d->nodes, d->n_nodes, &S.nodes);
    const ctl_bvh_node* sb; UP(d->scene_bvh_nodes, d->n_scene_bvh_nodes, &sb);
    const ctl_float4x4* xf; UP(d->node_xf, d->n_nodes, &xf);
    const ctl_float4x4* ixf; UP(d->node_inv_xf, d->n_nodes, &ixf);
    UP(d->lights, d->n_lights, &S.lights);
    UP(d->light_tris, d->n_light_tris, &S.light_tris);
    UP(d->light_tri_cdf, d->n_light_tri_cdf, &S.light_tri_cdf);
    // decoded spherical-normal table (Uchar2ToNormalizedFloat3, Compression.h:20-31)
    std::vector<float4> lut(65536);
    for (uint32_t code = 0; code < 65536; code++) {
        f3 v = normal_decode16(code);
        lut[code] = make_float4(v.x, v.y, v.z, 0.0f);
    }
    UP(lut.data(), lut.size(), &S.normal_lut);
#undef UP
    S.bvh = reinterpret_cast<const float4*>(bvh);
    S.woop = reinterpret_cast<const float4*>(woop);
    S.scene_bvh = reinterpret_cast<const float4*>(sb);
    S.xf = reinterpret_cast<const float4*>(xf);
    S.inv_xf = reinterpret_cast<const float4*>(ixf);
    S.n_nodes = d->n_nodes;
    S.start_node = d->scene_start_node;
    S.n_lights = d->n_lights;
    S.flags = d->flags;
    S.ray_eps = d->ray_eps;
    for (int i = 0; i < CTL_MAX_NUM_LIGHTS; i++) S.light_cdf[i] = d->light_cdf[i];
    S.camera = d->camera;
    S.single = 0;
    if (d->n_nodes > 0 && d->scene_start_node < 0) {
        uint32_t node = ~(uint32_t)d->scene_start_node;
        if (node >= d->n_nodes) { free_scene(c); c->err = "scene_upload: start node out of range"; return CTL_ERR_INVALID; }
        const ctl_kernel_mesh& M = d->meshes[d->nodes[node].mesh_index];
        S.single = 1;
        S.s_node_base = M.bvh_node_offset;
        S.s_tri_base = M.bvh_triangle_offset;
        S.s_idx_base = M.bvh_indices_offset;
        S.s_tri_offset = M.triangle_offset;
    }
    c->scene = S;
    c->half_quirk = (d->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0;
    c->has_scene = true;
    return CTL_OK;
}

CTL_API ctl_status ctl_sampler_upload(ctl_ctx* c, const float* seq1d, const float* seq2d, uint32_t nseq, uint32_t len,
                                      void* stream) {
    if (!c || !seq1d || !seq2d) return CTL_ERR_INVALID;
    if (nseq != c->nseq || len != c->len) { c->err = "sampler_upload: tables must be 4096 x 30"; return CTL_ERR_INVALID; }
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int b = c->next_buf;
    size_t n1 = (size_t)nseq * len;
    CTL_HIP(c, hipEventSynchronize(c->ev[b]));
    std::memcpy(c->h_s1[b], seq1d, n1 * sizeof(float));
    std::memcpy(c->h_s2[b], seq2d, n1 * 2 * sizeof(float));
    CTL_HIP(c, hipMemcpyAsync(c->d_s1[b], c->h_s1[b], n1 * sizeof(float), hipMemcpyHostToDevice, s));
    CTL_HIP(c, hipMemcpyAsync(c->d_s2[b], c->h_s2[b], n1 * 2 * sizeof(float), hipMemcpyHostToDevice, s));
    CTL_HIP(c, hipEventRecord(c->ev[b], s));
    c->active = b;
    c->next_buf = 1 - b;
    return CTL_OK;
}

CTL_API ctl_status ctl_sampler_generate(ctl_ctx* c, uint64_t pass_index, void* stream) {
    // Generated on the device (sampler_kernel); stream order makes the buffer
    // reuse safe: the pass that read buffer b two calls ago precedes this launch.
    if (!c) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int b = c->next_buf;
    XorwowDev base;
    ctl::sampler_pass_state(pass_index, c->nseq, c->len, base.v, &base.d);
    hipLaunchKernelGGL(sampler_kernel, dim3((c->nseq + 255) / 256), dim3(256), 0, s, c->d_powers, base, c->nseq,
                       c->len, c->d_s1[b], c->d_s2[b]);
    CTL_HIP(c, hipGetLastError());
    c->active = b;
    c->next_buf = 1 - b;
    return CTL_OK;
}

static ctl_status launch_intersect(ctl_ctx* c, int64_t n, const ctl_ray* rays, ctl_hit* hits, int32_t any_hit,
                                   bool stats, void* stream) {
    if (!c || n < 0 || (n > 0 && (!rays || !hits))) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "intersect: no scene uploaded"; return CTL_ERR_STATE; }
    CTL_HIP(c, hipSetDevice(c->device));
    if (n == 0) return CTL_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    if (stats) {
        if (any_hit) hipLaunchKernelGGL((intersect_kernel<true, true>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, n, rays, hits, c->d_counters);
        else hipLaunchKernelGGL((intersect_kernel<false, true>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, n, rays, hits, c->d_counters);
    } else {
        if (any_hit) hipLaunchKernelGGL((intersect_kernel<true, false>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, n, rays, hits, c->d_counters);
        else hipLaunchKernelGGL((intersect_kernel<false, false>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, n, rays, hits, c->d_counters);
    }
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

static ctl_status add_rays(ctl_ctx* c, uint64_t n, hipStream_t s);

CTL_API ctl_status ctl_intersect(ctl_ctx* c, int64_t n, const ctl_ray* d_rays, ctl_hit* d_hits, int32_t any_hit,
                                 void* stream) {
    ctl_status r = launch_intersect(c, n, d_rays, d_hits, any_hit, false, stream);
    if (r != CTL_OK) return r;
    // the batch call counts N rays (g_RayTracedCounterHost += N, TraceHelper.cu:745)
    return add_rays(c, (uint64_t)n, reinterpret_cast<hipStream_t>(stream));
}

static ctl_status prepare_pass(ctl_ctx* c, const ctl_pt_params* p, ctl_pixel* fb, PathParams& P) {
    if (!c || !p || !fb) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "render_pass: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->active < 0) { c->err = "render_pass: no sampler tables (call ctl_sampler_generate)"; return CTL_ERR_STATE; }
    if (!p->direct) { c->err = "render_pass: only Direct=1 is supported"; return CTL_ERR_INVALID; }
    uint32_t ts = p->tile_size ? p->tile_size : 64;
    if (ts % 8 != 0) { c->err = "render_pass: tile_size must be a multiple of 8"; return CTL_ERR_INVALID; }
    uint32_t nr = p->num_ranks ? p->num_ranks : 1;
    if (p->rank >= nr) { c->err = "render_pass: rank >= num_ranks"; return CTL_ERR_INVALID; }
    const ctl_camera& cam = c->scene.camera;
    P.width = cam.width; P.height = cam.height;
    P.max_path_length = p->max_path_length;
    P.rr_start_depth = p->rr_start_depth;
    P.tile_size = ts;
    P.tiles_x = (cam.width + ts - 1) / ts;
    uint32_t tiles_y = (cam.height + ts - 1) / ts;
    P.num_tiles = P.tiles_x * tiles_y;
    P.num_ranks = nr;
    P.rank = p->rank;
    P.nseq = c->nseq; P.len = c->len;
    P.shadow_any_hit = p->shadow_any_hit;
    P.half_quirk = c->half_quirk;
    return CTL_OK;
}

static ctl_status launch_pass(ctl_ctx* c, const ctl_pt_params* p, ctl_pixel* fb, bool stats, void* stream) {
    PathParams P;
    ctl_status r = prepare_pass(c, p, fb, P);
    if (r != CTL_OK) return r;
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t owned = (P.num_tiles > P.rank) ? (P.num_tiles - P.rank + P.num_ranks - 1) / P.num_ranks : 0;
    uint64_t threads = (uint64_t)owned * P.tile_size * P.tile_size;
    if (threads == 0) return CTL_OK;
    dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
    const float* s1 = c->d_s1[c->active];
    const float2* s2 = c->d_s2[c->active];
    if (!(p->flags & CTL_PT_MEGAKERNEL)) {
        int r2 = ctl::wavefront_pass(c, P, fb, stats, s);
        return r2;
    }
    if (stats) hipLaunchKernelGGL((path_kernel<true>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, P, s1, s2, fb, c->d_counters);
    else hipLaunchKernelGGL((path_kernel<false>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, P, s1, s2, fb, c->d_counters);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

CTL_API ctl_status ctl_render_pass(ctl_ctx* c, const ctl_pt_params* params, ctl_pixel* d_fb, void* stream) {
    return launch_pass(c, params, d_fb, false, stream);
}

__global__ void add_kernel(unsigned long long* ctr, unsigned long long k) { ctr[0] += k; }

static ctl_status add_rays(ctl_ctx* c, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL(add_kernel, dim3(1), dim3(1), 0, s, c->d_counters, (unsigned long long)n);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

CTL_API uint64_t ctl_rays_traced(ctl_ctx* c) {
    if (!c) return 0;
    unsigned long long v[2] = {0, 0};
    if (hipSetDevice(c->device) != hipSuccess) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 0;
    if (hipMemcpy(v, c->d_counters, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    if (v[1]) c->err = "traversal stack overflow on " + std::to_string(v[1]) + " lanes";
    return v[0];
}

CTL_API ctl_status ctl_reset_rays(ctl_ctx* c, void* stream) {
    if (!c) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    CTL_HIP(c, hipMemsetAsync(c->d_counters, 0, 8 * sizeof(unsigned long long), reinterpret_cast<hipStream_t>(stream)));
    return CTL_OK;
}

CTL_API ctl_status ctl_sync(ctl_ctx* c, void* stream) {
    if (!c) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    CTL_HIP(c, hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return CTL_OK;
}

static ctl_status read_stats(ctl_ctx* c, uint64_t out[4], uint64_t rays_before, hipStream_t s) {
    unsigned long long v[5];
    CTL_HIP(c, hipStreamSynchronize(s));
    CTL_HIP(c, hipMemcpy(v, c->d_counters, sizeof(v), hipMemcpyDeviceToHost));
    out[0] = v[0] - rays_before;
    out[1] = v[2]; out[2] = v[3]; out[3] = v[4];
    CTL_HIP(c, hipMemset(c->d_counters + 2, 0, 3 * sizeof(unsigned long long)));
    if (v[1]) { c->err = "traversal stack overflow"; return CTL_ERR_STATE; }
    return CTL_OK;
}

CTL_API ctl_status ctl_intersect_stats(ctl_ctx* c, int64_t n, const ctl_ray* d_rays, ctl_hit* d_hits, int32_t any_hit,
                                       uint64_t out[4], void* stream) {
    if (!c || !out) return CTL_ERR_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned long long before = 0;
    CTL_HIP(c, hipStreamSynchronize(s));
    CTL_HIP(c, hipMemset(c->d_counters + 2, 0, 3 * sizeof(unsigned long long)));
    CTL_HIP(c, hipMemcpy(&before, c->d_counters, sizeof(before), hipMemcpyDeviceToHost));
    ctl_status r = launch_intersect(c, n, d_rays, d_hits, any_hit, true, stream);
    if (r != CTL_OK) return r;
    if ((r = add_rays(c, (uint64_t)n, s)) != CTL_OK) return r;
    return read_stats(c, out, before, s);
}

CTL_API ctl_status ctl_render_pass_stats(ctl_ctx* c, const ctl_pt_params* params, ctl_pixel* d_fb, uint64_t out[4],
                                         void* stream) {
    if (!c || !out) return CTL_ERR_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned long long before = 0;
    CTL_HIP(c, hipStreamSynchronize(s));
    CTL_HIP(c, hipMemset(c->d_counters + 2, 0, 3 * sizeof(unsigned long long)));
    CTL_HIP(c, hipMemcpy(&before, c->d_counters, sizeof(before), hipMemcpyDeviceToHost));
    ctl_status r = launch_pass(c, params, d_fb, true, stream);
    if (r != CTL_OK) return r;
    return read_stats(c, out, before, s);
}

}  // extern "C"

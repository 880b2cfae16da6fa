// wavefront.hip — the PathTracer pass as a wavefront pipeline on gfx950.
//
// Same per-path arithmetic and random-number order as the megakernel restatement
// of PathTrace<true> (Integrators/PathTracer.cu:10-113), reorganised per bounce:
//
//   gen      sensor ray per owned pixel               (pathKernel2, PathTracer.cu:182-194)
//   trace    closest hit over the extension queue     (traceRay, TraceHelper.cu:174-180)
//   shade    emission + MIS, BSDF sample, NEE light sample, Russian roulette;
//            pushes the shadow ray (Occluded, KernelDynamicScene.cu:70-80) and the
//            next extension ray into compacted queues
//   trace    any-hit over the shadow queue
//   resolve  cl += NEE contribution if unoccluded; AddSample of finished paths
//
// The NEE term of bounce k is added to cl after bounce k's emission and before
// bounce k+1's, so every fp32 addition happens in the reference order and the
// framebuffer is bit-identical to the megakernel and to the CPU oracle.
// Why: the traversal kernel stays lean (no shading state -> high occupancy) and
// always runs on compacted, full waves of live rays instead of idling lanes whose
// paths already ended.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"

namespace ctl {
namespace {

constexpr int kMaxBounces = 64;   // count slots per pass (MaxPathLength is clamped to this)

__device__ __forceinline__ uint32_t queue_push(uint32_t* count, bool want) {
    // wave-aggregated append: one atomic per wave
    const uint64_t mask = __ballot(want);
    if (!mask) return 0xffffffffu;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    const uint32_t rank = lanes_below(mask);
    return want ? base + rank : 0xffffffffu;
}

// Samples go to per-work-item slots (store_sample, common.h), folded into the
// framebuffer in image order after the pass.
__device__ __forceinline__ void wf_store(const PathParams& P, const SampleSlots& SS, uint32_t i, f2 pX, spec col) {
    uint32_t px, py;
    work_pixel(P, i, px, py);
    store_sample(P, SS, 0, i, px, py, pX, col);
}

__global__ __launch_bounds__(kBlock) void wf_gen_kernel(DevScene S_arg, PathParams P_arg, const float* s1, const float2* s2,
                                                        WfState W, uint64_t n_items, SampleSlots SS) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;; g += (uint64_t)gridDim.x * kBlock) {
        // keep whole waves in the loop so the ballot in queue_push sees every lane
        const bool inRange = g < n_items;
        if (!__any(inRange)) break;
        uint32_t px = 0, py = 0;
        bool valid = inRange && work_pixel(P, g, px, py);
        f2 pX = mk2(0, 0);
        f3 o = mk3s(0), d = mk3s(0);
        uint32_t idx = py * P.width + px;
        if (valid) {
            SamplerDev rng;
            rng.init(s1, s2, P, idx, 0, 0);
            pX = mk2((float)px, (float)py) + rng.next2();
            (void)rng.next2();   // aperture sample
            sensor_ray(S, pX, o, d);
            valid = apron_keep(P, g, pX);   // an apron path landing outside the tile: no sample (slot stays 0)
        }
        const bool live = valid && P.max_path_length > 0;
        if (valid && !live) wf_store(P, SS, (uint32_t)g, pX, mk3s(0.0f) + (mk3s(1.0f) * 1.0f) * mk3s(0.0f));
        const uint32_t slot = queue_push(&W.counts[0], live);
        if (live) {
            const uint32_t i = (uint32_t)g;
            W.q[0][slot] = i;
            W.o[i] = make_float4(o.x, o.y, o.z, 0.0f);
            W.d[i] = make_float4(d.x, d.y, d.z, 0.0f);
            W.cl[i] = make_float4(0.0f, 0.0f, 0.0f, pX.x);
            W.cf[i] = make_float4(1.0f, 1.0f, 1.0f, pX.y);
            W.wo[i] = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
            W.ln[i] = make_float2(0.0f, 0.0f);
            W.meta[i] = make_uint4(idx, 0u | (2u << 16), 1u, 0u);   // d1=0, d2=2, depth=1 (while(depth++ < max))
        }
    }
}

// Persistent trace over a queue: MODE 0 = extension rays (closest hit),
// 1 = shadow rays any-hit over (eps, dist - eps), 2 = shadow rays as the
// reference's closest-hit Occluded().  Lanes whose ray finished fetch the next
// queue entry between traversal rounds (one atomic per wave), so waves stay
// full while long rays finish (dynamic fetch, cf. intersectKernel's warp
// fetch at TraceHelper.cu:379-399, here per round instead of per batch).
#ifndef CTL_WF_REFILL_MIN
#define CTL_WF_REFILL_MIN 40   // refill once this many lanes of the wave wait (as the batch traversal)
#endif
constexpr int kWfRefillMin = CTL_WF_REFILL_MIN;
template <int MODE, bool STATS, bool SINGLE, int WIDE, bool ALPHA>
__global__ __launch_bounds__(kBlock) void wf_trace_kernel(DevScene S_arg, WfState W, const uint32_t* queue,
                                                          const uint32_t* countp, uint32_t* cursor,
                                                          unsigned long long* counters) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    CTL_LANE_STACK(st);
    const uint32_t count = *countp;
    if (count == 0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&counters[0], (unsigned long long)count);
    TraceStats ts{0, 0, 0};
    Traverser<MODE == 1, STATS, SINGLE, WIDE, ALPHA> T;
    T.done = true;
    bool haveRay = false, exhausted = false, ovf = false;
    uint32_t ray = 0;
    const int lane = threadIdx.x & 63;
    while (true) {
        if (haveRay && T.done) {
            if (MODE == 0) {
                W.hit[ray] = make_float4(T.h.t, T.h.u, T.h.v, __int_as_float((int)T.h.tri));
                W.hit_node[ray] = T.h.node;
            } else if (MODE == 1) {
                W.sh_occ[ray] = T.h.tri != 0xffffffffu ? 1u : 0u;
            } else {
                W.sh_occ[ray] = shadow_occluded(S, false, T.h, W.sh_d[ray].w) ? 1u : 0u;
            }
            ovf |= st.overflow;
            haveRay = false;
        }
        const bool need = !haveRay && !exhausted;
        const uint64_t mask = __ballot(need);
        if (mask && (__popcll(mask) >= kWfRefillMin || !__any(haveRay))) {
            const int leader = __ffsll((unsigned long long)mask) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(cursor, (uint32_t)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t k = base + lanes_below(mask);
                if (k < count) {
                    ray = queue[k];
                    haveRay = true;
                    if (MODE == 0) {
                        const float4 o = W.o[ray], d = W.d[ray];
                        T.init(S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), 0.0f, S.ray_eps, FLT_MAX, st, &ts);
                    } else {
                        const float4 o = W.sh_o[ray], d = W.sh_d[ray];
                        T.init(S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), 0.0f, S.ray_eps,
                               MODE == 1 ? o.w : FLT_MAX, st, &ts, MODE == 1 ? d.w : -1.0f);
                    }
                } else {
                    exhausted = true;
                }
            }
        }
        if (!__any(haveRay)) break;
        if (haveRay && !T.done) T.round(S, st, &ts);
    }
    if (ovf) atomicAdd(&counters[1], 1ull);
    if (STATS) {
        wave_add_u64(&counters[2], ts.nodes);
        wave_add_u64(&counters[3], ts.tris);
        wave_add_u64(&counters[4], ts.inst);
    }
}

template <int MODE>
void launch_trace(ctl_ctx* c, hipStream_t s, const uint32_t* queue, const uint32_t* cnt, uint32_t* cursor, bool stats) {
    WfState& W = c->wf;
    const bool single = c->scene.single != 0;
#define LT(ST, SG, WD, AL)                                                                                      \
    do {                                                                                                        \
        const int blocks = resident_blocks(c, wf_trace_kernel<MODE, ST, SG, WD, AL>, kStackLdsBytes);           \
        hipLaunchKernelGGL((wf_trace_kernel<MODE, ST, SG, WD, AL>), dim3(blocks), dim3(kBlock), kStackLdsBytes, s, \
                           c->scene, W, queue, cnt, cursor, c->d_counters);                                     \
    } while (0)
#define LT2(SG, WD) do { if (alpha) LT(false, SG, WD, true); else LT(false, SG, WD, false); } while (0)
    const bool wide = c->scene.wide != 0 && !stats;   // stats: the reference's binary traversal
    const bool alpha = c->scene.alpha != 0;
    if (stats) { if (single) LT(true, true, 0, false); else LT(true, false, 0, false); }
    else if (wide) { if (single) LT2(true, 1); else LT2(false, 1); }
    else { if (single) LT2(true, 0); else LT2(false, 0); }
#undef LT2
#undef LT
}

template <int FULL>
__global__ __launch_bounds__(kBlock) void wf_shade_kernel(DevScene S_arg, PathParams P_arg, const float* s1, const float2* s2,
                                                          WfState W, int bounce, SampleSlots SS) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    const uint32_t count = W.counts[2 * bounce];
    const uint32_t* qin = W.q[bounce & 1];
    uint32_t* qout = W.q[(bounce + 1) & 1];
    uint32_t* nextCount = &W.counts[2 * (bounce + 1)];
    uint32_t* shCount = &W.counts[2 * bounce + 1];
    const uint32_t stride = gridDim.x * kBlock;
    const uint32_t rounds = (count + stride - 1) / stride;
    for (uint32_t r = 0; r < rounds; r++) {
        const uint32_t k = r * stride + blockIdx.x * kBlock + threadIdx.x;
        const bool act = k < count;
        const uint32_t i = act ? qin[k] : 0u;
        bool pushShadow = false, pushNext = false;
        ShadowReq sh;
        if (act) {
            const float4 o4 = W.o[i], d4 = W.d[i], cl4 = W.cl[i], cf4 = W.cf[i], wo4 = W.wo[i];
            const float2 ln2 = W.ln[i];
            const uint4 meta = W.meta[i];
            const float4 hit = W.hit[i];
            PathVars v;
            v.rori = mk3(o4.x, o4.y, o4.z); v.rdir = mk3(d4.x, d4.y, d4.z);
            v.cl = mk3(cl4.x, cl4.y, cl4.z); v.cf = mk3(cf4.x, cf4.y, cf4.z);
            v.pX = mk2(cl4.w, cf4.w);
            v.brdf_pdf = o4.w;
            v.wo = mk3(wo4.x, wo4.y, wo4.z);
            v.last_nor = mk3(wo4.w, ln2.x, ln2.y);
            v.depth = (int)(meta.z & 0xffffu);
            v.specular = (meta.z >> 16) & 1u;
            v.has_partials = meta.w != 0u;
            if (v.has_partials) {
                const float4 pt = W.part[i];
                v.dudx = pt.x; v.dudy = pt.y; v.dvdx = pt.z; v.dvdy = pt.w;
            }
            SamplerDev rng;
            rng.init(s1, s2, P, meta.x, meta.y & 0xffffu, meta.y >> 16);
            HitRec h;
            h.t = hit.x; h.u = hit.y; h.v = hit.z; h.tri = (uint32_t)__float_as_int(hit.w); h.node = W.hit_node[i];
            if (h.tri != 0xffffffffu) {
                bool terminated = !shade_hit<FULL>(S, P, rng, v, h, sh);
                pushShadow = sh.valid;
                if (!terminated) {
                    // loop head of the next bounce: `while (depth++ < MaxPathLength)`
                    if (v.depth < P.max_path_length) { v.depth++; pushNext = true; }
                    else terminated = true;
                }
                W.o[i] = make_float4(v.rori.x, v.rori.y, v.rori.z, v.brdf_pdf);
                W.d[i] = make_float4(v.rdir.x, v.rdir.y, v.rdir.z, 0.0f);
                W.cf[i] = make_float4(v.cf.x, v.cf.y, v.cf.z, v.pX.y);
                W.wo[i] = make_float4(v.wo.x, v.wo.y, v.wo.z, v.last_nor.x);
                W.ln[i] = make_float2(v.last_nor.y, v.last_nor.z);
                W.meta[i] = make_uint4(meta.x, rng.d1 | (rng.d2 << 16), (uint32_t)v.depth | ((v.specular ? 1u : 0u) << 16),
                                       v.has_partials ? 1u : 0u);
                if (v.has_partials && !meta.w) W.part[i] = make_float4(v.dudx, v.dudy, v.dvdx, v.dvdy);
                if (terminated && !pushShadow) wf_store(P, SS, i, v.pX, mk3s(1.0f) * v.cl);
                if (pushShadow) {
                    W.sh_o[i] = make_float4(v.rori.x, v.rori.y, v.rori.z, sh.dist - S.ray_eps);
                    W.sh_d[i] = make_float4(sh.d.x, sh.d.y, sh.d.z, sh.dist);
                    // w: the path ended here -> resolve adds NEE, then AddSample
                    W.sh_val[i] = make_float4(sh.add.x, sh.add.y, sh.add.z, terminated ? 1.0f : 0.0f);
                }
            } else {
                // miss: loop ends; environment term of PathTracer.cu:98-111
                v.cl = v.cl + env_miss<FULL>(S, P, v);
                wf_store(P, SS, i, v.pX, mk3s(1.0f) * v.cl);
            }
            W.cl[i] = make_float4(v.cl.x, v.cl.y, v.cl.z, v.pX.x);
        }
        const uint32_t ns = queue_push(shCount, pushShadow);
        if (pushShadow) W.sq[ns] = i;
        const uint32_t nn = queue_push(nextCount, pushNext);
        if (pushNext) qout[nn] = i;
    }
}

__global__ __launch_bounds__(kBlock) void wf_resolve_kernel(PathParams P, WfState W, int bounce, SampleSlots SS) {
    const uint32_t count = W.counts[2 * bounce + 1];
    for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < count; k += gridDim.x * kBlock) {
        const uint32_t i = W.sq[k];
        const float4 v = W.sh_val[i];
        float4 cl4 = W.cl[i];
        spec cl = mk3(cl4.x, cl4.y, cl4.z);
        if (!W.sh_occ[i]) cl = cl + mk3(v.x, v.y, v.z);
        W.cl[i] = make_float4(cl.x, cl.y, cl.z, cl4.w);
        if (v.w != 0.0f) wf_store(P, SS, i, mk2(cl4.w, W.cf[i].w), mk3s(1.0f) * cl);
    }
}

template <class T>
bool wf_alloc(ctl_ctx* c, T** p, size_t n) {
    if (hipMalloc((void**)p, n * sizeof(T) + 16) != hipSuccess) return false;
    c->wf_allocs.push_back((void*)*p);
    return true;
}

}  // namespace

void wavefront_free(ctl_ctx* c) {
    for (void* p : c->wf_allocs) (void)hipFree(p);
    c->wf_allocs.clear();
    c->wf = WfState{};
}

int wavefront_pass(ctl_ctx* c, const PathParams& P, const SampleSlots& SS, bool stats, hipStream_t s) {
    const uint64_t items = pass_items_of(P);   // owned pixels + apron items
    if (items == 0) return 0;
    // the 32-bit queue cursors take at most one extra fetch per resident lane after a queue runs
    // dry (at most 2048 lanes per CU): leave that much headroom so a cursor cannot wrap onto live work
    const int persist = c->cu_count * 8;
    if (items > 0xffffffffull - (uint64_t)c->cu_count * 2048u) {
        c->err = "wavefront: too many paths per pass";
        return CTL_ERR_INVALID;
    }
    WfState& W = c->wf;
    if (W.capacity < items) {
        (void)hipStreamSynchronize(s);
        wavefront_free(c);
        size_t n = items;
        bool ok = wf_alloc(c, &W.o, n) && wf_alloc(c, &W.d, n) && wf_alloc(c, &W.cl, n) && wf_alloc(c, &W.cf, n) &&
                  wf_alloc(c, &W.wo, n) && wf_alloc(c, &W.ln, n) && wf_alloc(c, &W.meta, n) && wf_alloc(c, &W.part, n) &&
                  wf_alloc(c, &W.hit, n) && wf_alloc(c, &W.hit_node, n) && wf_alloc(c, &W.q[0], n) &&
                  wf_alloc(c, &W.q[1], n) && wf_alloc(c, &W.sq, n) && wf_alloc(c, &W.sh_o, n) &&
                  wf_alloc(c, &W.sh_d, n) && wf_alloc(c, &W.sh_val, n) && wf_alloc(c, &W.sh_occ, n) &&
                  wf_alloc(c, &W.counts, 4 * (kMaxBounces + 2));
        if (!ok) { wavefront_free(c); c->err = "wavefront: state allocation failed"; return CTL_ERR_NOMEM; }
        W.capacity = items;
    }
    if (hipMemsetAsync(W.counts, 0, 4 * (kMaxBounces + 2) * sizeof(uint32_t), s) != hipSuccess) {
        c->err = "wavefront: memset failed";
        return CTL_ERR_HIP;
    }
    const float* s1 = c->d_s1[c->active];
    const float2* s2 = c->d_s2[c->active];
    const unsigned genBlocks = (unsigned)std::min<uint64_t>((items + kBlock - 1) / kBlock, (uint64_t)persist);
    // a path cut off by kMaxBounces stores nothing: its slot must read "no sample"
    if (hipMemsetAsync(SS.s, 0, items * sizeof(float4), s) != hipSuccess) {
        c->err = "wavefront: memset failed";
        return CTL_ERR_HIP;
    }
    hipLaunchKernelGGL(wf_gen_kernel, dim3(genBlocks), dim3(kBlock), 0, s, c->scene, P, s1, s2, W, items, SS);
    const int maxB = std::min(P.max_path_length, kMaxBounces);
    uint32_t* cursors = W.counts + 2 * (kMaxBounces + 2);
    for (int b = 0; b < maxB; b++) {
        const uint32_t* cnt = &W.counts[2 * b];
        launch_trace<0>(c, s, W.q[b & 1], cnt, &cursors[2 * b], stats);
        if (CTL_NO_TRACE_LEVEL(c->scene.full_shading) == kShadeEnv)
            hipLaunchKernelGGL((wf_shade_kernel<kShadeEnv>), dim3(persist), dim3(kBlock), 0, s, c->scene, P, s1, s2, W, b, SS);
        else if (c->scene.full_shading)
            hipLaunchKernelGGL((wf_shade_kernel<kShadeFull>), dim3(persist), dim3(kBlock), 0, s, c->scene, P, s1, s2, W, b, SS);
        else
            hipLaunchKernelGGL((wf_shade_kernel<kShadeLean>), dim3(persist), dim3(kBlock), 0, s, c->scene, P, s1, s2, W, b, SS);
        const uint32_t* scnt = &W.counts[2 * b + 1];
        if (P.shadow_any_hit) launch_trace<1>(c, s, W.sq, scnt, &cursors[2 * b + 1], stats);
        else launch_trace<2>(c, s, W.sq, scnt, &cursors[2 * b + 1], stats);
        hipLaunchKernelGGL(wf_resolve_kernel, dim3(persist), dim3(kBlock), 0, s, P, W, b, SS);
    }
    if (hipGetLastError() != hipSuccess) { c->err = "wavefront: launch failed"; return CTL_ERR_HIP; }
    return 0;
}

}  // namespace ctl

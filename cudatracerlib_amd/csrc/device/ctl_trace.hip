// ctl_trace.hip — gfx950 kernels and the device half of the C ABI
// (include/ctl_trace.h).
//
//   intersect_kernel   batch closest/any hit over ctl_ray -> ctl_hit
//                      (intersectKernel<ANY_HIT> + __internal__IntersectBuffers,
//                       Kernel/TraceHelper.cu:326-746)
//   path_kernel_persistent  one PathTracer pass (default schedule): resident
//                      grid, path regeneration from an atomic pixel cursor
//   path_kernel        one PathTracer pass, one thread per pixel path
//                      (both: sensor ray + PathTrace<true> + AddSample;
//                       pathKernel2 / PathTrace, Integrators/PathTracer.cu:10-113,182-194;
//                       Image::AddSample, Engine/Image.cu:22-44)
//   sampler_kernel     SequenceSamplerData tables of a pass (Sampler.cu, CudaRandom.cu)
// The wavefront schedule lives in wavefront.hip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/ctl_trace.h"
#include "../host/bvh_wide.h"
#include "../ctl_qnode.h"
#include "common.h"

namespace ctl {
void sampler_tables(uint64_t pass, uint32_t nseq, uint32_t len, float* seq1d, float* seq2d);
void sampler_pass_state(uint64_t pass, uint32_t nseq, uint32_t len, uint32_t v[5], uint32_t* d);
void sampler_step_powers(uint32_t* out, int kmax);
void sampler_seq_powers(uint32_t* out, uint32_t len);
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
static_assert(sizeof(ctl_material) == 80, "ctl_material is 80 B");
static_assert(sizeof(ctl_texture) == 380, "ctl_texture is 380 B");
static_assert(sizeof(ctl_pixel_variance) == 44, "PixelVarianceInfo is 44 B");

#ifndef CTL_PERSIST_WAVES_FULL
#define CTL_PERSIST_WAVES_FULL 4   // ... with the C5 shading (out-of-line texture / microfacet / fp64 math
                                   // calls; path state parked in LDS): C5 3 waves 1480, 4 waves 1658 Mrays/s
#endif
#ifndef CTL_PERSIST_WAVES
#define CTL_PERSIST_WAVES 4   // waves/SIMD for the persistent path kernel, measured on C3 with the packed
                              // wide-node step: 2: 1576, 3: 1590, 4: 1666, 5: 1601, 6: 1505 Mrays/s
#endif

namespace {

// Path state of path_kernel_persistent parked in LDS while the lane's ray is
// traced: everything the shading needs and the traversal does not (throughput,
// radiance, last normal, wo, pixel position, BSDF pdf, depth and specular flag,
// the pending shadow ray's contribution, the sampler's sequence offsets and
// draw counters) -- 23 words per lane in [word][thread] layout (conflict-free
// ds_read/ds_write_b32).  Only the ray (origin, both directions, shadow
// distance) and a few flags stay in VGPRs across the traversal loop, so the
// traversal's register peak no longer stacks on top of the shading state.
// 16 KB stacks + 1 KB work words + 23 KB parked state = 40 KB per 256-thread
// block: 4 blocks per CU, i.e. the 4 waves/SIMD the VGPR budget targets.
// Lean kernel VGPR spills 36 -> 11; C3 2983 -> 3219 Mrays/s (profiles/r03_park_slack_ab.txt).
constexpr int kParkWords = 23;
struct Park {
    int tid;
    __device__ __forceinline__ void put(int w, float x) const {
        ctl_lds_stack[kExtraLdsOff + w * kStackBlock + tid] = __float_as_int(x);
    }
    __device__ __forceinline__ void puti(int w, uint32_t x) const {
        ctl_lds_stack[kExtraLdsOff + w * kStackBlock + tid] = (int)x;
    }
    __device__ __forceinline__ float get(int w) const {
        return __int_as_float(ctl_lds_stack[kExtraLdsOff + w * kStackBlock + tid]);
    }
    __device__ __forceinline__ uint32_t geti(int w) const {
        return (uint32_t)ctl_lds_stack[kExtraLdsOff + w * kStackBlock + tid];
    }
    __device__ __forceinline__ void put3(int w, f3 x) const { put(w, x.x); put(w + 1, x.y); put(w + 2, x.z); }
    __device__ __forceinline__ f3 get3(int w) const { return mk3(get(w), get(w + 1), get(w + 2)); }
    __device__ __forceinline__ void store(const PathVars& v, const ShadowReq& sh, const SamplerDev& rng) const {
        put3(0, v.cl); put3(3, v.cf); put3(6, v.last_nor); put3(9, v.wo);
        put(12, v.pX.x); put(13, v.pX.y); put(14, v.brdf_pdf);
        puti(15, ((uint32_t)v.depth << 1) | (v.specular ? 1u : 0u));
        put3(16, sh.add);
        puti(19, rng.a); puti(20, rng.b); puti(21, rng.d1); puti(22, rng.d2);
    }
    // a new path (refill): everything but the shadow contribution, which only the
    // shadow phase reads and store_shaded always writes first -- so the previous
    // path's value is not carried through the loop just to be written here
    __device__ __forceinline__ void begin(const PathVars& v, const SamplerDev& rng) const {
        put3(0, v.cl); put3(3, v.cf); put3(6, v.last_nor); put3(9, v.wo);
        put(12, v.pX.x); put(13, v.pX.y); put(14, v.brdf_pdf);
        puti(15, ((uint32_t)v.depth << 1) | (v.specular ? 1u : 0u));
        puti(19, rng.a); puti(20, rng.b); puti(21, rng.d1); puti(22, rng.d2);
    }
    __device__ __forceinline__ void load(PathVars& v, ShadowReq& sh, SamplerDev& rng) const {
        v.cl = get3(0); v.cf = get3(3); v.last_nor = get3(6); v.wo = get3(9);
        v.pX.x = get(12); v.pX.y = get(13); v.brdf_pdf = get(14);
        const uint32_t ds = geti(15);
        v.depth = (int)(ds >> 1); v.specular = (ds & 1u) != 0;
        sh.add = get3(16);
        rng.a = geti(19); rng.b = geti(20); rng.d1 = geti(21); rng.d2 = geti(22);
    }
    // Partial loads and stores (the FULL kernels): after a trace the lane loads only
    // depth / specular and the sampler state; shade_hit reads the rest where it
    // is used (common.h shade_hit, `pk`), and only what changed goes back.
    __device__ __forceinline__ void load_core(PathVars& v, SamplerDev& rng) const {
        const uint32_t ds = geti(15);
        v.depth = (int)(ds >> 1); v.specular = (ds & 1u) != 0;
        rng.a = geti(19); rng.b = geti(20); rng.d1 = geti(21); rng.d2 = geti(22);
    }
    __device__ __forceinline__ void load_px(PathVars& v) const { v.pX.x = get(12); v.pX.y = get(13); }
    __device__ __forceinline__ void load_mis(PathVars& v) const { v.brdf_pdf = get(14); v.last_nor = get3(6); }
    __device__ __forceinline__ void load_sample_state(PathVars& v) const { v.wo = get3(9); v.brdf_pdf = get(14); }
    __device__ __forceinline__ void load_cl_cf(PathVars& v) const { v.cl = get3(0); v.cf = get3(3); }
    __device__ __forceinline__ void store_cl(const PathVars& v) const { put3(0, v.cl); }
    __device__ __forceinline__ void store_depth(const PathVars& v) const {
        puti(15, ((uint32_t)v.depth << 1) | (v.specular ? 1u : 0u));
    }
    // after shade_hit: everything it can change (not the pixel position)
    __device__ __forceinline__ void store_shaded(const PathVars& v, const ShadowReq& sh, const SamplerDev& rng) const {
        put3(0, v.cl); put3(3, v.cf); put3(6, v.last_nor); put3(9, v.wo);
        put(14, v.brdf_pdf);
        store_depth(v);
        put3(16, sh.add);
        puti(21, rng.d1); puti(22, rng.d2);
    }
};

// dynamic LDS of path_kernel_persistent: lane stacks + the work item word per
// lane + the parked path state
constexpr size_t persistent_lds_bytes() {
    return kStackLdsBytes + sizeof(int) * kStackBlock * (1 + kParkWords);
}

// Megakernel schedule: PathTrace<true> (PathTracer.cu:10-113) with the
// traversals inline in the bounce, as the reference's pathKernel2 runs it.
template <bool STATS, bool SINGLE, int WIDE, int FULL>
struct PathCtx {
    const DevScene& S;
    const PathParams& P;
    SamplerDev& rng;
    LaneStack& st;
    uint32_t rays;
    TraceStats ts;
    bool ok;
    PathVars v;

    // one iteration of `while (depth++ < MaxPathLength)`; false = path done
    __device__ __forceinline__ bool bounce() {
        if (!(v.depth++ < P.max_path_length)) return false;
        HitRec r2;   // traceRay (TraceHelper.cu:174-180)
        r2.t = FLT_MAX; r2.tri = 0xffffffffu; r2.node = 0xffffffffu; r2.u = r2.v = 0.0f;
        rays++;
        ok &= trace_one<0, STATS, SINGLE, WIDE, CTL_ALPHA_OF(FULL)>(S, v.rori, v.rdir, 0.0f, S.ray_eps, r2, st, &ts);
        if (r2.tri == 0xffffffffu) {
            v.cl = v.cl + env_miss<FULL>(S, P, v);   // PathTracer.cu:98-111
            return false;
        }
        ShadowReq sh;
        const bool cont = shade_hit<FULL, SINGLE>(S, P, rng, v, r2, sh);
        if (sh.valid) {
            const bool any = P.shadow_any_hit != 0;
            HitRec h;
            h.t = any ? sh.dist - S.ray_eps : FLT_MAX; h.tri = 0xffffffffu; h.node = 0xffffffffu; h.u = h.v = 0.0f;
            rays++;
            if (any) ok &= trace_one<1, STATS, SINGLE, WIDE, CTL_ALPHA_OF(FULL)>(S, v.rori, sh.d, 0.0f, S.ray_eps, h, st, &ts,
                                                                                sh.dist);
            else ok &= trace_one<0, STATS, SINGLE, WIDE, CTL_ALPHA_OF(FULL)>(S, v.rori, sh.d, 0.0f, S.ray_eps, h, st, &ts);
            if (!shadow_occluded(S, any, h, sh.dist)) v.cl = v.cl + sh.add;
        }
        return cont;
    }
};

// SequenceSamplerData tables of one pass generated on the device: sequence q
// starts q*len*3 draws after the pass's first state (host-computed), reached
// with the GF(2) step powers M^(2^k); then curand_uniform * (1 - 1e-5f)
// exactly as Base/CudaRandom.cu:8-17 and the CUDA toolkit's XORWOW.
constexpr int kJumpBits = 24;
struct XorwowDev { uint32_t v[5]; uint32_t d; };

// One wave per sequence: the GF(2) matrix-vector product of each jump is
// split over the lanes by input bit (lane j holds state bits j, j+64, j+128)
// and XOR-reduced across the wave, so a jump costs one round of column loads
// and a 6-step butterfly instead of ~80 dependent column loads on one lane.
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x ^= (uint32_t)__shfl_xor((int)x, m);
    return x;
}

// powers: [kJumpBits] M^(2^k), then (sampler_seq_powers) [64] A^ql and
// [64] A^(64 qh) with A = M^(3 len), then M^len and M^(len + 2 (len / 2)), all 800 words.
// Sequence q < 4096 jumps in two rounds (A^ql, A^(64 qh)); a larger q by the
// binary powers of its offset.  The rounds are dependent memory round trips,
// so two instead of the ~10 set bits of q * 3 len is what the kernel's time is
// made of (30.6 -> 18.4 us per pass).  Then three lanes draw a third of the
// sequence each, from the states len and len + 2 (len / 2) steps on (one more round each,
// independent of each other): lane 0 the 1-D values, lanes 1 and 2 the first
// and second half of the 2-D pairs.
constexpr int kSeqPowBase = kJumpBits * 800;
// v <- M v over the wave (lane j holds input bits j, j + 64, j + 128)
__device__ __forceinline__ void wave_apply(const uint32_t* __restrict__ M, uint32_t v[5], int lane) {
    const bool lo = lane < 32;
    const uint32_t sh = (uint32_t)(lane & 31);
    const uint32_t w0 = lo ? v[0] : v[1], w1 = lo ? v[2] : v[3];
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
    auto col = [&](uint32_t word, int b) {
        if ((word >> sh) & 1u) {
            const uint32_t* c = M + b * 5;
            r0 ^= c[0]; r1 ^= c[1]; r2 ^= c[2]; r3 ^= c[3]; r4 ^= c[4];
        }
    };
    col(w0, lane);
    col(w1, lane + 64);
    if (lo) col(v[4], lane + 128);
    v[0] = wave_xor(r0); v[1] = wave_xor(r1); v[2] = wave_xor(r2); v[3] = wave_xor(r3); v[4] = wave_xor(r4);
}

__device__ __forceinline__ void sampler_sequence(const uint32_t* __restrict__ powers, const XorwowDev& base,
                                                 uint32_t nseq, uint32_t len, float* s1, float2* s2) {
    const uint32_t q = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (q >= nseq) return;   // whole wave
    const uint32_t off = q * len * 3;
    uint32_t v[5] = {base.v[0], base.v[1], base.v[2], base.v[3], base.v[4]};
    const bool twoStep = q < 4096u;
    for (int k = 0; k < (twoStep ? 2 : kJumpBits); k++) {
        const uint32_t* M;
        if (twoStep) {
            const uint32_t digit = k == 0 ? (q & 63u) : (q >> 6);
            if (!digit) continue;   // identity; uniform over the wave
            M = powers + kSeqPowBase + (k * 64 + digit) * 800;
        } else {
            if (!((off >> k) & 1u)) continue;   // uniform over the wave
            M = powers + k * 800;
        }
        wave_apply(M, v, lane);
    }
    // the states len and len + 2 (len / 2) draws on, for lanes 1 and 2
    uint32_t va[5] = {v[0], v[1], v[2], v[3], v[4]}, vb[5] = {v[0], v[1], v[2], v[3], v[4]};
    wave_apply(powers + kSeqPowBase + 128 * 800, va, lane);
    wave_apply(powers + kSeqPowBase + 129 * 800, vb, lane);
    if (lane > 2) return;
    uint32_t start = 0;
    if (lane == 1) { for (int w = 0; w < 5; w++) v[w] = va[w]; start = len; }
    if (lane == 2) { for (int w = 0; w < 5; w++) v[w] = vb[w]; start = len + 2 * (len / 2); }
    uint32_t d = base.d + 362437u * (off + start);
    auto next = [&]() -> float {
        uint32_t t = v[0] ^ (v[0] >> 2);
        v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
        v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
        d += 362437u;
        const float kInv = 2.3283064e-10f;
        float f = (float)(v[4] + d) * kInv + (kInv / 2.0f);
        return f * (1 - 1e-5f);
    };
    if (lane == 0) {
        for (uint32_t i = 0; i < len; i++) s1[i * nseq + q] = next();
    } else {
        // lane 1: pairs 0 .. len/2 - 1 (draws len .. len + 2 (len / 2) - 1); lane 2: the rest
        const uint32_t i0 = lane == 1 ? 0u : len / 2, i1 = lane == 1 ? len / 2 : len;
        for (uint32_t i = i0; i < i1; i++) {
            float x = next();
            float y = next();
            s2[i * nseq + q] = make_float2(x, y);
        }
    }
}

__global__ __launch_bounds__(256) void sampler_kernel(const uint32_t* __restrict__ powers, XorwowDev base,
                                                      uint32_t nseq, uint32_t len, float* s1, float2* s2) {
    sampler_sequence(powers, base, nseq, len, s1, s2);
}

// The tables of up to kSamplerBatch passes in one launch (ctl_render_passes):
// blockIdx.y = pass slot, whose first state is B.b[slot] and whose tables
// start slot * tbl elements in.  One launch keeps the GPU busier than a chain
// of single-pass launches of 4096 waves each (latency-bound jump rounds).
constexpr uint32_t kSamplerBatch = 128;
struct SamplerBases { XorwowDev b[kSamplerBatch]; };
static_assert(sizeof(SamplerBases) <= 3584, "sampler bases must fit the 4 KB kernel-argument segment");
__global__ __launch_bounds__(256) void sampler_batch_kernel(const uint32_t* __restrict__ powers, SamplerBases B,
                                                            uint32_t nseq, uint32_t len, float* s1, float2* s2,
                                                            uint64_t tbl) {
    const uint32_t slot = blockIdx.y;
    sampler_sequence(powers, B.b[slot], nseq, len, s1 + slot * tbl, s2 + slot * tbl);
}

// One path per thread (the reference's pathKernel2 launch shape).
template <bool STATS, bool SINGLE, int WIDE, int FULL>
__global__ __launch_bounds__(kBlock) void path_kernel(DevScene S_arg, PathParams P_arg, const float* s1, const float2* s2,
                                                      ctl_pixel* fb, unsigned long long* counters, SampleSlots PS) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    CTL_LANE_STACK(st);
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t rays = 0;
    TraceStats ts{0, 0, 0};
    bool ok = true;
    uint32_t px, py;
    if (work_pixel(P, g, px, py)) {
        const uint32_t idx = py * P.width + px;   // TracerBase::getPixelIndex (Tracer.h:89-97)
        SamplerDev rng{s1, s2, P.nseq, P.len, idx % P.nseq, (idx / P.nseq) % P.nseq, 0, 0};
        PathCtx<STATS, SINGLE, WIDE, FULL> C{S, P, rng, st, 0, TraceStats{0, 0, 0}, true, PathVars{}};
        f3 o, dw;
        const f2 pX = primary_ray(S, rng, px, py, o, dw);
        if (apron_keep(P, g, pX)) {
            C.v.begin(pX, o, dw);
            while (C.bounce()) {}
            store_sample(P, PS, 0, (uint32_t)g, px, py, pX, mk3s(1.0f) * C.v.cl);
        } else {
            PS.s[g] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // apron path landing outside the tile
        }
        rays = C.rays;
        ts = C.ts;
        ok = C.ok;
    } else if (g < PS.per_pass) {
        PS.s[g] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // work item outside the image: no sample
    }
    wave_add_u64(&counters[0], rays);
    if (!ok) atomicAdd(&counters[1], 1ull);
    if (STATS) {
        wave_add_u64(&counters[2], ts.nodes);
        wave_add_u64(&counters[3], ts.tris);
        wave_add_u64(&counters[4], ts.inst);
    }
}

// Persistent path kernel with path regeneration (default schedule).  A
// resident grid of lanes, each owning one path at a time:
//  * every iteration a lane traces its pending ray to completion (extension
//    ray, or the NEE shadow ray of its last bounce) with one traversal call
//    site in the kernel, then shades / resolves it; the shadow ray is traced
//    right after the bounce that made it, so radiance sums happen in the
//    reference's order;
//  * a lane whose path ended stores its sample and takes the next work item
//    from a wave-aggregated 64-bit atomic cursor, so waves stay full through
//    the Russian-roulette tail instead of idling until their longest path
//    ends;
//  * the traverser is local to an iteration: only the path variables and the
//    pending ray are loop-carried, keeping the register peak low.
// Work items are independent (own sampler index, own sample slot), so the
// framebuffer is bit-identical to path_kernel's.
template <bool STATS, bool SINGLE, int WIDE, int FULL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SINGLE ? (FULL ? CTL_PERSIST_WAVES_FULL : CTL_PERSIST_WAVES) : 2))) void path_kernel_persistent(DevScene S_arg, PathParams P_arg, const float* s1,
                                                                 const float2* s2, uint64_t items,
                                                                 unsigned long long* cursor, unsigned long long* counters,
                                                                 SampleSlots PS, uint32_t tbl) {
    // Work item k renders pass slot k / PS.per_pass (sampler tables at
    // s1/s2 + slot * tbl) of work item k % PS.per_pass; every finished sample
    // goes to its own slot, folded into the framebuffer afterwards (store_sample).
    // The scene and pass records are read in place from the kernel-argument
    // segment (scalar loads at their uses) rather than held in SGPRs for the
    // kernel's lifetime: 100+ live SGPRs spilled into VGPR lanes and from
    // there to scratch.  C3 3184 -> 3310, C5 1662 -> 1772 Mrays/s; VGPR spills
    // lean 10 -> 0, full 98 -> 40 (profiles/r03_park_slack_ab.txt).
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    CTL_LANE_STACK(st);
    SamplerDev rng{s1, s2, P.nseq, P.len, 0, 0, 0, 0};
    // work item of the lane's path (pass slot * PS.per_pass + item), parked in
    // LDS for the path's lifetime instead of holding a VGPR through the traces
    int* pkw = ctl_lds_stack + kPathWordOff + threadIdx.x;
    const Park park{(int)threadIdx.x};
    auto split = [&](uint32_t k, uint32_t& ps, uint32_t& kk) { PS.split(k, ps, kk); };
    PathVars v;
    ShadowReq sh;
    sh.valid = false;
    sh.dist = 0.0f;
    TraceStats ts{0, 0, 0};
    uint32_t rays = 0;
    bool active = false, exhausted = false, shadowPhase = false, ending = false, ok = true;
#ifdef CTL_PROFILE_TRACE
    long long prof_trace = 0;
    const long long prof_start = wall_clock64();
#endif
    const bool shadowAny = P.shadow_any_hit != 0;
    const int lane = threadIdx.x & 63;
    while (true) {
        const bool need = !active && !exhausted;
        const uint64_t mask = __ballot(need);
        if (mask) {
            const int leader = __ffsll((unsigned long long)mask) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(cursor, (unsigned long long)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint64_t k64 = base + (uint64_t)lanes_below(mask);
                if (k64 >= items) {
                    exhausted = true;
                } else {
                    const uint32_t k = (uint32_t)k64;   // items < 2^32 (checked on the host)
                    uint32_t px, py, ps, kk;
                    split(k, ps, kk);
                    // FULL: the pass record read through an opaque pointer here, so the
                    // divisions by its fields keep their reciprocals local to the refill
                    // (hoisted, they held VGPRs the FULL kernel spilled for its lifetime;
                    // the lean kernel has the registers and keeps them hoisted)
                    const PathParams& Pw = FULL ? *opaque_ptr(&P) : P;
                    if (work_pixel(Pw, kk, px, py)) {
                        const uint32_t idx = py * Pw.width + px;
                        // the pass slot's tables start ps * tbl elements in: folded into
                        // the two sequence offsets so the table bases stay kernel-uniform
                        rng.a = idx % Pw.nseq + ps * tbl; rng.b = (idx / Pw.nseq) % Pw.nseq + ps * tbl;
                        rng.d1 = 0; rng.d2 = 0;
                        *pkw = (int)k;
                        f3 o, dw;
                        const f2 pX = primary_ray(S, rng, px, py, o, dw);
                        v.begin(pX, o, dw);
                        shadowPhase = false;
                        ending = false;
                        // loop head of PathTrace: `while (depth++ < MaxPathLength)`
                        if (!apron_keep(Pw, kk, pX)) PS.s[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        else if (v.depth++ < P.max_path_length) active = true;
                        else store_sample(P, PS, ps, kk, px, py, v.pX, mk3s(1.0f) * v.cl);
                        if (active) park.begin(v, rng);
                    } else {
                        PS.s[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // work item outside the image: no sample
                    }
                }
            }
        }
        if (!__any(active)) {
            if (__all(exhausted)) break;
            continue;
        }
        if (active) {
            HitRec h;
            h.t = (shadowPhase && shadowAny) ? sh.dist - S.ray_eps : FLT_MAX;
            h.u = h.v = 0.0f; h.tri = 0xffffffffu; h.node = 0xffffffffu;
            rays++;
#ifdef CTL_PROFILE_TRACE
            const long long pc0 = wall_clock64();
#endif
            if (S.n_nodes != 0) {
                Traverser<2, STATS, SINGLE, WIDE, CTL_ALPHA_OF(FULL)> T;
                T.anyhit = shadowPhase && shadowAny;
                T.init(S, v.rori, shadowPhase ? sh.d : v.rdir, 0.0f, S.ray_eps, h.t, st, &ts,
                       T.anyhit ? sh.dist : -1.0f);
                while (!T.done) T.round(S, st, &ts);
                h = T.h;
                ok &= !st.overflow;
            }
#ifdef CTL_PROFILE_TRACE
            prof_trace += wall_clock64() - pc0;
#endif
            // the FULL kernels read parked state where the shading uses it (Park's
            // partial loads), the lean kernel all of it after the trace
            constexpr bool lazy = FULL != kShadeLean;
            if (lazy) park.load_core(v, rng);
            else park.load(v, sh, rng);
            bool cont;
            if (shadowPhase) {
                if (lazy) { v.cl = park.get3(0); sh.add = park.get3(16); }
                if (!shadow_occluded(S, shadowAny, h, sh.dist)) v.cl = v.cl + sh.add;
                shadowPhase = false;
                cont = !ending && v.depth++ < P.max_path_length;
                if (lazy && cont) { park.store_cl(v); park.store_depth(v); }
            } else if (h.tri == 0xffffffffu) {
                if (lazy) park.load(v, sh, rng);
                v.cl = v.cl + env_miss<FULL>(S, P, v);   // PathTracer.cu:98-111
                cont = false;
            } else {
                // the FULL kernel keeps the path's first-hit texture partials in its own
                // sample slot (written only when the path ends), not in four VGPRs
                // carried through every trace
                float4* part = PS.s + *pkw;
                ending = lazy ? !shade_hit<FULL, SINGLE, Park>(S, P, rng, v, h, sh, part, &park)
                              : !shade_hit<FULL, SINGLE>(S, P, rng, v, h, sh, part);
                shadowPhase = sh.valid;
                cont = sh.valid || (!ending && v.depth++ < P.max_path_length);
                if (lazy && cont) park.store_shaded(v, sh, rng);
            }
            if (!cont) {
                uint32_t px, py, ps, kk;
                split((uint32_t)*pkw, ps, kk);
                const PathParams& Pw = FULL ? *opaque_ptr(&P) : P;   // as at the refill
                work_pixel(Pw, kk, px, py);
                if (lazy) park.load_px(v);
                store_sample(Pw, PS, ps, kk, px, py, v.pX, mk3s(1.0f) * v.cl);
                active = false;
            } else if (!lazy) {
                park.store(v, sh, rng);
            }
        }
    }
    wave_add_u64(&counters[0], rays);
    if (!ok) atomicAdd(&counters[1], 1ull);
    if (STATS) {
        wave_add_u64(&counters[2], ts.nodes);
        wave_add_u64(&counters[3], ts.tris);
        wave_add_u64(&counters[4], ts.inst);
    }
#ifdef CTL_PROFILE_TRACE
    // wall-clock ticks (100 MHz) per wave: in the trace call site / in the kernel
    if (lane == 0) {
        atomicAdd(&counters[5], (unsigned long long)prof_trace);
        atomicAdd(&counters[6], (unsigned long long)(wall_clock64() - prof_start));
    }
    wave_add_u64(&counters[8], ts.inner_lanes);
    wave_add_u64(&counters[9], ts.inner_waves);
    wave_add_u64(&counters[10], ts.leaf_lanes);
    wave_add_u64(&counters[11], ts.leaf_waves);
    wave_add_u64(&counters[12], ts.inner_r);
    wave_add_u64(&counters[13], ts.rounds);
    wave_add_u64(&counters[14], ts.leafphase_in);
#endif
}

// Batch closest/any hit (intersectKernel<ANY_HIT>, TraceHelper.cu:326-734):
// ray tmin bounds both the node spans and the triangle test (:650).  Resident
// grid; lanes whose ray finished take the next ray from a wave-aggregated
// atomic cursor between traversal rounds (the reference fetches per warp per
// batch of 32 rays, :379-399), so waves stay full on incoherent rays.
template <int ANY, bool STATS, bool SINGLE, int WIDE>
// Two segments (rays, hits)[0, n) then (rays2, hits2)[0, n2) in one launch: the
// wavefront tracer's payload and secondary batches share one resident grid and
// one tail.  ANY: 0 closest hit, 1 any hit (intersectKernel<true>, culled at the
// ray's tmax), 2 closest hit for the first segment and, for the second, the
// shadow query (any hit below tmax, boxes culled at tmax + slab_slack: the
// WavefrontPathTracer's CTL_WPT_SHADOW_ANY_HIT).
#ifndef CTL_REFILL_MIN
#define CTL_REFILL_MIN 40   // batch traversal: refill once at least this many lanes of the wave wait for a ray
                           // (C3 WPT sweep 1/8/24/32/40/48/56: 1093/1222/1505/1563/1564/1569/1545 Mrays/s)
#endif
__global__ __launch_bounds__(kBlock) void intersect_kernel(DevScene S_arg, int64_t n, const ctl_ray* rays, ctl_hit* hits,
                                                           int64_t n2, const ctl_ray* rays2, ctl_hit* hits2,
                                                           unsigned long long* cursor, unsigned long long* counters,
                                                           const uint32_t* dcount, uint32_t band_w) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    // dcount: the two segment sizes read from device memory (the WavefrontPathTracer's
    // queue counts, written by the previous bounce's scan: no host round trip); the
    // batch is then counted here as traced rays
    if (dcount) {
        n = dcount[0];
        n2 = dcount[1];
        if (blockIdx.x == 0 && threadIdx.x == 0 && n + n2 > 0) atomicAdd(&counters[0], (unsigned long long)(n + n2));
    }
    const int64_t total = n + n2;
    CTL_LANE_STACK(st);
    TraceStats ts{0, 0, 0};
    Traverser<ANY, STATS, SINGLE, WIDE> T;
    T.done = true;
    bool haveRay = false, exhausted = false, ovf = false, seg2 = false;
    int64_t ray = 0;   // slot in its segment
    const int lane = threadIdx.x & 63;
    while (true) {
        if (haveRay && T.done) {
            uint4 res = make_uint4((uint32_t)__float_as_int(T.h.t), 0xffffffffu, 0xffffffffu, 0u);
            if (T.h.tri != 0xffffffffu) {   // TraceHelper.cu:722-731
                res.y = T.h.node;
                res.z = T.h.tri;
                uint16_t xd = (uint16_t)(T.h.u * 65535), yd = (uint16_t)(T.h.v * 65535);
                res.w = ((uint32_t)yd << 16) | (uint32_t)xd;
            }
            reinterpret_cast<uint4*>(seg2 ? hits2 + ray : hits + ray)[0] = res;
            ovf |= st.overflow;
            haveRay = false;
        }
        const bool need = !haveRay && !exhausted;
        const uint64_t mask = __ballot(need);
        if (mask && (__popcll(mask) >= CTL_REFILL_MIN || !__any(haveRay))) {
            const int leader = __ffsll((unsigned long long)mask) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(cursor, (unsigned long long)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                int64_t k = (int64_t)base + (int64_t)lanes_below(mask);
                if (k < total) {
                    // band_w: the first segment is a row-major image of that width (the
                    // WavefrontPathTracer's camera rays); trace it in 8-row bands, column by
                    // column, so a wave's 64 rays form an 8 x 8 block (hits go to their own
                    // slots, so the results are those of row order)
                    if (band_w && k < n) {
                        const int64_t bw = 8 * (int64_t)band_w, band = k / bw, h = n / band_w;
                        const int64_t bh = h - 8 * band < 8 ? h - 8 * band : 8, r = k - band * bw;
                        k = (8 * band + r % bh) * band_w + r / bh;
                    }
                    seg2 = k >= n;
                    ray = seg2 ? k - n : k;
                    haveRay = true;
                    const float4* r4 = reinterpret_cast<const float4*>(seg2 ? rays2 + ray : rays + ray);
                    const float4 o = r4[0], d = r4[1];
                    if (ANY == 2) T.anyhit = seg2;
                    T.init(S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), o.w, o.w, d.w, st, &ts,
                           ANY == 2 && seg2 ? d.w : -1.0f);
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

// Primary rays of one pass in work order (the path kernels' first ray: pixel
// jitter + aperture draw + PerspectiveSensor, Sensor.cu:130-144), as a
// traversalRay batch: tmin = scene eps, tmax = FLT_MAX.  Work items outside
// the image get an empty interval (tmax = 0).
__global__ __launch_bounds__(kBlock) void camera_ray_kernel(DevScene S_arg, PathParams P_arg, const float* s1, const float2* s2,
                                                            uint64_t items, ctl_ray* rays) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    const PathParams& P = kernarg_ref<PathParams>(P_arg, kernarg_next<DevScene, PathParams>(0));
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= items) return;
    uint32_t px, py;
    float4 o4 = make_float4(0.0f, 0.0f, 0.0f, S.ray_eps), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
    if (work_pixel(P, g, px, py)) {
        const uint32_t idx = py * P.width + px;
        SamplerDev rng{s1, s2, P.nseq, P.len, idx % P.nseq, (idx / P.nseq) % P.nseq, 0, 0};
        f3 o, d;
        (void)primary_ray(S, rng, px, py, o, d);
        o4 = make_float4(o.x, o.y, o.z, S.ray_eps);
        d4 = make_float4(d.x, d.y, d.z, FLT_MAX);
    }
    float4* r4 = reinterpret_cast<float4*>(rays + g);
    r4[0] = o4;
    r4[1] = d4;
}

// Batch KernelDynamicScene::Occluded(Ray(o, d), 0, tmax) (KernelDynamicScene.cu:70-80),
// tmax = the ray's d.w (o.w ignored), with the path kernels' semantics: the
// reference's closest-hit form (ANYQ false) or the any-hit query of
// shadow_any_hit = 1 (boxes culled at tmax + slab_slack, traverse.h).  traceRay flavour: span tmin
// 0, triangles t > eps, the alpha test when the scene has alpha maps.  One ray
// per lane: a checker and a drop-in for callers of Occluded, not a hot path.
template <bool ANYQ, bool SINGLE, int WIDE>
__global__ __launch_bounds__(kBlock) void occluded_kernel(DevScene S_arg, int64_t n, const ctl_ray* rays, uint32_t* out,
                                                          unsigned long long* counters) {
    const DevScene& S = kernarg_ref<DevScene>(S_arg, 0);   // read in place (common.h kernarg_ref)
    CTL_LANE_STACK(st);
    TraceStats ts{0, 0, 0};
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= n) return;
    const float4* r4 = reinterpret_cast<const float4*>(rays + g);
    const float4 o = r4[0], d = r4[1];
    const float dist = d.w;
    HitRec h;
    h.t = ANYQ ? dist - S.ray_eps : FLT_MAX;
    h.u = h.v = 0.0f; h.tri = 0xffffffffu; h.node = 0xffffffffu;
    bool ok = true;
    if (S.n_nodes != 0)
        ok = trace_one<ANYQ ? 1 : 0, false, SINGLE, WIDE, true>(S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), 0.0f,
                                                               S.ray_eps, h, st, &ts, ANYQ ? dist : -1.0f);
    out[g] = shadow_occluded(S, ANYQ, h, dist) ? 1u : 0u;
    if (!ok) atomicAdd(&counters[1], 1ull);
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
    if (hipMalloc(&c->d_counters, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_counters, 0, 16 * sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return fail("ctl_create: counter allocation failed");
    }
    if (hipMalloc(&c->d_cursors, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_cursors, 0, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&c->h_overflow, sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreate(&c->pass_ev[0]) != hipSuccess || hipEventCreate(&c->pass_ev[1]) != hipSuccess) {
        ctl_destroy(c);
        return fail("ctl_create: cursor/event allocation failed");
    }
    {
        std::vector<uint32_t> pw((size_t)kJumpBits * 800 + 130 * 800);
        ctl::sampler_step_powers(pw.data(), kJumpBits);
        ctl::sampler_seq_powers(pw.data() + kSeqPowBase, c->len);
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
    ctl::wpt_free(c);
    ctl::anim_free(c);
    if (c->d_mt1) (void)hipFree(c->d_mt1);
    if (c->d_mt2) (void)hipFree(c->d_mt2);
    if (c->d_slices) (void)hipFree(c->d_slices);
    for (int i = 0; i < 2; i++) {
        if (c->d_s1[i]) (void)hipFree(c->d_s1[i]);
        if (c->d_s2[i]) (void)hipFree(c->d_s2[i]);
        if (c->h_s1[i]) (void)hipHostFree(c->h_s1[i]);
        if (c->h_s2[i]) (void)hipHostFree(c->h_s2[i]);
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    }
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->d_cursors) (void)hipFree(c->d_cursors);
    if (c->h_overflow) (void)hipHostFree(c->h_overflow);
    if (c->d_tile_flags) (void)hipFree(c->d_tile_flags);
    for (int i = 0; i < 2; i++)
        if (c->pass_ev[i]) (void)hipEventDestroy(c->pass_ev[i]);
    if (c->d_powers) (void)hipFree(c->d_powers);
    delete c;
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
    c->tables_pass = -1;   // caller's tables: no pass index to render ahead from
    c->scene_epoch++;
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
    hipLaunchKernelGGL(sampler_kernel, dim3((c->nseq + 3) / 4), dim3(256), 0, s, c->d_powers, base, c->nseq,
                       c->len, c->d_s1[b], c->d_s2[b]);
    CTL_HIP(c, hipGetLastError());
    c->active = b;
    c->next_buf = 1 - b;
    c->tables_pass = (int64_t)std::min<uint64_t>(pass_index, (uint64_t)INT64_MAX - 16);
    return CTL_OK;
}

// dcount != NULL: n and n2 are upper bounds (grid sizing); the kernel reads the
// segment sizes from dcount[0..1] on the device.
static ctl_status launch_intersect(ctl_ctx* c, int64_t n, const ctl_ray* rays, ctl_hit* hits, int32_t any_hit,
                                   bool stats, void* stream, int64_t n2 = 0, const ctl_ray* rays2 = nullptr,
                                   ctl_hit* hits2 = nullptr, const uint32_t* dcount = nullptr, uint32_t band_w = 0) {
    if (!c || n < 0 || (n > 0 && (!rays || !hits)) || n2 < 0 || (n2 > 0 && (!rays2 || !hits2))) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "intersect: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->overflow_seen) return CTL_ERR_STATE;   // c->err names the overflow (ctl_sync)
    if (n + n2 > 0xffffffffll) { c->err = "intersect: more than 2^32-1 rays per call"; return CTL_ERR_INVALID; }
    CTL_HIP(c, hipSetDevice(c->device));
    if (n + n2 == 0) return CTL_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned long long* cursor = c->d_cursors;
    CTL_HIP(c, hipMemsetAsync(cursor, 0, sizeof(unsigned long long), s));
    const bool single = c->scene.single != 0;
    const uint64_t want = ((uint64_t)(n + n2) + kBlock - 1) / kBlock;
#ifndef CTL_INTERSECT_BPC
#define CTL_INTERSECT_BPC 3   // resident blocks per CU of the batch traversal (0: occupancy limit)
#endif
#define IK(AN, ST, SG, WD)                                                                                       \
    do {                                                                                                         \
        int nb = resident_blocks(c, intersect_kernel<AN, ST, SG, WD>, kStackLdsBytes);                           \
        if (CTL_INTERSECT_BPC > 0) nb = std::min(nb, CTL_INTERSECT_BPC * c->cu_count);                          \
        hipLaunchKernelGGL((intersect_kernel<AN, ST, SG, WD>), dim3((unsigned)std::min<uint64_t>(nb, want)),     \
                           dim3(kBlock), kStackLdsBytes, s, c->scene, n, rays, hits, n2, rays2, hits2, cursor,  \
                           c->d_counters, dcount, band_w);                                                       \
    } while (0)
    // stats launches count the reference's binary traversal (the roofline's algorithmic bytes)
    const bool wide = c->scene.wide != 0 && !stats;
#define IK2(AN, ST)                                                       \
    do {                                                                  \
        if (ST) { if (single) IK(AN, true, true, 0); else IK(AN, true, false, 0); } \
        else if (wide) { if (single) IK(AN, false, true, 1); else IK(AN, false, false, 1); } \
        else { if (single) IK(AN, false, true, 0); else IK(AN, false, false, 0); } \
    } while (0)
    if (stats) { if (any_hit) IK2(1, true); else IK2(0, true); }
    else if (any_hit == 2) IK2(2, false);   // internal: the WavefrontPathTracer's shadow query segment
    else { if (any_hit) IK2(1, false); else IK2(0, false); }
#undef IK2
#undef IK
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

static ctl_status add_rays(ctl_ctx* c, uint64_t n, hipStream_t s);

CTL_API ctl_status ctl_intersect(ctl_ctx* c, int64_t n, const ctl_ray* d_rays, ctl_hit* d_hits, int32_t any_hit,
                                 void* stream) {
    ctl_status r = launch_intersect(c, n, d_rays, d_hits, any_hit ? 1 : 0, false, stream);
    if (r != CTL_OK) return r;
    // the batch call counts N rays (g_RayTracedCounterHost += N, TraceHelper.cu:745)
    return add_rays(c, (uint64_t)n, reinterpret_cast<hipStream_t>(stream));
}

CTL_API ctl_status ctl_occluded(ctl_ctx* c, int64_t n, const ctl_ray* d_rays, uint32_t* d_out, int32_t any_hit,
                                void* stream) {
    if (!c || n < 0 || (n > 0 && (!d_rays || !d_out))) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "occluded: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->overflow_seen) return CTL_ERR_STATE;   // c->err names the overflow (ctl_sync)
    CTL_HIP(c, hipSetDevice(c->device));
    if (n == 0) return CTL_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    if (grid.x == 0 || (uint64_t)(n + kBlock - 1) / kBlock > 0x7fffffffull) {
        c->err = "occluded: batch too large for one launch";
        return CTL_ERR_INVALID;
    }
    const bool single = c->scene.single != 0, wide = c->scene.wide != 0;
#define OK_(AQ, SG, WD) hipLaunchKernelGGL((occluded_kernel<AQ, SG, WD>), grid, dim3(kBlock), kStackLdsBytes, s, \
                                           c->scene, n, d_rays, d_out, c->d_counters)
#define OK2(AQ) do { if (wide) { if (single) OK_(AQ, true, 1); else OK_(AQ, false, 1); } \
                     else { if (single) OK_(AQ, true, 0); else OK_(AQ, false, 0); } } while (0)
    if (any_hit) OK2(true); else OK2(false);
#undef OK2
#undef OK_
    CTL_HIP(c, hipGetLastError());
    return add_rays(c, (uint64_t)n, s);   // each Occluded is one traceRay (TraceHelper.cu:176)
}

static ctl_status prepare_pass(ctl_ctx* c, const ctl_pt_params* p, ctl_pixel* fb, PathParams& P,
                               bool need_tables = true) {
    if (!c || !p || !fb) return CTL_ERR_INVALID;
    if (!c->has_scene) { c->err = "render_pass: no scene uploaded"; return CTL_ERR_STATE; }
    if (c->overflow_seen) return CTL_ERR_STATE;   // c->err names the overflow (ctl_sync)
    if (need_tables && c->active < 0) {
        c->err = "render_pass: no sampler tables (call ctl_sampler_generate)";
        return CTL_ERR_STATE;
    }
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
    P.direct = p->direct != 0;
    P.half_quirk = c->half_quirk;
    P.owned_items = 0;
    P.apron = nr > 1 ? 2 * ts + 1 : 0;
    const uint64_t own = (uint64_t)owned_tiles_of(P) * ts * ts;
    if (own + (uint64_t)owned_tiles_of(P) * P.apron >= 0xffffffffull) {
        c->err = "render_pass: 2^32-1 or more work items per pass";
        return CTL_ERR_INVALID;
    }
    P.owned_items = (uint32_t)own;
    return CTL_OK;
}

static ctl_status launch_schedule(ctl_ctx* c, const ctl_pt_params* p, const PathParams& P, ctl_pixel* fb, bool stats,
                                  hipStream_t s, uint64_t threads, dim3 grid, const float* s1, const float2* s2,
                                  SampleSlots PS = make_slots(nullptr, 0), uint32_t tbl = 0);

static ctl_status prepare_slots(ctl_ctx* c, uint64_t items, hipStream_t s);
static void launch_fold(ctl_ctx* c, const PathParams& P, uint32_t per_pass, uint32_t n, ctl_pixel* fb, hipStream_t s,
                        uint32_t first_slice);

static ctl_status launch_pass(ctl_ctx* c, const ctl_pt_params* p, ctl_pixel* fb, bool stats, void* stream) {
    PathParams P;
    ctl_status r = prepare_pass(c, p, fb, P);
    if (r != CTL_OK) return r;
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t threads = pass_items_of(P);   // owned pixels + apron items
    if (threads == 0) return CTL_OK;
    dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
    const float* s1 = c->d_s1[c->active];
    const float2* s2 = c->d_s2[c->active];
    CTL_HIP(c, hipEventRecord(c->pass_ev[0], s));
    ctl_status r1 = prepare_slots(c, threads, s);   // every schedule stores samples per work item
    if (r1 != CTL_OK) return r1;
    ctl_status r2 = launch_schedule(c, p, P, fb, stats, s, threads, grid, s1, s2,
                                    make_slots(c->d_slices, (uint32_t)threads), 0);
    if (r2 != CTL_OK) return r2;
    launch_fold(c, P, (uint32_t)threads, 1, fb, s, 0);
    CTL_HIP(c, hipEventRecord(c->pass_ev[1], s));
    c->pass_timed = true;
    return CTL_OK;
}

static ctl_status launch_schedule(ctl_ctx* c, const ctl_pt_params* p, const PathParams& P, ctl_pixel* fb, bool stats,
                                  hipStream_t s, uint64_t threads, dim3 grid, const float* s1, const float2* s2,
                                  SampleSlots PS, uint32_t tbl) {
    if (p->flags & CTL_PT_WAVEFRONT) return (ctl_status)ctl::wavefront_pass(c, P, PS, stats, s);
    const bool single = c->scene.single != 0;
    // stats launches count the reference's binary traversal (the roofline's algorithmic bytes)
    const bool wide = c->scene.wide != 0 && !stats;
    const uint32_t full = c->scene.full_shading;
    if (!(p->flags & CTL_PT_MEGAKERNEL)) {
        unsigned long long* cursor = c->d_cursors + 1;
        CTL_HIP(c, hipMemsetAsync(cursor, 0, sizeof(unsigned long long), s));
        const uint64_t want = (threads + kBlock - 1) / kBlock;
#ifndef CTL_PERSIST_BPC
#define CTL_PERSIST_BPC 0   // resident blocks per CU of the persistent path kernel (0: occupancy limit)
#endif
#define PK(ST, SG, WD, FU)                                                                                       \
        do {                                                                                                     \
            constexpr size_t lds = persistent_lds_bytes();                                                      \
            int nb = resident_blocks(c, path_kernel_persistent<ST, SG, WD, FU>, lds);                            \
            if (CTL_PERSIST_BPC > 0) nb = std::min(nb, CTL_PERSIST_BPC * c->cu_count);                          \
            hipLaunchKernelGGL((path_kernel_persistent<ST, SG, WD, FU>), dim3((unsigned)std::min<uint64_t>(nb, want)), \
                               dim3(kBlock), lds, s, c->scene, P, s1, s2, threads, cursor,                       \
                               c->d_counters, PS, tbl);                                                          \
        } while (0)
#define PK2(ST, SG, WD) do { if (full == kShadeEnv) PK(ST, SG, WD, kShadeEnv); else if (full == kShadeAlpha) PK(ST, SG, WD, kShadeAlpha); \
                              else if (full) PK(ST, SG, WD, kShadeFull); else PK(ST, SG, WD, kShadeLean); } while (0)
        if (stats) { if (single) PK2(true, true, 0); else PK2(true, false, 0); }
        else if (wide) { if (single) PK2(false, true, 1); else PK2(false, false, 1); }
        else { if (single) PK2(false, true, 0); else PK2(false, false, 0); }
#undef PK2
#undef PK
    } else {
#define MK(ST, SG, WD, FU) hipLaunchKernelGGL((path_kernel<ST, SG, WD, FU>), grid, dim3(kBlock), kStackLdsBytes, s, c->scene, \
                                              P, s1, s2, fb, c->d_counters, PS)
#define MK2(ST, SG, WD) do { if (full == kShadeEnv) MK(ST, SG, WD, kShadeEnv); else if (full == kShadeAlpha) MK(ST, SG, WD, kShadeAlpha); \
                              else if (full) MK(ST, SG, WD, kShadeFull); else MK(ST, SG, WD, kShadeLean); } while (0)
        if (stats) { if (single) MK2(true, true, 0); else MK2(true, false, 0); }
        else if (wide) { if (single) MK2(false, true, 1); else MK2(false, false, 1); }
        else { if (single) MK2(false, true, 0); else MK2(false, false, 0); }
#undef MK2
#undef MK
    }
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

// Sample slots -> framebuffer: per target pixel, the samples that landed on it
// (its own and the ones that rounded over from the left / upper / upper-left
// neighbour) in image order of their pixels, pass by pass -- one sequential
// AddSample per pixel in image order (Image.cu:22-44), as the oracle adds them.
// Only this rank's pixels are targets; a source of another rank is read from
// the target tile's apron item (source_item), so each pixel is summed by one
// rank in the 1-GPU order and the N-rank reduce is exact.
__global__ __launch_bounds__(kBlock) void fold_samples_kernel(PathParams P, const float4* __restrict__ slots,
                                                              uint32_t per_pass, uint32_t n, ctl_pixel* fb) {
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= (uint64_t)P.width * P.height) return;
    const uint32_t x = (uint32_t)(q % P.width), y = (uint32_t)(q / P.width);
    const uint32_t ts = P.tile_size;
    if (((y / ts) * P.tiles_x + x / ts) % P.num_ranks != P.rank) return;   // the owner sums it (apron items)
    const uint32_t x0 = x - x % ts, y0 = y - y % ts;
    uint32_t ks[4];
    float codes[4];
    int nc = 0;
    // sources in image order: (x-1, y-1), (x, y-1), (x-1, y), (x, y)
#pragma unroll
    for (int d = 3; d >= 0; d--) {
        const uint32_t dx = d & 1, dy = d >> 1;
        uint32_t k;
        if (x >= dx && y >= dy && source_item(P, x - dx, y - dy, x0, y0, k)) {
            ks[nc] = k;
            codes[nc] = (float)(1 + d);
            nc++;
        }
    }
    if (nc == 0) return;
    ctl_pixel* pp = fb + q;
    float r = 0.0f, g = 0.0f, b = 0.0f, w = 0.0f;
    bool any = false;
    for (uint32_t k = 0; k < n; k++) {
        for (int i = 0; i < nc; i++) {
            const float4 v = slots[(size_t)k * per_pass + ks[i]];
            if (v.w == codes[i]) {
                if (!any) { r = pp->rgb[0]; g = pp->rgb[1]; b = pp->rgb[2]; w = pp->weight_sum; any = true; }
                r += v.x; g += v.y; b += v.z; w += 1.0f;
            }
        }
    }
    if (any) {
        pp->rgb[0] = r; pp->rgb[1] = g; pp->rgb[2] = b;
        pp->weight_sum = w;
    }
}

// Sample slots for n passes of per_pass work items, grown on demand.  Every
// work item writes its slot (code 0 when it has no pixel or AddSample would
// drop the sample), so no clearing is needed.
static ctl_status prepare_slots(ctl_ctx* c, uint64_t items, hipStream_t s) {
    c->spec.pending = false;   // the slots are about to be overwritten
    if (c->slices_cap < items) {
        CTL_HIP(c, hipStreamSynchronize(s));
        if (c->d_slices) (void)hipFree(c->d_slices);
        c->d_slices = nullptr; c->slices_cap = 0;
        if (hipMalloc(&c->d_slices, items * sizeof(float4)) != hipSuccess) {
            c->err = "render_pass: sample slot allocation failed";
            return CTL_ERR_NOMEM;
        }
        c->slices_cap = items;
    }
    return CTL_OK;
}

static void launch_fold(ctl_ctx* c, const PathParams& P, uint32_t per_pass, uint32_t n, ctl_pixel* fb, hipStream_t s,
                        uint32_t first_slice = 0) {
    const uint64_t px = (uint64_t)P.width * P.height;
    hipLaunchKernelGGL(fold_samples_kernel, dim3((unsigned)((px + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, P,
                       c->d_slices + (size_t)first_slice * per_pass, per_pass, n, fb);
}

// n_passes consecutive passes in one persistent launch; the first n_fold of them
// are folded into d_fb, the rest stay in the sample slots (a speculative window).
static ctl_status launch_window(ctl_ctx* c, const ctl_pt_params* params, uint64_t first_pass, uint32_t n_passes,
                                uint32_t n_fold, ctl_pixel* d_fb, hipStream_t s, uint64_t* per_pass_out);

CTL_API ctl_status ctl_render_passes(ctl_ctx* c, const ctl_pt_params* params, uint64_t first_pass, uint32_t n_passes,
                                     ctl_pixel* d_fb, void* stream) {
    if (!c || !params || !d_fb) return CTL_ERR_INVALID;
    if (n_passes == 0) return CTL_OK;
    c->spec.last_valid = false;
    return launch_window(c, params, first_pass, n_passes, n_passes, d_fb, reinterpret_cast<hipStream_t>(stream), nullptr);
}

static ctl_status launch_window(ctl_ctx* c, const ctl_pt_params* params, uint64_t first_pass, uint32_t n_passes,
                                uint32_t n_fold, ctl_pixel* d_fb, hipStream_t s, uint64_t* per_pass_out) {
    void* stream = reinterpret_cast<void*>(s);
    if (params->flags & (CTL_PT_WAVEFRONT | CTL_PT_MEGAKERNEL)) {
        // the other schedules: one pass at a time
        for (uint32_t i = 0; i < n_passes; i++) {
            ctl_status r = ctl_sampler_generate(c, first_pass + i, stream);
            if (r == CTL_OK) r = launch_pass(c, params, d_fb, false, stream);
            if (r != CTL_OK) return r;
        }
        return CTL_OK;
    }
    PathParams P;
    ctl_status r = prepare_pass(c, params, d_fb, P, false);
    if (r != CTL_OK) return r;
    CTL_HIP(c, hipSetDevice(c->device));
    const uint64_t per_pass = pass_items_of(P);   // owned pixels + apron items
    if (per_pass_out) *per_pass_out = per_pass;
    if (per_pass == 0) return CTL_OK;
    const uint64_t items = per_pass * n_passes;
    if (items >= 0xffffffffull) { c->err = "render_passes: 2^32-1 or more work items"; return CTL_ERR_INVALID; }
    const size_t tbl = (size_t)c->nseq * c->len;
    if (c->mt_cap < n_passes) {
        CTL_HIP(c, hipStreamSynchronize(s));
        if (c->d_mt1) (void)hipFree(c->d_mt1);
        if (c->d_mt2) (void)hipFree(c->d_mt2);
        c->d_mt1 = nullptr; c->d_mt2 = nullptr; c->mt_cap = 0;
        if (hipMalloc(&c->d_mt1, tbl * n_passes * sizeof(float)) != hipSuccess ||
            hipMalloc(&c->d_mt2, tbl * n_passes * sizeof(float2)) != hipSuccess) {
            c->err = "render_passes: sampler table allocation failed";
            return CTL_ERR_NOMEM;
        }
        c->mt_cap = n_passes;
    }
    CTL_HIP(c, hipEventRecord(c->pass_ev[0], s));
    for (uint32_t i0 = 0; i0 < n_passes; i0 += kSamplerBatch) {
        const uint32_t nb = std::min(kSamplerBatch, n_passes - i0);
        SamplerBases B;
        for (uint32_t i = 0; i < nb; i++)
            ctl::sampler_pass_state(first_pass + i0 + i, c->nseq, c->len, B.b[i].v, &B.b[i].d);
        hipLaunchKernelGGL(sampler_batch_kernel, dim3((c->nseq + 3) / 4, nb), dim3(256), 0, s, c->d_powers, B, c->nseq,
                           c->len, c->d_mt1 + i0 * tbl, c->d_mt2 + i0 * tbl, (uint64_t)tbl);
    }
    r = prepare_slots(c, items, s);
    if (r != CTL_OK) return r;
    r = launch_schedule(c, params, P, d_fb, false, s, items, dim3(1), c->d_mt1, c->d_mt2,
                        make_slots(c->d_slices, (uint32_t)per_pass), (uint32_t)tbl);
    if (r != CTL_OK) return r;
    launch_fold(c, P, (uint32_t)per_pass, n_fold, d_fb, s, 0);
    CTL_HIP(c, hipGetLastError());
    CTL_HIP(c, hipEventRecord(c->pass_ev[1], s));
    c->pass_timed = true;
    return CTL_OK;
}

// Tracer::DoPass through the C ABI with CTL_PT_RENDER_AHEAD (see ctl_ctx::Spec):
// a call whose pass was rendered ahead by an earlier call of the same window
// only folds its samples; a call that continues a steady loop renders a window
// of 2, 4, then 8 passes and folds the first.  Bit-exact to one launch per pass (the fold adds pass by
// pass in the same order); ctl_rays_traced counts a window's rays when it is
// launched, ctl_last_pass_ms times the call's own device work.
static ctl_status render_pass_speculative(ctl_ctx* c, const ctl_pt_params* params, ctl_pixel* d_fb, void* stream) {
    if (!c || !params || !d_fb) return CTL_ERR_INVALID;
    ctl_ctx::Spec& W = c->spec;
    const bool same_state = W.last_valid && std::memcmp(&W.params, params, sizeof(ctl_pt_params)) == 0 && W.fb == d_fb &&
                            W.stream == stream && W.epoch == c->scene_epoch && c->tables_pass >= 0;
    const bool next_pass = same_state && c->tables_pass == W.last_pass + 1;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (W.pending && next_pass && c->tables_pass == W.next && !c->overflow_seen) {
        // rendered ahead: fold its slice
        PathParams P;
        ctl_status r = prepare_pass(c, params, d_fb, P);
        if (r != CTL_OK) return r;
        CTL_HIP(c, hipSetDevice(c->device));
        CTL_HIP(c, hipEventRecord(c->pass_ev[0], s));
        launch_fold(c, P, (uint32_t)W.per_pass, 1, d_fb, s, (uint32_t)(W.next - W.first));
        CTL_HIP(c, hipGetLastError());
        CTL_HIP(c, hipEventRecord(c->pass_ev[1], s));
        c->pass_timed = true;
        W.last_pass = W.next++;
        if (W.next == W.end) { W.pending = false; W.streak++; }
        return CTL_OK;
    }
    if (W.pending) W.streak = 0;   // the loop left the window: its passes are dropped
    W.pending = false;
    const bool speculate = next_pass && (params->flags & CTL_PT_RENDER_AHEAD) &&
                           !(params->flags & (CTL_PT_WAVEFRONT | CTL_PT_MEGAKERNEL));
    if (!speculate) W.streak = 0;
    const uint32_t n = speculate ? (W.streak >= 2 ? 8u : W.streak == 1 ? 4u : 2u) : 1u;
    ctl_status r;
    uint64_t per_pass = 0;
    if (n == 1) {
        r = launch_pass(c, params, d_fb, false, stream);
    } else {
        PathParams P;
        r = prepare_pass(c, params, d_fb, P);   // the tables of this pass are there; refusals as launch_pass's
        if (r == CTL_OK) r = launch_window(c, params, (uint64_t)c->tables_pass, n, 1, d_fb, s, &per_pass);
    }
    if (r != CTL_OK) { W.last_valid = false; return r; }
    W.last_valid = c->tables_pass >= 0;
    W.last_pass = c->tables_pass;
    W.params = *params;
    W.fb = d_fb;
    W.stream = stream;
    W.epoch = c->scene_epoch;
    if (n > 1 && per_pass > 0) {
        W.pending = true;
        W.per_pass = per_pass;
        W.first = c->tables_pass;
        W.next = c->tables_pass + 1;
        W.end = c->tables_pass + n;
    }
    return CTL_OK;
}

CTL_API ctl_status ctl_render_pass(ctl_ctx* c, const ctl_pt_params* params, ctl_pixel* d_fb, void* stream) {
#ifdef CTL_PROFILE_TRACE
    ctl_status r = launch_pass(c, params, d_fb, false, stream);
    unsigned long long v[10];
    if (hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) == hipSuccess &&
        hipMemcpy(v, c->d_counters + 5, sizeof(v), hipMemcpyDeviceToHost) == hipSuccess) {
        fprintf(stderr, "[profile] trace/total wave time %.4f (%llu / %llu); inner loop: %llu wave iterations, "
                        "%.1f lanes each; leaf entries: %llu wave iterations, %.1f lanes each\n",
                (double)v[0] / (double)v[1], v[0], v[1], v[4], (double)v[3] / (double)v[4], v[6],
                (double)v[5] / (double)v[6]);
        fprintf(stderr, "[profile] lanes in the round per inner iteration %.1f; rounds %llu, lanes holding a leaf at the "
                        "leaf phase %.1f\n", (double)v[7] / (double)v[4], v[8], (double)v[9] / (double)v[8]);
        (void)hipMemset(c->d_counters + 5, 0, sizeof(v));
    }
    return r;
#else
    return render_pass_speculative(c, params, d_fb, stream);
#endif
}

CTL_API ctl_status ctl_last_pass_ms(ctl_ctx* c, float* ms) {
    if (!c || !ms) return CTL_ERR_INVALID;
    if (!c->pass_timed) { c->err = "last_pass_ms: no render pass yet"; return CTL_ERR_STATE; }
    CTL_HIP(c, hipSetDevice(c->device));
    CTL_HIP(c, hipEventSynchronize(c->pass_ev[1]));
    CTL_HIP(c, hipEventElapsedTime(ms, c->pass_ev[0], c->pass_ev[1]));
    return CTL_OK;
}

CTL_API ctl_status ctl_camera_rays(ctl_ctx* c, const ctl_pt_params* params, ctl_ray* d_rays, int64_t capacity,
                                   int64_t* n_out, void* stream) {
    if (!c || !params || !n_out) return CTL_ERR_INVALID;
    PathParams P;
    ctl_pixel dummy;
    ctl_status r = prepare_pass(c, params, &dummy, P);
    if (r != CTL_OK) return r;
    const uint64_t items = P.owned_items;   // this rank's pixels
    *n_out = (int64_t)items;
    if (items == 0 || !d_rays) return CTL_OK;   // d_rays == NULL: size query
    if (capacity < (int64_t)items) { c->err = "camera_rays: ray buffer too small"; return CTL_ERR_INVALID; }
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(camera_ray_kernel, dim3((unsigned)((items + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, c->scene,
                       P, c->d_s1[c->active], c->d_s2[c->active], items, d_rays);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

__global__ void add_kernel(unsigned long long* ctr, unsigned long long k) { ctr[0] += k; }

static ctl_status add_rays(ctl_ctx* c, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL(add_kernel, dim3(1), dim3(1), 0, s, c->d_counters, (unsigned long long)n);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

}  // extern "C"

namespace ctl {
int intersect_launch(ctl_ctx* c, int64_t n, const ctl_ray* rays, ctl_hit* hits, int32_t any_hit, hipStream_t s,
                     int64_t n2, const ctl_ray* rays2, ctl_hit* hits2, const uint32_t* dcount, uint32_t band_w) {
    return launch_intersect(c, n, rays, hits, any_hit, false, s, n2, rays2, hits2, dcount, band_w);
}
int count_rays(ctl_ctx* c, uint64_t n, hipStream_t s) { return add_rays(c, n, s); }
}  // namespace ctl

extern "C" {

static void note_overflow(ctl_ctx* c, unsigned long long lanes) {
    if (!lanes) return;
    c->overflow_seen = true;
    c->err = "traversal stack overflow on " + std::to_string(lanes) + " lanes (results invalid; ctl_reset_rays clears)";
}

CTL_API uint64_t ctl_rays_traced(ctl_ctx* c) {
    if (!c) return 0;
    unsigned long long v[2] = {0, 0};
    if (hipSetDevice(c->device) != hipSuccess) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 0;
    if (hipMemcpy(v, c->d_counters, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    note_overflow(c, v[1]);
    return v[0];
}

CTL_API int32_t ctl_scene_stack_bound(const ctl_ctx* c) { return c && c->has_scene ? c->stack_bound : 0; }

CTL_API ctl_status ctl_reset_rays(ctl_ctx* c, void* stream) {
    if (!c) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    CTL_HIP(c, hipMemsetAsync(c->d_counters, 0, 8 * sizeof(unsigned long long), reinterpret_cast<hipStream_t>(stream)));
    c->overflow_seen = false;
    return CTL_OK;
}

// The sync point of the C ABI: waits for the stream, then reports a traversal
// stack overflow of any earlier launch as CTL_ERR_STATE (sticky until
// ctl_reset_rays; every later render / intersect call refuses to run).
CTL_API ctl_status ctl_sync(ctl_ctx* c, void* stream) {
    if (!c) return CTL_ERR_INVALID;
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    CTL_HIP(c, hipMemcpyAsync(c->h_overflow, c->d_counters + 1, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    CTL_HIP(c, hipStreamSynchronize(s));
    note_overflow(c, *c->h_overflow);
    return c->overflow_seen ? CTL_ERR_STATE : CTL_OK;
}

static ctl_status read_stats(ctl_ctx* c, uint64_t out[4], uint64_t rays_before, hipStream_t s) {
    unsigned long long v[5];
    CTL_HIP(c, hipStreamSynchronize(s));
    CTL_HIP(c, hipMemcpy(v, c->d_counters, sizeof(v), hipMemcpyDeviceToHost));
    out[0] = v[0] - rays_before;
    out[1] = v[2]; out[2] = v[3]; out[3] = v[4];
    CTL_HIP(c, hipMemset(c->d_counters + 2, 0, 3 * sizeof(unsigned long long)));
    note_overflow(c, v[1]);
    if (c->overflow_seen) return CTL_ERR_STATE;
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
    ctl_status r = launch_intersect(c, n, d_rays, d_hits, any_hit ? 1 : 0, true, stream);
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

// traverse.h — gfx950 two-level BVH traversal + Woop intersection.
//
// Semantics are those of the reference's __traceRay_internal__<false>
// (Kernel/TraceHelper.cu:88-172) and intersectKernel<ANY_HIT>
// (TraceHelper.cu:326-734): Aila–Laine while-while traversal of the instance
// BVH, per-instance ray transform by the inverse node matrix, while-while
// traversal of the mesh BVH, Woop test per leaf entry until the last-in-leaf
// flag, postponing one leaf, wave-wide exit of the inner-node loop once every
// active lane holds a postponed leaf (ballot; reference: vote.ballot,
// BVHTraversal.h:92-105).  Box spans use the same integer min/max on the fp32
// bit patterns (kepler_math, Math/MathFunc.h:402-445 -> v_min3/v_max3_i32).
//
// MI355X-specific structure:
//  * the traversal is a resumable per-lane state machine (Traverser): one
//    round() = inner nodes until every active lane holds a leaf, then the
//    postponed leaves.  Persistent kernels refill lanes whose ray finished
//    between rounds, so waves stay full on incoherent secondary rays;
//  * one traversal stack per lane for BOTH levels; the 16 most recent entries
//    live in LDS ([entry][thread] layout: consecutive lanes hit consecutive
//    banks), deeper entries spill to a private scratch array;
//  * level switch without a second stack: entering an instance pushes the
//    pending top-level node and a sentinel; the mesh level ends when that
//    sentinel (or a sentinel child, as in the reference) comes up;
//  * SINGLE specialisation for one-instance scenes (startNode < 0): the ray is
//    transformed once and only the mesh level runs (fewer live VGPRs);
//  * node = 4 x 16-B loads, Woop triangle = 3 x 16-B loads (dwordx4);
//  * no FMA contraction (-ffp-contract=off) => bit-identical to the CPU oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

#include "../ctl_bsdf.h"

namespace ctl {

#define CTL_SENTINEL 0x76543210

#ifndef CTL_LDS_STACK
#define CTL_LDS_STACK 16
#endif
constexpr int kLdsStack = CTL_LDS_STACK;   // stack entries per lane held in LDS
constexpr int kStackMax = 128;

// The wide inner-node loop hands over to the leaves once fewer than this many
// lanes of the wave still look for a leaf (1 = the reference's rule: none;
// C3 sweep: 1 -> 2098, 2 -> 2164, 4 -> 2225, 6 -> 2237, 8 -> 2216, 16 -> 2146 Mrays/s;
// later, with the current kernel, 5 / 6 / 7 agree within run-to-run noise, ~2250;
// round 3 with the LDS-parked path state: 3 / 4 / 5 / 7 -> 3185 / 3187 / 3170 / 3151;
// round 6, interleaved on one box: 1 / 2 / 3 / 4 / 6 / 8 -> 3139 / 3228 / 3235 / 3216 /
// 3166 / 3134, C5 7.99 / 7.87 / 7.87 / 7.93 / 8.03 / 8.10 ms per pass).
#ifndef CTL_LEAF_BREAK
#define CTL_LEAF_BREAK 3
#endif

// Per-ray visit order (round 4).  Every traversal is a function of its ray
// alone, never of the other rays of its wave:
//  * binary trees (CTL_SCENE_BINARY_BVH, stats launches) run the reference's
//    host order exactly (BVHTraversal.h:214: the vote mask of a lone lane), so
//    a lane stops at its first postponed leaf; results equal the reference's
//    CPU traversal bit for bit, ties included;
//  * 4-wide mesh trees speculate: after postponing leaf L1 the lane walks on to
//    its next leaf L2 with the cull distance of before L1 (`tcull`), then tests
//    L1, L2 (and the leaves stacked right behind) and takes the new distance.
//    A wave may end its node loop while such a lane is still walking (every
//    lane holds a leaf, or CTL_LEAF_BREAK); the lane then tests L1, keeps
//    `tcull`, and resumes holding a phantom leaf (kPhantomLeaf, skipped by the
//    leaf test) so it stops at L2 exactly as if it had never been interrupted.
//  Culling is the reference's (`far >= entry` against tcull), ties first-found.
// The oracle restates the same order over the same 4-wide arrays
// (oracle/oracle.cpp trace_two_level_wide).
constexpr int kPhantomLeaf = ~(int)(214783647u << 3);   // counted-leaf code of the reference's skipped
                                                        // leaf value -214783648 (BVHTraversal.h:109,221)

struct DevScene {
    const float4* bvh;          // mesh BVHNodeData, float4 units
    const float4* woop;         // TriIntersectorData, float4 units
    const uint32_t* tri_idx;    // TriIntersectorData2
    const ctl_triangle_data* tri_data;
    const ctl_material* mats;
    const ctl_kernel_mesh* meshes;
    const ctl_node* nodes;
    const float4* scene_bvh;    // instance BVH
    const float4* xf;           // node transforms, 4 float4 rows each
    const float4* inv_xf;
    const ctl_light* lights;
    const ctl_light_tri* light_tris;
    const float* light_tri_cdf;
    const float4* normal_lut;   // 65536 decoded spherical normals (Compression.h:20-31)
    const ctl_texture* textures;   // ImageTexture + KernelMIPMap records
    const uint32_t* tex_data;      // RGBCOL texels of all MIP levels
    uint32_t n_nodes;
    int32_t start_node;
    uint32_t n_lights;
    uint32_t flags;
    float ray_eps;
    // per axis, max |coordinate| of the scene box and of every mesh's local box:
    // bounds |lo| of every BVH box for the any-hit shadow cull (slab_slack)
    float cull_m[3];
    float light_cdf[CTL_MAX_NUM_LIGHTS];
    ctl_camera camera;
    // single-instance fast path (start_node < 0): mesh of node ~start_node
    uint32_t single;
    uint32_t s_node_base, s_tri_base, s_idx_base, s_tri_offset;
    // 4-wide BVH collapsed on upload (host/bvh_wide.h), traversed when WIDE
    const float4* wbvh;          // mesh wide nodes, 8 float4 (128 B) each
    const float4* scene_wbvh;    // instance-level wide nodes
    const uint32_t* mesh_wbase;  // first wide node of each mesh
    uint32_t wide;               // wide trees present (scene flag CTL_SCENE_BINARY_BVH clear)
    uint32_t full_shading;       // shading level of the path kernels: kShadeLean / kShadeFull / kShadeEnv
    uint32_t alpha;              // KernelDynamicScene::doAlphaMapping (some material has an alpha map)
    uint32_t s_wnode_base;
    uint32_t quant;              // wide trees in the 64-B quantized format (ctl_qnode.h)
    // InfiniteLight (ctl_env.h): light env_index of lights[], 0xFFFFFFFF without one
    uint32_t env_index;
    const ctl_env_light* env;
    const float* env_data;
};

struct TraceStats {
    uint32_t nodes, tris, inst;
#ifdef CTL_PROFILE_TRACE
    // SIMD occupancy of the traversal loops: per lane, iterations it was active
    // in; per wave (counted on the first active lane), iterations executed
    uint32_t inner_lanes = 0, inner_waves = 0, leaf_lanes = 0, leaf_waves = 0;
    uint32_t round_r = 0, inner_r = 0, rounds = 0, leafphase_in = 0;
#endif
};
#ifdef CTL_PROFILE_TRACE
#define CTL_PROF_COUNT(stats, L, W)                                                    \
    do {                                                                              \
        (stats)->L++;                                                                 \
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) {          \
            (stats)->W++;                                                             \
            if (&(stats)->W == &(stats)->inner_waves) (stats)->inner_r += (stats)->round_r; \
        }                                                                             \
    } while (0)
#else
#define CTL_PROF_COUNT(stats, L, W) do {} while (0)
#endif

struct HitRec {
    float t, u, v;
    uint32_t tri, node;
};

__device__ __forceinline__ int imin3(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

__device__ __forceinline__ float span_begin(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    return __int_as_float(imax3(__float_as_int(tmin(a0, a1)), __float_as_int(tmin(b0, b1)),
                                max(min(__float_as_int(c0), __float_as_int(c1)), __float_as_int(d))));
}
__device__ __forceinline__ float span_end(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    return __int_as_float(imin3(__float_as_int(tmax(a0, a1)), __float_as_int(tmax(b0, b1)),
                                min(max(__float_as_int(c0), __float_as_int(c1)), __float_as_int(d))));
}

// LDS part of the per-lane stacks: [entry][thread] (dynamic shared memory,
// kLdsStack * blockDim ints).  Indexed through this address-space-3 array so
// every push/pop is a ds_read/ds_write, never a generic (flat) access.
extern __shared__ int ctl_lds_stack[];
constexpr int kStackBlock = 256;   // every kernel using LaneStack runs 256-thread blocks

struct LaneStack {
    int* spill;     // private array of kStackMax - kLdsStack entries (scratch, deep stacks only)
    int sp;
    int tid;
    bool overflow;
    // sp never drops below 0: every pop is matched by an earlier push (the
    // bottom entry is the sentinel), so the common case is one ds op and one
    // rarely-taken branch for the deep part.
    __device__ __forceinline__ void push(int v) {
        if (sp < kLdsStack) {
            ctl_lds_stack[sp * kStackBlock + tid] = v;
        } else {
            if (sp < kStackMax) spill[sp - kLdsStack] = v;
            else overflow = true;
        }
        sp++;
    }
    __device__ __forceinline__ int pop() {
        --sp;
        int v = ctl_lds_stack[min(sp, kLdsStack - 1) * kStackBlock + tid];
        if (sp >= kLdsStack) v = sp < kStackMax ? spill[sp - kLdsStack] : CTL_SENTINEL;
        return v;
    }
};
#define CTL_LANE_STACK(name)                       \
    int name##_spill[kStackMax - kLdsStack];       \
    LaneStack name;                                \
    name.spill = name##_spill;                     \
    name.sp = 0;                                   \
    name.tid = (int)threadIdx.x;                   \
    name.overflow = false
constexpr size_t kStackLdsBytes = sizeof(int) * kLdsStack * kStackBlock;
// path_kernel_persistent keeps one word per thread after the stacks (the work
// item of the lane's path); the tail/balance experiments' areas follow it
constexpr int kPathWordOff = kLdsStack * kStackBlock;
constexpr int kExtraLdsOff = kPathWordOff + kStackBlock;

struct RayLocal {
    float ox, oy, oz, dx, dy, dz;
    float idx, idy, idz, oodx, oody, oodz;
    __device__ __forceinline__ void set(float px, float py, float pz, float qx, float qy, float qz) {
        ox = px; oy = py; oz = pz; dx = qx; dy = qy; dz = qz;
        const float ooeps = 0x1p-80f;   // exp2(-80), TraceHelper.cu:412
        idx = 1.0f / (fabsf(qx) > ooeps ? qx : copysign_ref(ooeps, qx));
        idy = 1.0f / (fabsf(qy) > ooeps ? qy : copysign_ref(ooeps, qy));
        idz = 1.0f / (fabsf(qz) > ooeps ? qz : copysign_ref(ooeps, qz));
        oodx = ox * idx; oody = oy * idy; oodz = oz * idz;
    }
};

// Bound on the rounding error of a slab distance of ray r (the Aila-Laine
// `lo * idir - o * idir`: each product and the difference rounded, idir itself
// rounded: at most 3 * 2^-24 (|lo| + |o|) |idir| per axis), with m[a] >= |lo|
// of every box (DevScene::cull_m): 2^-20 max_a (|o_a| + m_a) |idir_a|.  A box
// whose computed entry exceeds dist + slack has its exact entry past dist, so
// the any-hit shadow query culls at dist + slack (oracle occluded_query).
// Evaluated in this order on both sides, so the cull distance is bit-identical.
__host__ __device__ inline float slab_slack(float ox, float oy, float oz, float idx, float idy, float idz,
                                            const float* m) {
    const float ex = (fabsf(ox) + m[0]) * fabsf(idx);
    const float ey = (fabsf(oy) + m[1]) * fabsf(idy);
    const float ez = (fabsf(oz) + m[2]) * fabsf(idz);
    const float e = ex > ey ? ex : ey;
    return (e > ez ? e : ez) * 0x1p-20f;
}
// DevScene::cull_m: per axis, max |coordinate| of the scene box (lo, hi) and of
// the local boxes of the meshes (6 floats each, lo xyz then hi xyz).
__host__ __device__ inline void cull_bound(const float* lo, const float* hi, const float* mesh_boxes, uint32_t n_meshes,
                                           float m[3]) {
    for (int a = 0; a < 3; a++) {
        float v = fabsf(lo[a]) > fabsf(hi[a]) ? fabsf(lo[a]) : fabsf(hi[a]);
        for (uint32_t i = 0; mesh_boxes && i < n_meshes; i++) {
            const float l = fabsf(mesh_boxes[6 * i + a]), h = fabsf(mesh_boxes[6 * i + 3 + a]);
            v = l > v ? l : v;
            v = h > v ? h : v;
        }
        m[a] = v;
    }
}
__device__ __forceinline__ float slab_slack(const RayLocal& r, const float* m) {
    return slab_slack(r.ox, r.oy, r.oz, r.idx, r.idy, r.idz, m);
}

// Transform by a row-major float4x4 given as 4 float4 rows (float4x4.h:398-408).
__device__ __forceinline__ void xform_rows(const float4* M, f3 p, f3 d, f3& po, f3& doo) {
    float4 r0 = M[0], r1 = M[1], r2 = M[2], r3 = M[3];
    m44 m;
    m.d[0] = r0.x; m.d[1] = r0.y; m.d[2] = r0.z; m.d[3] = r0.w;
    m.d[4] = r1.x; m.d[5] = r1.y; m.d[6] = r1.z; m.d[7] = r1.w;
    m.d[8] = r2.x; m.d[9] = r2.y; m.d[10] = r2.z; m.d[11] = r2.w;
    m.d[12] = r3.x; m.d[13] = r3.y; m.d[14] = r3.z; m.d[15] = r3.w;
    doo = xform_dir(m, d);
    po = xform_point(m, p);
}

// Closest (ANY=0) or any (ANY=1) hit with tri_tmin < t < h.t, or chosen per
// ray by the `anyhit` member (ANY=2); box spans start at span_tmin.
// ALPHA: the traceRay flavour with Material::AlphaTest on candidate hits
// (__traceRay_internal__<true>, TraceHelper.cu:136-154), active when the scene
// has alpha maps; the batch intersectKernel never alpha-tests.
template <int ANY, bool STATS, bool SINGLE, bool WIDE = false, bool ALPHA = false>
struct Traverser4 {
    RayLocal cur;
    RayLocal world;   // unused when SINGLE
    HitRec h;
    float span_tmin, tri_tmin;
    // cull distance of the node loops: h.t, or its value before a phantom leaf;
    // the any-hit shadow query's: dist + slab_slack of the current level's ray
    // (init's anyDist = dist; its acceptance bound is h.t = dist - eps)
    float tcull;
    float cullDist;   // that query's dist (instance entry / exit recompute tcull)
    int nodeAddr, leafAddr, level, meshSent;
    uint32_t nodeBase, triBase, idxBase, triOffset, instIdx;
    bool done, resumeLeaves;
    bool anyhit;   // ANY == 2 only

    __device__ __forceinline__ void enter_instance(const DevScene& S, uint32_t inst, f3 o, f3 d) {
        instIdx = inst;
        f3 o2, d2;
        xform_rows(S.inv_xf + 4 * inst, o, d, o2, d2);
        cur.set(o2.x, o2.y, o2.z, d2.x, d2.y, d2.z);
    }

    // any-hit: h.t only changes when the query ends, so tcull keeps its start value
    __device__ __forceinline__ bool any_query() const { return ANY == 1 || (ANY == 2 && anyhit); }

    // anyDist >= 0: an any-hit shadow query to a light at anyDist (boxes culled
    // at anyDist + slab_slack); ignored by closest-hit queries
    __device__ __forceinline__ void init(const DevScene& S, f3 o, f3 d, float smin, float tmn, float tmaxv,
                                         LaneStack& st, TraceStats* stats, float anyDist = -1.0f) {
        h.t = tmaxv; h.u = h.v = 0.0f; h.tri = 0xffffffffu; h.node = 0xffffffffu;
        tcull = tmaxv;
        cullDist = anyDist;
        span_tmin = smin; tri_tmin = tmn;
        st.sp = 0;
        st.overflow = false;
        st.push(CTL_SENTINEL);
        done = (S.n_nodes == 0);
        resumeLeaves = false;
        meshSent = 0;
        if (SINGLE) {
            // start_node < 0: TracerayTemplate calls the instance callback directly (BVHTraversal.h:130-131)
            if (STATS) stats->inst++;
            enter_instance(S, ~(uint32_t)S.start_node, o, d);
            nodeBase = WIDE ? S.s_wnode_base : S.s_node_base;
            triBase = S.s_tri_base; idxBase = S.s_idx_base; triOffset = S.s_tri_offset;
            level = 1;
            nodeAddr = 0;
            leafAddr = 0;
        } else {
            world.set(o.x, o.y, o.z, d.x, d.y, d.z);
            cur = world;
            level = 0;
            nodeBase = triBase = idxBase = triOffset = instIdx = 0;
            if (S.start_node < 0) { leafAddr = S.start_node; nodeAddr = CTL_SENTINEL; }
            else { leafAddr = 0; nodeAddr = WIDE ? 0 : S.start_node; }
        }
        if (any_query() && anyDist >= 0.0f) tcull = anyDist + slab_slack(cur, S.cull_m);
    }

    // TriangleData UV set 0 at (u, v) -> Material::AlphaTest (TraceHelper.cu:140-152)
    __device__ __forceinline__ bool alpha_survives(const DevScene& S, uint32_t gtri, float u, float v) const {
        const ctl_triangle_data td = S.tri_data[gtri];
        const ctl_material& m = S.mats[((td.w[1] >> 16) & 0xffu) + S.nodes[instIdx].material_offset];
        if (!m.alpha_state) return true;
        const bool q = (S.flags & CTL_SCENE_HALF_HOST_QUIRK) != 0;
        const f2 a = mk2(half_to_float(td.w[5] & 0xffffu, q), half_to_float(td.w[5] >> 16, q));
        const f2 b = mk2(half_to_float(td.w[6] & 0xffffu, q), half_to_float(td.w[6] >> 16, q));
        const f2 c = mk2(half_to_float(td.w[7] & 0xffffu, q), half_to_float(td.w[7] >> 16, q));
        const f2 uv = u * a + v * b + (1 - u - v) * c;
        return material_alpha_test(m, TexView{S.textures, S.tex_data}, uv);
    }

    // Leaf entries from ~leafAddr until the last-in-leaf flag.  Entry i+1 is
    // loaded while entry i is tested (the uploads carry one zeroed entry past
    // the end), so a leaf costs one dependent load latency, not one per entry.
    __device__ __forceinline__ void leaf_tris(const DevScene& S, TraceStats* stats) {
        uint32_t triAddr = (uint32_t)(~leafAddr);
        const float4* tv = S.woop + triBase + triAddr * 3u;
        const uint32_t* ti = S.tri_idx + idxBase + triAddr;
        float4 v00 = tv[0], v11 = tv[1], v22 = tv[2];
        uint32_t index = ti[0];
        for (;;) {
            tv += 3;
            ti += 1;
            const float4 n00 = tv[0], n11 = tv[1], n22 = tv[2];
            const uint32_t nindex = ti[0];
            CTL_PROF_COUNT(stats, leaf_lanes, leaf_waves);
            if (STATS) stats->tris++;
            float Oz = v00.w - cur.ox * v00.x - cur.oy * v00.y - cur.oz * v00.z;
            float invDz = 1.0f / (cur.dx * v00.x + cur.dy * v00.y + cur.dz * v00.z);
            float t = Oz * invDz;
            if (t > tri_tmin && t < h.t) {   // TraceHelper.cu:121 (first found wins a tie)
                float Ox = v11.w + cur.ox * v11.x + cur.oy * v11.y + cur.oz * v11.z;
                float Dx = cur.dx * v11.x + cur.dy * v11.y + cur.dz * v11.z;
                float u = Ox + t * Dx;
                if (u >= 0.0f) {
                    float Oy = v22.w + cur.ox * v22.x + cur.oy * v22.y + cur.oz * v22.z;
                    float Dy = cur.dx * v22.x + cur.dy * v22.y + cur.dz * v22.z;
                    float v = Oy + t * Dy;
                    const uint32_t gtri = (index >> 1) + triOffset;
                    if (v >= 0.0f && u + v <= 1.0f && (!ALPHA || !S.alpha || alpha_survives(S, gtri, u, v))) {
                        h.node = instIdx;
                        h.tri = gtri;
                        h.u = u;
                        h.v = v;
                        h.t = t;
                        if (ANY == 1 || (ANY == 2 && anyhit)) { done = true; break; }
                    }
                }
            }
            if (index & 1) break;
            v00 = n00; v11 = n11; v22 = n22; index = nindex;
        }
    }

    // One Woop test of a counted leaf's entry (t, u, v exactly as leaf_tris);
    // the entry's TriIntersectorData2 word, only needed for the triangle index,
    // is loaded once the entry passes the geometric test (a candidate hit).
    __device__ __forceinline__ bool test_entry(const DevScene& S, float4 v00, float4 v11, float4 v22, uint32_t entry,
                                               uint32_t index, TraceStats* stats) {
        CTL_PROF_COUNT(stats, leaf_lanes, leaf_waves);
        if (STATS) stats->tris++;
        float Oz = v00.w - cur.ox * v00.x - cur.oy * v00.y - cur.oz * v00.z;
        float invDz = 1.0f / (cur.dx * v00.x + cur.dy * v00.y + cur.dz * v00.z);
        float t = Oz * invDz;
        if (t > tri_tmin && t < h.t) {
            float Ox = v11.w + cur.ox * v11.x + cur.oy * v11.y + cur.oz * v11.z;
            float Dx = cur.dx * v11.x + cur.dy * v11.y + cur.dz * v11.z;
            float u = Ox + t * Dx;
            if (u >= 0.0f) {
                float Oy = v22.w + cur.ox * v22.x + cur.oy * v22.y + cur.oz * v22.z;
                float Dy = cur.dx * v22.x + cur.dy * v22.y + cur.dz * v22.z;
                float v = Oy + t * Dy;
                if (v >= 0.0f && u + v <= 1.0f) {
                    (void)entry;
                    const uint32_t gtri = (index >> 1) + triOffset;
                    if (!ALPHA || !S.alpha || alpha_survives(S, gtri, u, v)) {
                        h.node = instIdx;
                        h.tri = gtri;
                        h.u = u;
                        h.v = v;
                        h.t = t;
                        if (ANY == 1 || (ANY == 2 && anyhit)) { done = true; return true; }
                    }
                }
            }
        }
        return false;
    }

    // A leaf child of a 4-wide mesh tree carries its entry count
    // (host/bvh_wide.h: ~((first << 3) | count), count 1..7, 0 = 8 or more):
    // the entries' Woop records are loaded two at a time up front, with no
    // look-ahead past the leaf and no TriIntersectorData2 load per test.  The
    // entries are tested in the reference's order; a long leaf walks its
    // last-in-leaf flags as leaf_tris does.
    __device__ __forceinline__ void leaf_counted(const DevScene& S, TraceStats* stats) {
        const uint32_t code = (uint32_t)(~leafAddr);
        const uint32_t first = code >> 3, cnt = code & 7u;
        if (first == 214783647u) return;   // the reference's -214783648 leaf value (BVHTraversal.h:109,221)
        if (cnt == 0) {
            leafAddr = ~(int)first;
            leaf_tris(S, stats);
            return;
        }
        const float4* tv = S.woop + triBase + first * 3u;
        const uint32_t* ti = S.tri_idx + idxBase + first;
        for (uint32_t i = 0; i < cnt; i += 2) {
            const float4 a0 = tv[3 * i], a1 = tv[3 * i + 1], a2 = tv[3 * i + 2];
            const uint32_t ia = ti[i];
            uint32_t ib = ia;
            float4 b0 = a0, b1 = a1, b2 = a2;
            if (i + 1 < cnt) {
                b0 = tv[3 * i + 3]; b1 = tv[3 * i + 4]; b2 = tv[3 * i + 5];
                ib = ti[i + 1];
            }
            if (test_entry(S, a0, a1, a2, first + i, ia, stats)) return;
            if (i + 1 < cnt && test_entry(S, b0, b1, b2, first + i + 1, ib, stats)) return;
        }
    }

    // Sort the hit children near-first (5-comparator network on the entry
    // distances; misses carry 0x7fffffff and sort last), take the nearest,
    // push the others far-to-near, postpone a leaf.  Shared by the float and
    // quantized 4-wide loops.
    __device__ __forceinline__ int wide_advance(int k0, int k1, int k2, int k3, int c0, int c1, int c2, int c3,
                                                bool fast, int sp, int top1, int top2, LaneStack& st) {
#define CTL_CX(KA, CA, KB, CB)                      \
        {                                       \
            const bool sw = KB < KA;            \
            const int tk = sw ? KB : KA, tc = sw ? CB : CA; \
            KB = sw ? KA : KB; CB = sw ? CA : CB; \
            KA = tk; CA = tc;                   \
        }
        CTL_CX(k0, c0, k1, c1)
        CTL_CX(k2, c2, k3, c3)
        CTL_CX(k0, c0, k2, c2)
        CTL_CX(k1, c1, k3, c3)
        CTL_CX(k1, c1, k2, c2)
#undef CTL_CX
        if (fast) {
            const int m = (k0 != 0x7fffffff) + (k1 != 0x7fffffff) + (k2 != 0x7fffffff) + (k3 != 0x7fffffff);
            // far-to-near pushes c[m-1] .. c[1] land in slots sp .. sp+m-2
            int* slot = &ctl_lds_stack[sp * kStackBlock + st.tid];
            slot[0] = m == 4 ? c3 : (m == 3 ? c2 : c1);
            slot[kStackBlock] = m == 4 ? c2 : c1;
            slot[2 * kStackBlock] = c1;
            int next, below, nsp;
            if (m == 0) { next = top1; below = top2; nsp = sp - 1; }
            else { next = c0; below = m == 1 ? top1 : c1; nsp = sp + m - 1; }
            if (next < 0 && leafAddr >= 0) {
                leafAddr = next;
                next = below;
                nsp--;
            }
            nodeAddr = next;
            st.sp = nsp;
            return m;
        } else {
            if (k3 != 0x7fffffff) st.push(c3);
            if (k2 != 0x7fffffff) st.push(c2);
            if (k1 != 0x7fffffff) st.push(c1);
            nodeAddr = (k0 != 0x7fffffff) ? c0 : st.pop();
            if (nodeAddr < 0 && leafAddr >= 0) {
                leafAddr = nodeAddr;
                nodeAddr = st.pop();
            }
            return k0 != 0x7fffffff;
        }
    }

    // 4-wide inner-node loop over 128-B float nodes (host/bvh_wide.h).
    //  * slabs in packed fp32 (v_pk_mul_f32 / v_pk_add_f32 on child pairs, the
    //    same mul-then-sub rounding as the reference's scalar code);
    //  * near/far planes picked per ray in the load address (sign of idir),
    //    which replaces the reference's per-axis min/max of the slab pair
    //    (C3: 1977 -> 2105 Mrays/s).  The pick equals `a < b ? a : b` except
    //    on a {-0, +0} pair (and NaN); under the int-ordered span, clamped
    //    below by tmin >= +0, that can only add visits to boxes that end behind
    //    the ray origin, which hold no hit with t > eps, so hits are unchanged.
    //  * empty child slots carry NaN boxes: their span compare is false, so no
    //    sentinel test per child;
    //  * hit children sorted near-first by a 5-comparator network on the entry
    //    distances (non-negative floats compare as ints), the nearest taken,
    //    the others pushed far-to-near;
    //  * stack: with room for three pushes in LDS, the two top entries are read
    //    before the node arrives and the pushes are three unconditional
    //    ds_writes (slots above the new top hold garbage), so a step carries no
    //    stack branches and no dependent LDS read; deep stacks take the
    //    generic push/pop.
    // Same postponed-leaf / wave-exit rule as the binary loop.
    __device__ __forceinline__ void inner_wide_float(const DevScene& S, LaneStack& st, TraceStats* stats) {
        typedef float v2f __attribute__((ext_vector_type(2)));
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f* nodes = reinterpret_cast<const v4f*>((SINGLE || level) ? S.wbvh : S.scene_wbvh);
        const v2f ix = {cur.idx, cur.idx}, iy = {cur.idy, cur.idy}, iz = {cur.idz, cur.idz};
        const v2f ox = {cur.oodx, cur.oodx}, oy = {cur.oody, cur.oody}, oz = {cur.oodz, cur.oodz};
        const int tminBits = __float_as_int(span_tmin);
        // Near/far planes chosen per ray by the sign of its inverse direction:
        // for idir >= 0, lo*idir - ood <= hi*idir - ood (rounding is monotone),
        // so the near plane IS the reference's min of the pair and the far
        // plane its max; the selection moves into the load address (byte
        // offsets 0/16 inside each axis' 32-B lo/hi pair) and the per-child
        // min/max disappear.  NaN (empty) slots still fail the span compare.
        const char* nbytes = reinterpret_cast<const char*>(nodes);
        const uint32_t sx = (uint32_t)(__float_as_int(cur.idx) >> 31) & 16u;
        const uint32_t sy = (uint32_t)(__float_as_int(cur.idy) >> 31) & 16u;
        const uint32_t sz = (uint32_t)(__float_as_int(cur.idz) >> 31) & 16u;
        uint32_t onx = sx, ofx = 16u - sx, ony = 32u + sy, ofy = 48u - sy, onz = 64u + sz, ofz = 80u - sz;
        // opaque to the optimiser: otherwise it splits off + (16 - s) into two ops per load
        asm volatile("" : "+v"(onx), "+v"(ofx), "+v"(ony), "+v"(ofy), "+v"(onz), "+v"(ofz));
        // speculation only inside a mesh (the instance level stops at its first leaf)
        const bool spec = SINGLE || level == 1;
        const int tBits = __float_as_int(tcull);
        while (!resumeLeaves && (unsigned)nodeAddr < (unsigned)CTL_SENTINEL &&
               (spec || leafAddr >= 0)) {
            const int sp = st.sp;
            const bool fast = sp + 3 <= kLdsStack;
            const int top1 = ctl_lds_stack[max(min(sp - 1, kLdsStack - 1), 0) * kStackBlock + st.tid];
            const int top2 = ctl_lds_stack[max(min(sp - 2, kLdsStack - 1), 0) * kStackBlock + st.tid];
            CTL_PROF_COUNT(stats, inner_lanes, inner_waves);
            if (STATS) stats->nodes++;
            int k0, k1, k2, k3;
            const uint32_t off = (nodeBase + (uint32_t)nodeAddr) << 7;
            const v4f nx = *reinterpret_cast<const v4f*>(nbytes + (off + onx));
            const v4f fx = *reinterpret_cast<const v4f*>(nbytes + (off + ofx));
            const v4f ny = *reinterpret_cast<const v4f*>(nbytes + (off + ony));
            const v4f fy = *reinterpret_cast<const v4f*>(nbytes + (off + ofy));
            const v4f nz = *reinterpret_cast<const v4f*>(nbytes + (off + onz));
            const v4f fz = *reinterpret_cast<const v4f*>(nbytes + (off + ofz));
            int4 ch = *reinterpret_cast<const int4*>(nbytes + (off + 96u));
            asm volatile("" : "+v"(ch.x), "+v"(ch.y), "+v"(ch.z), "+v"(ch.w));
            const v2f nx01 = nx.xy * ix - ox, nx23 = nx.zw * ix - ox;
            const v2f fx01 = fx.xy * ix - ox, fx23 = fx.zw * ix - ox;
            const v2f ny01 = ny.xy * iy - oy, ny23 = ny.zw * iy - oy;
            const v2f fy01 = fy.xy * iy - oy, fy23 = fy.zw * iy - oy;
            const v2f nz01 = nz.xy * iz - oz, nz23 = nz.zw * iz - oz;
            const v2f fz01 = fz.xy * iz - oz, fz23 = fz.zw * iz - oz;
            int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
#define CTL_WIDE_CHILD(K, NX, FX, NY, FY, NZ, FZ)                                                       \
            {                                                                                           \
                const float cmin = __int_as_float(imax3(__float_as_int(NX), __float_as_int(NY),          \
                                                        max(__float_as_int(NZ), tminBits)));             \
                const float cmax = __int_as_float(imin3(__float_as_int(FX), __float_as_int(FY),          \
                                                        min(__float_as_int(FZ), tBits)));                \
                K = (cmax >= cmin) ? __float_as_int(cmin) : 0x7fffffff;                                 \
            }
            CTL_WIDE_CHILD(k0, nx01.x, fx01.x, ny01.x, fy01.x, nz01.x, fz01.x)
            CTL_WIDE_CHILD(k1, nx01.y, fx01.y, ny01.y, fy01.y, nz01.y, fz01.y)
            CTL_WIDE_CHILD(k2, nx23.x, fx23.x, ny23.x, fy23.x, nz23.x, fz23.x)
            CTL_WIDE_CHILD(k3, nx23.y, fx23.y, ny23.y, fy23.y, nz23.y, fz23.y)
#undef CTL_WIDE_CHILD
            wide_advance(k0, k1, k2, k3, c0, c1, c2, c3, fast, sp, top1, top2, st);
            if (__popcll(__ballot(leafAddr >= 0)) < CTL_LEAF_BREAK) break;
        }
    }

    // 4-wide loop over 64-B quantized nodes (ctl_qnode.h, CTL_SCENE_WIDE_QUANT):
    // four 16-B loads per node instead of seven.  The near/far plane of each
    // axis is a choice between two packed words (one byte per child), made per
    // ray; each bound is decoded exactly as the encoder checked it
    // (p + float(q) * s, mul then add), then the same slab test, sort and
    // stack update as the float loop.
    __device__ __forceinline__ void inner_wide_quant(const DevScene& S, LaneStack& st, TraceStats* stats) {
        typedef float v2f __attribute__((ext_vector_type(2)));
        const char* nbytes = reinterpret_cast<const char*>((SINGLE || level) ? S.wbvh : S.scene_wbvh);
        const v2f ix = {cur.idx, cur.idx}, iy = {cur.idy, cur.idy}, iz = {cur.idz, cur.idz};
        const v2f ox = {cur.oodx, cur.oodx}, oy = {cur.oody, cur.oody}, oz = {cur.oodz, cur.oodz};
        const int tminBits = __float_as_int(span_tmin);
        const bool negx = __float_as_int(cur.idx) < 0, negy = __float_as_int(cur.idy) < 0;
        const bool negz = __float_as_int(cur.idz) < 0;
        // speculation only inside a mesh (the instance level stops at its first leaf)
        const bool spec = SINGLE || level == 1;
        const int tBits = __float_as_int(tcull);
        while (!resumeLeaves && (unsigned)nodeAddr < (unsigned)CTL_SENTINEL &&
               (spec || leafAddr >= 0)) {
            const int sp = st.sp;
            const bool fast = sp + 3 <= kLdsStack;
            const int top1 = ctl_lds_stack[max(min(sp - 1, kLdsStack - 1), 0) * kStackBlock + st.tid];
            const int top2 = ctl_lds_stack[max(min(sp - 2, kLdsStack - 1), 0) * kStackBlock + st.tid];
            CTL_PROF_COUNT(stats, inner_lanes, inner_waves);
            if (STATS) stats->nodes++;
            const uint32_t off = (nodeBase + (uint32_t)nodeAddr) << 6;
            const float4 qa = *reinterpret_cast<const float4*>(nbytes + off);
            const float4 qb = *reinterpret_cast<const float4*>(nbytes + off + 16u);
            const float4 qc = *reinterpret_cast<const float4*>(nbytes + off + 32u);
            int4 ch = *reinterpret_cast<const int4*>(nbytes + off + 48u);
            asm volatile("" : "+v"(ch.x), "+v"(ch.y), "+v"(ch.z), "+v"(ch.w));
            const uint32_t wlx = __float_as_uint(qb.z), whx = __float_as_uint(qb.w);
            const uint32_t wly = __float_as_uint(qc.x), why = __float_as_uint(qc.y);
            const uint32_t wlz = __float_as_uint(qc.z), whz = __float_as_uint(qc.w);
            const uint32_t nxw = negx ? whx : wlx, fxw = negx ? wlx : whx;
            const uint32_t nyw = negy ? why : wly, fyw = negy ? wly : why;
            const uint32_t nzw = negz ? whz : wlz, fzw = negz ? wlz : whz;
#define CTL_QB(W, K) ((float)(((W) >> (8 * (K))) & 0xffu))
            // p + q * s in one fused op: q * s is exact (q < 256, s a power of two), so the
            // fused result is the encoder's p + q * s (mul, then add) bit for bit
#define CTL_QPAIR(W, P, SC, K0, K1) \
    __builtin_elementwise_fma(v2f{CTL_QB(W, K0), CTL_QB(W, K1)}, v2f{(SC), (SC)}, v2f{(P), (P)})
            const v2f nx01 = CTL_QPAIR(nxw, qa.x, qa.w, 0, 1) * ix - ox, nx23 = CTL_QPAIR(nxw, qa.x, qa.w, 2, 3) * ix - ox;
            const v2f fx01 = CTL_QPAIR(fxw, qa.x, qa.w, 0, 1) * ix - ox, fx23 = CTL_QPAIR(fxw, qa.x, qa.w, 2, 3) * ix - ox;
            const v2f ny01 = CTL_QPAIR(nyw, qa.y, qb.x, 0, 1) * iy - oy, ny23 = CTL_QPAIR(nyw, qa.y, qb.x, 2, 3) * iy - oy;
            const v2f fy01 = CTL_QPAIR(fyw, qa.y, qb.x, 0, 1) * iy - oy, fy23 = CTL_QPAIR(fyw, qa.y, qb.x, 2, 3) * iy - oy;
            const v2f nz01 = CTL_QPAIR(nzw, qa.z, qb.y, 0, 1) * iz - oz, nz23 = CTL_QPAIR(nzw, qa.z, qb.y, 2, 3) * iz - oz;
            const v2f fz01 = CTL_QPAIR(fzw, qa.z, qb.y, 0, 1) * iz - oz, fz23 = CTL_QPAIR(fzw, qa.z, qb.y, 2, 3) * iz - oz;
#undef CTL_QPAIR
#undef CTL_QB
            int k0, k1, k2, k3, c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
#define CTL_WIDE_CHILD(K, C, NX, FX, NY, FY, NZ, FZ)                                                    \
            {                                                                                           \
                const float cmin = __int_as_float(imax3(__float_as_int(NX), __float_as_int(NY),          \
                                                        max(__float_as_int(NZ), tminBits)));             \
                const float cmax = __int_as_float(imin3(__float_as_int(FX), __float_as_int(FY),          \
                                                        min(__float_as_int(FZ), tBits)));                \
                K = (cmax >= cmin && C != CTL_SENTINEL) ? __float_as_int(cmin) : 0x7fffffff;            \
            }
            CTL_WIDE_CHILD(k0, c0, nx01.x, fx01.x, ny01.x, fy01.x, nz01.x, fz01.x)
            CTL_WIDE_CHILD(k1, c1, nx01.y, fx01.y, ny01.y, fy01.y, nz01.y, fz01.y)
            CTL_WIDE_CHILD(k2, c2, nx23.x, fx23.x, ny23.x, fy23.x, nz23.x, fz23.x)
            CTL_WIDE_CHILD(k3, c3, nx23.y, fx23.y, ny23.y, fy23.y, nz23.y, fz23.y)
#undef CTL_WIDE_CHILD
            wide_advance(k0, k1, k2, k3, c0, c1, c2, c3, fast, sp, top1, top2, st);
            if (__popcll(__ballot(leafAddr >= 0)) < CTL_LEAF_BREAK) break;
        }
    }

    __device__ __forceinline__ void inner_binary(const DevScene& S, LaneStack& st, TraceStats* stats) {
        const float4* nodes = (SINGLE || level) ? S.bvh : S.scene_bvh;
        // the reference's host order: the lane stops at its first postponed leaf
        // (BVHTraversal.h:214, mask = leafAddr >= 0)
        while (!resumeLeaves && (unsigned)nodeAddr < (unsigned)CTL_SENTINEL && leafAddr >= 0) {
            const float4* n = nodes + nodeBase + nodeAddr;
            const float4 n0xy = n[0];
            const float4 n1xy = n[1];
            const float4 nz = n[2];
            const float4 tmp = n[3];
            if (STATS) stats->nodes++;
            int c0i = __float_as_int(tmp.x), c1i = __float_as_int(tmp.y);
            // keep the child-index load beside the box loads: left to itself the
            // compiler sinks it behind the box test, a second dependent L2 trip
            asm volatile("" : "+v"(c0i), "+v"(c1i));
            const float c0lox = n0xy.x * cur.idx - cur.oodx;
            const float c0hix = n0xy.y * cur.idx - cur.oodx;
            const float c0loy = n0xy.z * cur.idy - cur.oody;
            const float c0hiy = n0xy.w * cur.idy - cur.oody;
            const float c0loz = nz.x * cur.idz - cur.oodz;
            const float c0hiz = nz.y * cur.idz - cur.oodz;
            const float c1loz = nz.z * cur.idz - cur.oodz;
            const float c1hiz = nz.w * cur.idz - cur.oodz;
            const float c0min = span_begin(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, span_tmin);
            const float c0max = span_end(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, tcull);
            const float c1lox = n1xy.x * cur.idx - cur.oodx;
            const float c1hix = n1xy.y * cur.idx - cur.oodx;
            const float c1loy = n1xy.z * cur.idy - cur.oody;
            const float c1hiy = n1xy.w * cur.idy - cur.oody;
            const float c1min = span_begin(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, span_tmin);
            const float c1max = span_end(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, tcull);
            bool swp = (c1min < c0min);
            bool tc0 = (c0max >= c0min);
            bool tc1 = (c1max >= c1min);
            if (!tc0 && !tc1) {
                nodeAddr = st.pop();
            } else {
                nodeAddr = tc0 ? c0i : c1i;
                if (tc0 && tc1) {
                    if (swp) { int t = nodeAddr; nodeAddr = c1i; c1i = t; }
                    st.push(c1i);
                }
            }
            if (nodeAddr < 0 && leafAddr >= 0) {
                leafAddr = nodeAddr;
                nodeAddr = st.pop();
            }
            if (__popcll(__ballot(leafAddr >= 0)) < CTL_LEAF_BREAK) break;
        }
    }

    // One round: inner nodes until every active lane holds a postponed leaf,
    // then the postponed leaves (and the level transitions).
    __device__ __forceinline__ void round(const DevScene& S, LaneStack& st, TraceStats* stats) {
#ifdef CTL_PROFILE_TRACE
        stats->round_r = (uint32_t)__popcll(__ballot(1));
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) stats->rounds++;
#endif
        if (WIDE) {
            if (S.quant) inner_wide_quant(S, st, stats);
            else inner_wide_float(S, st, stats);
        }
        else inner_binary(S, st, stats);
        resumeLeaves = false;
        // a speculating lane the wave stopped before it reached its next leaf
        const bool cut = WIDE && (SINGLE || level == 1) && leafAddr < 0 && (unsigned)nodeAddr < (unsigned)CTL_SENTINEL;
#ifdef CTL_PROFILE_TRACE
        {
            const uint32_t nl = (uint32_t)__popcll(__ballot(leafAddr < 0));
            if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) stats->leafphase_in += nl;
        }
#endif
        while (leafAddr < 0) {
            if (SINGLE || level == 1) {
                if (WIDE) {
                    leaf_counted(S, stats);
                    if (done) return;
                } else if (leafAddr != -214783648) {
                    leaf_tris(S, stats);
                    if (done) return;
                }
                leafAddr = nodeAddr;
                if (nodeAddr < 0) nodeAddr = st.pop();
            } else {
                if (leafAddr != -214783648) {
                    // enter instance ~leafAddr (TraceHelper.cu:91-100, 528-561)
                    const uint32_t inst = (uint32_t)(~leafAddr);
                    if (STATS) stats->inst++;
                    const ctl_node& N = S.nodes[inst];
                    const ctl_kernel_mesh& M = S.meshes[N.mesh_index];
                    nodeBase = WIDE ? S.mesh_wbase[N.mesh_index] : M.bvh_node_offset;
                    triBase = M.bvh_triangle_offset;
                    idxBase = M.bvh_indices_offset;
                    triOffset = M.triangle_offset;
                    enter_instance(S, inst, mk3(world.ox, world.oy, world.oz), mk3(world.dx, world.dy, world.dz));
                    st.push(nodeAddr);        // pending top-level work
                    meshSent = st.sp;
                    st.push(CTL_SENTINEL);    // bottom of the mesh-level stack
                    level = 1;
                    nodeAddr = 0;             // mesh root (TraceHelper.cu:170)
                    leafAddr = 0;
                    if (!any_query()) tcull = h.t;
                    else if (cullDist >= 0.0f) tcull = cullDist + slab_slack(cur, S.cull_m);   // the mesh's ray
                    return;
                }
                leafAddr = nodeAddr;
                if (nodeAddr < 0) nodeAddr = st.pop();
            }
        }
        if (cut) leafAddr = kPhantomLeaf;   // walk on to the next leaf with the old tcull
        else if (!any_query()) tcull = h.t;
        if (nodeAddr == CTL_SENTINEL) {
            if (!SINGLE && level == 1) {
                // mesh traversal finished (bottom sentinel or a sentinel child)
                st.sp = meshSent;
                int saved = st.pop();
                level = 0;
                nodeBase = 0;
                cur = world;
                if (any_query() && cullDist >= 0.0f) tcull = cullDist + slab_slack(cur, S.cull_m);
                leafAddr = saved;
                nodeAddr = saved;
                if (saved < 0) nodeAddr = st.pop();
                resumeLeaves = leafAddr < 0;   // the reference's leaf loop continues right away
            } else {
                done = true;
            }
        }
    }
};

template <int ANY, bool STATS, bool SINGLE, int WIDE = 0, bool ALPHA = false>
using Traverser = Traverser4<ANY, STATS, SINGLE, WIDE != 0, ALPHA>;

// Whole traversal of one ray (megakernel, batch kernel).
template <int ANY, bool STATS, bool SINGLE, int WIDE = 0, bool ALPHA = false>
__device__ __forceinline__ bool trace_one(const DevScene& S, f3 ori, f3 dir, float span_tmin, float tri_tmin,
                                          HitRec& h, LaneStack& st, TraceStats* stats, float anyDist = -1.0f) {
    Traverser<ANY, STATS, SINGLE, WIDE, ALPHA> T;
    T.init(S, ori, dir, span_tmin, tri_tmin, h.t, st, stats, anyDist);
    while (!T.done) T.round(S, st, stats);
    h = T.h;
    return !st.overflow;
}

template <bool ANY, bool STATS>
__device__ __forceinline__ bool trace_ray_dev(const DevScene& S, f3 ori, f3 dir, float span_tmin, float tri_tmin,
                                              HitRec& h, LaneStack& st, TraceStats* stats) {
    if (S.single) return trace_one<ANY, STATS, true>(S, ori, dir, span_tmin, tri_tmin, h, st, stats);
    return trace_one<ANY, STATS, false>(S, ori, dir, span_tmin, tri_tmin, h, st, stats);
}

}  // namespace ctl

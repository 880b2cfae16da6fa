// anim.hip — animated (skinned) meshes on the device: AnimatedMesh::k_ComputeState
// (Engine/AnimatedMesh.cpp:163-184) as a chain of data-parallel kernels, and the
// instance tree after ctl_scene_animate / ctl_scene_set_transform.
//
//   skin     g_ComputeVertices (AnimatedMesh.cu:29-43): per vertex, two 8-bone
//            matrix blends, TransformPoint / TransformDirection, lerp
//   tris     g_ComputeTriangles -> TriangleData::setData (TriangleData.cu:35-63)
//   rebuild  the mesh tree as BVHRebuilder::Build(&p, true) leaves it
//            (AnimatedMesh.cpp:174-176, BVHRebuilder.cpp:281-340, 365-450): one
//            thread per leaf writes its entries' Woop data (AnimProvider::
//            setObject, AnimatedMesh.cpp:113-117) and the union of their
//            triangles' boxes into the slot that holds the leaf, then climbs:
//            the last of a node's children to arrive (an atomic counter per
//            node) recomputes the node -- its inner children's boxes, the best
//            of the four child/grandchild rotations by SAH if strictly cheaper
//            (host/bvh_rebuild.h states the rules), the moved subtrees' parent
//            words and leaf records -- and moves on to its parent.  A node is
//            recomputed after its whole subtree, as in the reference's
//            post-order recursion, and nodes of disjoint subtrees never touch
//            the same words, so the result is the recursion's.  The tree's
//            shape persists from frame to frame, as the reference's does.  The
//            4-wide copy keeps the topology the upload collapsed and is refit in
//            the same launch, bottom-up by arrival counts from the same leaves.
//   scene    instance boxes (mesh box x node transform) and the scene box ->
//            m_rayTraceEps on the device; the instance tree rebuilt on the host
//            along the moved instances' paths (SceneBVH::Build, the same
//            BVHRebuilder without invalidateAll), its 4-wide copy refit in its
//            topology, both uploaded.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"
#include "../ctl_anim.h"
#include "../ctl_shade.h"
#include "../host/bvh_wide.h"
#include "../host/bvh_rebuild.h"
#include "../ctl_qnode.h"

namespace ctl {

// The rebuild of one animated mesh's trees.
struct MeshRebuild {
    uint32_t n_nodes = 0;               // binary nodes of the mesh tree
    uint32_t n_leaf = 0;
    uint4* d_leaf = nullptr;            // {holder << 1 | slot, first entry, entries, wide node << 2 | slot}
    uint32_t* d_leaf_of = nullptr;      // per entry of the mesh: the record of the leaf starting there
    float* d_nrec = nullptr;            // per binary node: its box (6) and numLeafs (bvhNodeData), 32 B
    float* d_lrec = nullptr;            // per leaf: its box and entries, 32 B
    float* d_wrec = nullptr;            // per 4-wide node: its box, 32 B
    uint32_t* d_cnt = nullptr;          // arrival counters per binary node (0 between launches)
    uint32_t n_wide = 0;                // 4-wide nodes of the mesh (0: binary scene)
    uint32_t* d_wup = nullptr;          // per wide node: parent << 2 | slot (0xffffffff: the root)
    uint32_t* d_wcnt = nullptr;         // arrival counters per wide node
};

struct AnimMeshPlan {
    ctl_anim_mesh am;
    ctl_kernel_mesh km;
    uint32_t n_entries = 0;
    uint32_t wide_base = 0;             // the mesh's first wide node
    MeshRebuild rb;
};

// Host copies of the instance trees: the rebuild changes their shape, so each
// call starts from the last one's.
struct SceneTrees {
    std::vector<ctl_bvh_node> bin;
    int32_t root = -1;                  // start node (float4 offset); < 0: no instance tree
    std::vector<WideNode> wide;
    std::vector<uint32_t> wide_post;    // wide nodes, children before parents
};

struct AnimState {
    std::vector<AnimMeshPlan> meshes;
    SceneTrees scene;
    const ctl_anim_vertex* d_verts = nullptr;
    const uint32_t* d_tris = nullptr;
    float* d_mesh_boxes = nullptr;      // 6 per mesh
    float* d_inst_boxes = nullptr;      // 6 per node
    float* d_eps = nullptr;             // scene box (6) + eps + cull_m (3)
    float* h_eps = nullptr;             // pinned: the same 10 floats, then 6 per node (instance boxes)
    float4* d_P = nullptr;
    float4* d_N = nullptr;
    size_t tmp_cap = 0;
    float* d_bones[2] = {nullptr, nullptr};
    size_t bones_cap = 0;
    uint32_t n_meshes = 0, n_nodes = 0;
    std::vector<uint32_t> node_mesh;    // Node::m_uMeshIndex per node
    std::vector<void*> allocs;
};

namespace {

constexpr int32_t kSent = 0x76543210;
constexpr int kAB = 256;

__device__ __forceinline__ void box_empty(float lo[3], float hi[3]) {
    lo[0] = lo[1] = lo[2] = FLT_MAX;
    hi[0] = hi[1] = hi[2] = -FLT_MAX;
}
__device__ __forceinline__ void box_extend(float lo[3], float hi[3], const float* plo, const float* phi) {
    for (int k = 0; k < 3; k++) { lo[k] = tmin(lo[k], plo[k]); hi[k] = tmax(hi[k], phi[k]); }
}

// Bone matrices of both frames staged in LDS (<= 256 bones x 2 x 64 B = 32 KB):
// each vertex reads 8 matrices per frame.
__global__ __launch_bounds__(kAB) void anim_skin_kernel(const ctl_anim_vertex* __restrict__ V, uint32_t n,
                                                       const float* __restrict__ b0, const float* __restrict__ b1,
                                                       uint32_t n_bones, float t, float4* P, float4* N) {
    // stride 17 floats: lanes reading the same element of different bones hit different banks
    extern __shared__ float bones[];
    const uint32_t nf = 17 * n_bones;
    for (uint32_t k = threadIdx.x; k < 32 * n_bones; k += kAB) {
        const uint32_t f = k >> 4, j = (f < n_bones ? f : f - n_bones), e = k & 15u;
        bones[(f < n_bones ? 0 : nf) + 17 * j + e] = f < n_bones ? b0[16 * j + e] : b1[16 * j + e];
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= n) return;
    f3 p, nn;
    skin_vertex(V[i], bones, bones + nf, 17, t, p, nn);
    P[i] = make_float4(p.x, p.y, p.z, 0.0f);
    N[i] = make_float4(nn.x, nn.y, nn.z, 0.0f);
}

__device__ __forceinline__ f3 ld3(const float4* a, uint32_t i) { float4 q = a[i]; return mk3(q.x, q.y, q.z); }

__global__ __launch_bounds__(kAB) void anim_tri_kernel(const uint32_t* __restrict__ tris, uint32_t n,
                                                      const float4* __restrict__ P, const float4* __restrict__ N,
                                                      ctl_triangle_data* td) {
    const uint32_t t = blockIdx.x * kAB + threadIdx.x;
    if (t >= n) return;
    const uint32_t a = tris[3 * t], b = tris[3 * t + 1], c = tris[3 * t + 2];
    ctl_triangle_data r = td[t];
    // g_ComputeTriangles runs setData on the device: UVs read back with __half2float
    triangle_set_data(r.w, ld3(P, a), ld3(P, b), ld3(P, c), ld3(N, a), ld3(N, b), ld3(N, c), false);
    td[t] = r;
}

// ---------------------------------------------------------------------------
// Mesh tree rebuild (one launch per animated mesh)
// ---------------------------------------------------------------------------
struct DBox {
    float lo[3], hi[3];
};

__device__ __forceinline__ DBox dbox_identity() {
    return DBox{{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}};
}
// AABB::Extend (Math/AABB.h:72-78), this box first
__device__ __forceinline__ DBox dbox_union(const DBox& a, const DBox& b) {
    DBox r;
    for (int k = 0; k < 3; k++) { r.lo[k] = tmin(a.lo[k], b.lo[k]); r.hi[k] = tmax(a.hi[k], b.hi[k]); }
    return r;
}
// AABB::Area (Math/AABB.h:19-23); no contraction (-ffp-contract=off)
__device__ __forceinline__ float dbox_area(const DBox& b) {
    const float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
    return 2.0f * (x * y + x * z + y * z);
}
// What one thread of the launch hands to another goes through small records
// written and read with agent-scope relaxed atomics (global_store / global_load
// with sc1 on gfx950), each access coherent across the XCDs' L2s by itself:
// per leaf its box and objects (lrec), per binary node its box and objects
// (nrec), per 4-wide node its box (wrec).  Words two threads of the launch may
// write (binary slots, child and parent words, a leaf's holder) are stored the
// same way, so the last writer wins whatever the XCDs' write-back order; the
// 4-wide slots have one writer each and take plain stores.  An acquire /
// release at agent scope would instead write back and
// invalidate the whole L2 at every arrival (buffer_wbl2 / buffer_inv sc1): the
// first version did, 7.85 ms per animate.  The arrival orders the accesses: a
// thread's records complete (s_waitcnt vmcnt(0)) before its arrival increments
// the counter, and the last arriver's loads are issued after the counter's
// value came back.
__device__ __forceinline__ float2 cld2(const float* p) {
    const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
}
__device__ __forceinline__ void cst2(float* p, float a, float b) {
    const uint64_t v = (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// BVHNodeData child slots (TriIntersectorData.h:44-88).  A slot can be written
// by two threads of one launch (the node's own rebuild, then a rotation at its
// parent that makes it the `other` child), so its stores are coherent: a plain
// store could sit dirty in one XCD's L2 and be written back after the other.
// Reads are plain: only empty slots are read, which nothing rewrites.
__device__ __forceinline__ DBox slot_box(const float* nd, int c) {
    const float4 q = reinterpret_cast<const float4*>(nd)[c];
    const float2 z = reinterpret_cast<const float2*>(nd + 8)[c];
    return DBox{{q.x, q.z, z.x}, {q.y, q.w, z.y}};
}
__device__ __forceinline__ void set_slot(float* nd, int c, const DBox& b) {
    cst2(nd + 4 * c, b.lo[0], b.hi[0]);
    cst2(nd + 4 * c + 2, b.lo[1], b.hi[1]);
    cst2(nd + 8 + 2 * c, b.lo[2], b.hi[2]);
}
// a node's child words: plain when no rotation of this launch can have moved
// them yet, coherent otherwise
__device__ __forceinline__ void kids_plain(const float* nd, int32_t k[2]) {
    const float2 v = reinterpret_cast<const float2*>(nd + 12)[0];
    k[0] = __float_as_int(v.x);
    k[1] = __float_as_int(v.y);
}
__device__ __forceinline__ void kids_coherent(const float* nd, int32_t k[2]) {
    const float2 v = cld2(nd + 12);
    k[0] = __float_as_int(v.x);
    k[1] = __float_as_int(v.y);
}
__device__ __forceinline__ void set_kids(float* nd, int32_t a, int32_t b) { cst2(nd + 12, __int_as_float(a), __int_as_float(b)); }

// A record: getBox and numLeafs (bvhNodeData) in 32 B
__device__ __forceinline__ void rec_load(const float* r, DBox& b, int& n) {
    const float2 a = cld2(r), c = cld2(r + 2), d = cld2(r + 4), e = cld2(r + 6);
    b = DBox{{a.x, a.y, c.x}, {c.y, d.x, d.y}};
    n = __float_as_int(e.x);
}
__device__ __forceinline__ void rec_store(float* r, const DBox& b, int n) {
    cst2(r, b.lo[0], b.lo[1]);
    cst2(r + 2, b.lo[2], b.hi[0]);
    cst2(r + 4, b.hi[1], b.hi[2]);
    cst2(r + 6, __int_as_float(n), 0.0f);
}

struct RebuildArgs {
    float* bin;                 // the mesh tree's node 0
    WideNode* wide;             // its first 4-wide node (nullptr: no wide copy)
    const uint32_t* idx;        // the mesh's TriIntersectorData2 entries
    const uint32_t* tris;       // the mesh's triangles (skinned vertex indices)
    const float4* P;            // skinned positions
    float4* woop;               // the mesh's TriIntersectorData entries
    uint4* leaf;
    const uint32_t* leaf_of;
    float* nrec;                // per binary node {lo xyz, hi xyz, objects, 0}: written when the node is rebuilt
    float* lrec;                // per leaf record, the same: written by the leaf's thread
    float* wrec;                // per 4-wide node, its box: written when the node is refit
    uint32_t* cnt;
    const uint32_t* wup;
    uint32_t* wcnt;
    float* mesh_box;            // m_sLocalBox: 6 floats
    uint32_t n_leaf;
};

// The last of `need` arrivals at counter k goes on (and leaves the counter at
// 0 for the next launch).  The caller's coherent stores complete first.
__device__ __forceinline__ bool arrive(uint32_t* cnt, uint32_t k, uint32_t need) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(cnt + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::: "memory");   // no load of the arrivals' records is hoisted above the counter
    if (old + 1 < need) return false;
    __hip_atomic_store(cnt + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// getBox / numLeafs of child value v (from the child's record)
__device__ __forceinline__ void child_info(const RebuildArgs& A, int32_t v, DBox& b, int& n) {
    if (v == kSent) { b = dbox_identity(); n = 0; }
    else if (v < 0) rec_load(A.lrec + 8 * (size_t)A.leaf_of[(uint32_t)~v], b, n);
    else rec_load(A.nrec + 8 * (size_t)((uint32_t)v >> 2), b, n);
}

// BVHRebuilder::setChild's array writes for a moved child (read by the next
// launch; a child can move twice in one launch): the parent word of an inner
// node, the holder of a leaf's record
__device__ __forceinline__ void moved_to(const RebuildArgs& A, int32_t v, uint32_t node, int slot) {
    if (v == kSent) return;
    if (v >= 0)
        __hip_atomic_store(reinterpret_cast<int32_t*>(A.bin + 16 * (size_t)((uint32_t)v >> 2) + 14), (int32_t)(node << 2),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        __hip_atomic_store(&A.leaf[A.leaf_of[(uint32_t)~v]].x, node << 1 | (uint32_t)slot, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// recomputeNode (BVHRebuilder.cpp:281-340) of node x, its subtree done.
// Returns x's box (BVHNodeData::getBox: both slots).
__device__ DBox rebuild_node(const RebuildArgs& A, uint32_t x, const int32_t c[2]) {
    float* X = A.bin + 16 * (size_t)x;
    DBox cb[2], gb[2][2], sb[2];
    int cn[2], gn[2][2];
    int32_t g[2][2];
    bool can[2];
    for (int i = 0; i < 2; i++) {
        child_info(A, c[i], cb[i], cn[i]);
        sb[i] = c[i] == kSent ? slot_box(X, i) : cb[i];   // the stored slot (an empty one as stored)
        can[i] = false;
        if (c[i] >= 0 && c[i] != kSent) {
            kids_coherent(A.bin + 16 * (size_t)((uint32_t)c[i] >> 2), g[i]);   // the child's rotation may have moved them
            for (int j = 0; j < 2; j++) child_info(A, g[i][j], gb[i][j], gn[i][j]);
            can[i] = g[i][0] != kSent && g[i][1] != kSent;   // numberGrandchildren == 2
        }
    }
    // sah(idx, child, grandchild) (:624-638) for the four rotations
    float rot[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    if (can[0]) {
        rot[0] = dbox_area(dbox_union(cb[1], gb[0][1])) * (float)(cn[1] + gn[0][1]) + dbox_area(gb[0][0]) * (float)gn[0][0];
        rot[1] = dbox_area(dbox_union(cb[1], gb[0][0])) * (float)(cn[1] + gn[0][0]) + dbox_area(gb[0][1]) * (float)gn[0][1];
    }
    if (can[1]) {
        rot[2] = dbox_area(dbox_union(cb[0], gb[1][0])) * (float)(cn[0] + gn[1][0]) + dbox_area(gb[1][1]) * (float)gn[1][1];
        rot[3] = dbox_area(dbox_union(cb[0], gb[1][1])) * (float)(cn[0] + gn[1][1]) + dbox_area(gb[1][0]) * (float)gn[1][0];
    }
    int best = 0;
    for (int i = 1; i < 4; i++)
        if (rot[i] < rot[best]) best = i;   // std::min_element: the first smallest
    const float now = dbox_area(cb[0]) * (float)cn[0] + dbox_area(cb[1]) * (float)cn[1];
    float* xr = A.nrec + 8 * (size_t)x;
    const int xn = __float_as_int(cld2(xr + 6).x);   // numLeafs(x): no rotation at x changes it
    if (!(rot[best] < now)) {
        // node->setLeft / setRight(newBox) for the recomputed children
        for (int i = 0; i < 2; i++)
            if (c[i] != kSent) set_slot(X, i, cb[i]);
        const DBox xb = dbox_union(sb[0], sb[1]);
        rec_store(xr, xb, xn);
        return xb;
    }
    // swapChildren(idx, lc, lg) (:691-702): child c[lc] and grandchild g[1-lc][lg] trade places
    const int lc = best < 2 ? 1 : 0, lg = (best == 1 || best == 2) ? 1 : 0, o = 1 - lc;
    const uint32_t other = (uint32_t)c[o] >> 2;
    float* O = A.bin + 16 * (size_t)other;
    set_kids(O, lg == 0 ? c[lc] : g[o][0], lg == 0 ? g[o][1] : c[lc]);
    set_slot(O, lg, cb[lc]);
    moved_to(A, c[lc], other, lg);
    // propagateBBChange(other -> x): the other child's box, its slots in order
    const DBox ob = lg == 0 ? dbox_union(cb[lc], gb[o][1]) : dbox_union(gb[o][0], cb[lc]);
    set_kids(X, lc == 0 ? g[o][lg] : c[0], lc == 0 ? c[1] : g[o][lg]);
    set_slot(X, o, ob);
    set_slot(X, lc, gb[o][lg]);
    moved_to(A, g[o][lg], x, lc);
    // BVHNodeInfo::changeCount, net: the other child's objects change by the swap
    rec_store(A.nrec + 8 * (size_t)other, ob, cn[o] + cn[lc] - gn[o][lg]);
    const DBox xb = lc == 0 ? dbox_union(gb[o][lg], ob) : dbox_union(ob, gb[o][lg]);
    rec_store(xr, xb, xn);
    return xb;
}

// One thread per leaf: Woop data and the leaf's box, then up both trees.
__global__ __launch_bounds__(kAB) void anim_rebuild_kernel(RebuildArgs A) {
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= A.n_leaf) return;
    const uint4 lf = A.leaf[i];
    float lo[3], hi[3];
    box_empty(lo, hi);
#pragma unroll 2
    for (uint32_t e = lf.y; e < lf.y + lf.z; e++) {
        const uint32_t t = A.idx[e] >> 1;
        const f3 a = ld3(A.P, A.tris[3 * t]), b = ld3(A.P, A.tris[3 * t + 1]), c = ld3(A.P, A.tris[3 * t + 2]);
        float w[12];
        woop_set_hd(a, b, c, w);
        A.woop[3 * e] = make_float4(w[0], w[1], w[2], w[3]);
        A.woop[3 * e + 1] = make_float4(w[4], w[5], w[6], w[7]);
        A.woop[3 * e + 2] = make_float4(w[8], w[9], w[10], w[11]);
        const float q0[3] = {tmin(tmin(a.x, b.x), c.x), tmin(tmin(a.y, b.y), c.y), tmin(tmin(a.z, b.z), c.z)};
        const float q1[3] = {tmax(tmax(a.x, b.x), c.x), tmax(tmax(a.y, b.y), c.y), tmax(tmax(a.z, b.z), c.z)};
        box_extend(lo, hi, q0, q1);
    }
    const DBox lb{{lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}};
    rec_store(A.lrec + 8 * (size_t)i, lb, (int)lf.z);
    // the 4-wide copy: its leaf slot, then every node whose slots have all arrived
    if (A.wide) {
        uint32_t w = lf.w >> 2, sl = lf.w & 3u;
        DBox b = lb;
        for (;;) {
            WideNode& W = A.wide[w];
            W.lo_x[sl] = b.lo[0]; W.lo_y[sl] = b.lo[1]; W.lo_z[sl] = b.lo[2];
            W.hi_x[sl] = b.hi[0]; W.hi_y[sl] = b.hi[1]; W.hi_z[sl] = b.hi[2];
            const int4 ch = *reinterpret_cast<const int4*>(W.child);   // the topology: fixed since the upload
            const uint32_t need = (ch.x != kSent) + (ch.y != kSent) + (ch.z != kSent) + (ch.w != kSent);
            if (!arrive(A.wcnt, w, need)) break;
            const uint32_t up = A.wup[w];
            if (up == 0xffffffffu) break;
            const int32_t chk[4] = {ch.x, ch.y, ch.z, ch.w};
            b = dbox_identity();
            for (int k = 0; k < 4; k++) {
                if (chk[k] == kSent) continue;
                DBox cbx;
                int n;
                if (chk[k] >= 0) rec_load(A.wrec + 8 * (size_t)chk[k], cbx, n);
                else rec_load(A.lrec + 8 * (size_t)A.leaf_of[(uint32_t)~chk[k] >> 3], cbx, n);
                b = dbox_union(b, cbx);
            }
            rec_store(A.wrec + 8 * (size_t)w, b, 0);
            w = up >> 2;
            sl = up & 3u;
        }
    }
    // the binary tree: each node whose children have all arrived (the holder writes
    // the leaf's slot from its record)
    uint32_t x = lf.x >> 1;
    for (;;) {
        float* X = A.bin + 16 * (size_t)x;
        int32_t k[2];
        kids_plain(X, k);   // unchanged until this node is rebuilt (by the last arrival)
        const uint32_t need = (k[0] != kSent) + (k[1] != kSent);
        if (!arrive(A.cnt, x, need)) return;
        const DBox xb = rebuild_node(A, x, k);
        const int32_t p = __float_as_int(X[14]);
        if (p < 0) {   // the root: m_sLocalBox = BVHNodeData::getBox, both slots
            for (int q = 0; q < 3; q++) { A.mesh_box[q] = xb.lo[q]; A.mesh_box[3 + q] = xb.hi[q]; }
            return;
        }
        x = (uint32_t)p >> 2;
    }
}

__global__ __launch_bounds__(kAB) void inst_box_kernel(const ctl_node* __restrict__ nodes, const float4* __restrict__ xf,
                                                      uint32_t n, const float* __restrict__ mesh_boxes, float* out) {
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= n) return;
    const float* mb = mesh_boxes + 6 * nodes[i].mesh_index;
    const float4* r = xf + 4 * i;
    m44 m;
    for (int k = 0; k < 4; k++) { m.d[4 * k] = r[k].x; m.d[4 * k + 1] = r[k].y; m.d[4 * k + 2] = r[k].z; m.d[4 * k + 3] = r[k].w; }
    instance_box(m, mb, mb + 3, out + 6 * i, out + 6 * i + 3);
}

// scene box = union of the instance boxes; eps = 1e-4 * |size| (DynamicScene.cpp:587);
// the environment light's scene sphere follows the box (UpdateScene re-runs
// InfiniteLight::Update, DynamicScene.cpp:540-542, Light.h:316-323)
__global__ void scene_eps_kernel(const float* inst, uint32_t n, float* out, ctl_env_light* env, const float* mesh_boxes,
                                 uint32_t n_meshes) {
    float lo[3], hi[3];
    box_empty(lo, hi);
    for (uint32_t i = 0; i < n; i++) box_extend(lo, hi, inst + 6 * i, inst + 6 * i + 3);
    for (int k = 0; k < 3; k++) { out[k] = lo[k]; out[3 + k] = hi[k]; }
    const f3 size = mk3(hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]);
    out[6] = 1e-4f * length(size);
    cull_bound(lo, hi, mesh_boxes, n_meshes, out + 7);   // DevScene::cull_m of the moved scene
    if (env) {
        const f3 l = mk3(lo[0], lo[1], lo[2]), h = mk3(hi[0], hi[1], hi[2]);
        const f3 c = (l + h) * 0.5f;   // AABB::Center
        env->scene_center[0] = c.x; env->scene_center[1] = c.y; env->scene_center[2] = c.z;
        env->scene_radius = length(h - l) / 1.5f;
    }
}

// DynamicScene::SetNodeTransform -> RecomputeShape (DynamicScene.cpp:433-443,
// ShapeSet.cpp:39-57): the ShapeSet of every diffuse light on `node`, one thread
// per light, its triangles in order (the area CDF is a sequential sum).
__global__ void light_recalc_kernel(ctl_light* lights, uint32_t n_lights, ctl_light_tri* tris, float* cdf,
                                    const float4* __restrict__ woop, const ctl_triangle_data* __restrict__ td,
                                    const float4* __restrict__ xf, uint32_t node) {
    const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n_lights) return;
    ctl_light& L = lights[li];
    if (L.kind != CTL_LIGHT_DIFFUSE || L.node_idx != node) return;
    m44 m;
    for (int k = 0; k < 4; k++) {
        const float4 r = xf[4 * node + k];
        m.d[4 * k] = r.x; m.d[4 * k + 1] = r.y; m.d[4 * k + 2] = r.z; m.d[4 * k + 3] = r.w;
    }
    for (uint32_t i = 0; i < L.tri_count; i++) {
        ctl_light_tri& t = tris[L.tri_first + i];
        const float4* w4 = woop + 3 * (size_t)t.i_dat;
        float w[12];
        for (int k = 0; k < 3; k++) { const float4 q = w4[k]; w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w; }
        light_tri_recalc(w, td[t.t_dat], m, t);
    }
    L.sum_area = shapeset_cdf(tris + L.tri_first, L.tri_count, cdf + L.cdf_first);
}

template <class T>
bool anim_alloc(AnimState* A, T** p, size_t n) {
    if (hipMalloc((void**)p, n * sizeof(T) + 64) != hipSuccess) return false;
    A->allocs.push_back((void*)*p);
    return true;
}

template <class T>
bool anim_upload(AnimState* A, T** dst, const T* src, size_t n) {
    if (!anim_alloc(A, dst, n)) return false;
    return n == 0 || hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
}

// The rebuild plan of a mesh tree (the compiled tree the upload put on the
// device): its leaves with the slots that hold them, the objects under every
// node, and the 4-wide copy's parent links and leaf slots.
bool plan_mesh(AnimState* A, MeshRebuild& R, const ctl_bvh_node* nodes, uint32_t n_nodes, uint32_t n_entries,
               const uint32_t* idx, const WideNode* wn, uint32_t n_wide, std::string& err) {
    R.n_nodes = n_nodes;
    if (n_nodes == 0) { err = "rebuild plan: empty tree"; return false; }
    std::vector<uint4> leaves;
    std::vector<int32_t> objects(n_nodes, 0);
    std::vector<uint8_t> seen(n_entries, 0), node_seen(n_nodes, 0);
    // pre-order from the root, then the objects children first
    std::vector<uint32_t> pre, st{0};
    node_seen[0] = 1;
    while (!st.empty()) {
        const uint32_t k = st.back();
        st.pop_back();
        pre.push_back(k);
        for (int c = 0; c < 2; c++) {
            const int32_t v = rb_kid(nodes[k], c);
            if (v == kSent) continue;
            if (v >= 0) {
                const uint32_t ch = (uint32_t)v >> 2;
                if (ch >= n_nodes || node_seen[ch] || rb_parent(nodes[ch]) != (int32_t)(k << 2)) {
                    err = "rebuild plan: malformed tree (child range, repeat or parent word)";
                    return false;
                }
                node_seen[ch] = 1;
                st.push_back(ch);
                continue;
            }
            uint32_t e = (uint32_t)~v;
            for (;; e++) {
                if (e >= n_entries || seen[e]) { err = "rebuild plan: a leaf's entries overrun or overlap"; return false; }
                seen[e] = 1;
                if (idx[e] & 1) break;
            }
            leaves.push_back(make_uint4(k << 1 | (uint32_t)c, (uint32_t)~v, e + 1 - (uint32_t)~v, 0xffffffffu));
        }
    }
    if (rb_parent(nodes[0]) >= 0) { err = "rebuild plan: the root has a parent word"; return false; }
    if (std::find(seen.begin(), seen.end(), 0) != seen.end()) { err = "rebuild plan: an entry lies in no leaf"; return false; }
    for (size_t i = pre.size(); i-- > 0;) {
        const uint32_t k = pre[i];
        for (int c = 0; c < 2; c++) {
            const int32_t v = rb_kid(nodes[k], c);
            if (v == kSent) continue;
            if (v >= 0) objects[k] += objects[(uint32_t)v >> 2];
            else for (uint32_t e = (uint32_t)~v;; e++) { objects[k]++; if (idx[e] & 1) break; }
        }
    }
    // node records: the box is written when the node is rebuilt, the objects persist
    std::vector<float> nrec(8ull * n_nodes, 0.0f);
    for (uint32_t k = 0; k < n_nodes; k++) std::memcpy(&nrec[8ull * k + 6], &objects[k], 4);
    std::sort(leaves.begin(), leaves.end(), [](uint4 a, uint4 b) { return a.y < b.y; });
    std::vector<uint32_t> leaf_of(n_entries, 0xffffffffu);
    for (size_t i = 0; i < leaves.size(); i++) leaf_of[leaves[i].y] = (uint32_t)i;
    // the 4-wide copy: every leaf slot is one binary leaf (counted: first entry << 3 | count)
    std::vector<uint32_t> wup(n_wide, 0xffffffffu);
    if (n_wide) {
        std::vector<uint32_t> wide_leaf(n_entries, 0xffffffffu);
        for (uint32_t i = 0; i < n_wide; i++)
            for (int q = 0; q < 4; q++) {
                const int32_t v = wn[i].child[q];
                if (v == kSent) continue;
                if (v >= 0) {
                    if ((uint32_t)v >= n_wide || wup[v] != 0xffffffffu) { err = "rebuild plan: malformed 4-wide tree"; return false; }
                    wup[v] = i << 2 | (uint32_t)q;
                } else {
                    const uint32_t first = (uint32_t)~v >> 3;
                    if (first >= n_entries || leaf_of[first] == 0xffffffffu) {
                        err = "rebuild plan: a 4-wide leaf is no binary leaf";
                        return false;
                    }
                    wide_leaf[first] = i << 2 | (uint32_t)q;
                }
            }
        for (uint4& l : leaves) {
            l.w = wide_leaf[l.y];
            if (l.w == 0xffffffffu) { err = "rebuild plan: a binary leaf is in no 4-wide leaf slot"; return false; }
        }
    }
    R.n_leaf = (uint32_t)leaves.size();
    R.n_wide = n_wide;
    if (!anim_upload(A, &R.d_leaf, leaves.data(), leaves.size()) ||
        !anim_upload(A, &R.d_leaf_of, leaf_of.data(), leaf_of.size()) ||
        !anim_upload(A, &R.d_nrec, nrec.data(), nrec.size()) || !anim_alloc(A, &R.d_cnt, n_nodes) ||
        !anim_alloc(A, &R.d_lrec, 8 * std::max<size_t>(1, leaves.size())) ||
        (n_wide && !anim_alloc(A, &R.d_wrec, 8ull * n_wide)) ||
        hipMemset(R.d_cnt, 0, n_nodes * sizeof(uint32_t)) != hipSuccess ||
        (n_wide && (!anim_upload(A, &R.d_wup, wup.data(), wup.size()) || !anim_alloc(A, &R.d_wcnt, n_wide) ||
                    hipMemset(R.d_wcnt, 0, n_wide * sizeof(uint32_t)) != hipSuccess))) {
        err = "rebuild plan: upload failed";
        return false;
    }
    return true;
}

// The instance tree along the moved instances' paths (host/bvh_rebuild.h), its
// 4-wide copy refit in its topology, both uploaded; inst = 6 floats per node.
bool rebuild_scene(AnimState* A, DevScene& S, const float* inst, const std::vector<uint32_t>& moved, hipStream_t s) {
    SceneTrees& T = A->scene;
    if (T.root < 0 || T.bin.empty()) return true;
    auto hit = [&](int32_t v) { return std::find(moved.begin(), moved.end(), (uint32_t)~v) != moved.end(); };
    const std::vector<uint8_t> flag = flag_paths(T.bin.data(), T.bin.size(), hit);
    auto leaf_box = [&](int32_t v) {
        const float* b = inst + 6 * (size_t)(uint32_t)~v;
        return RbBox{{b[0], b[1], b[2]}, {b[3], b[4], b[5]}};
    };
    auto one = [](int32_t) { return 1; };
    auto R = make_tree_rebuild(T.bin.data(), leaf_box, one, &flag);
    R.run(T.root, T.bin.size());
    if (hipMemcpyAsync(const_cast<float4*>(S.scene_bvh), T.bin.data(), T.bin.size() * sizeof(ctl_bvh_node),
                       hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (S.wide && !T.wide.empty()) {
        for (uint32_t i : T.wide_post) {
            WideNode& w = T.wide[i];
            for (int q = 0; q < 4; q++) {
                const int32_t v = w.child[q];
                if (v == kSent) continue;
                RbBox b;
                if (v < 0) {
                    b = leaf_box(v);
                } else {
                    const WideNode& ch = T.wide[(uint32_t)v];
                    b = rb_identity();
                    for (int k = 0; k < 4; k++)
                        if (ch.child[k] != kSent)
                            b = rb_union(b, RbBox{{ch.lo_x[k], ch.lo_y[k], ch.lo_z[k]}, {ch.hi_x[k], ch.hi_y[k], ch.hi_z[k]}});
                }
                w.lo_x[q] = b.lo[0]; w.lo_y[q] = b.lo[1]; w.lo_z[q] = b.lo[2];
                w.hi_x[q] = b.hi[0]; w.hi_y[q] = b.hi[1]; w.hi_z[q] = b.hi[2];
            }
        }
        if (hipMemcpyAsync(const_cast<float4*>(S.scene_wbvh), T.wide.data(), T.wide.size() * sizeof(WideNode),
                           hipMemcpyHostToDevice, s) != hipSuccess)
            return false;
    }
    return hipStreamSynchronize(s) == hipSuccess;   // the host trees are read by the copies
}

// Instance boxes and the scene box / epsilon on the device (inst_box_kernel,
// scene_eps_kernel), read back with the instance boxes for the host rebuild of
// the instance tree.
ctl_status scene_after_move(ctl_ctx* c, const std::vector<uint32_t>& moved, hipStream_t s, const char* what) {
    AnimState* A = c->anim;
    c->scene_epoch++;
    DevScene& S = c->scene;
    hipLaunchKernelGGL(inst_box_kernel, dim3((A->n_nodes + kAB - 1) / kAB), dim3(kAB), 0, s, S.nodes, S.xf, A->n_nodes,
                       A->d_mesh_boxes, A->d_inst_boxes);
    hipLaunchKernelGGL(scene_eps_kernel, dim3(1), dim3(1), 0, s, A->d_inst_boxes, A->n_nodes, A->d_eps,
                       const_cast<ctl_env_light*>(S.env), A->d_mesh_boxes, A->n_meshes);
    if (hipGetLastError() != hipSuccess) { c->err = std::string(what) + ": launch failed"; return CTL_ERR_HIP; }
    if (hipMemcpyAsync(A->h_eps, A->d_eps, 10 * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(A->h_eps + 10, A->d_inst_boxes, 6 * sizeof(float) * A->n_nodes, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        c->err = std::string(what) + ": readback failed";
        return CTL_ERR_HIP;
    }
    if (!rebuild_scene(A, S, A->h_eps + 10, moved, s)) {
        c->err = std::string(what) + ": instance tree upload failed";
        return CTL_ERR_HIP;
    }
    S.ray_eps = A->h_eps[6];
    for (int k = 0; k < 3; k++) S.cull_m[k] = A->h_eps[7 + k];
    c->device_eps = true;
    c->device_edited = true;
    return CTL_OK;
}

}  // namespace

void anim_free(ctl_ctx* c) {
    AnimState* A = c->anim;
    if (!A) return;
    for (void* p : A->allocs) (void)hipFree(p);
    if (A->h_eps) (void)hipHostFree(A->h_eps);
    delete A;
    c->anim = nullptr;
}

// Called by ctl_scene_upload once the scene arrays are on the device.
// wn / wbase / sw: the 4-wide trees built on upload (empty for binary scenes).
int anim_setup(ctl_ctx* c, const ctl_scene_desc* d, const std::vector<WideNode>& wn,
               const std::vector<uint32_t>& wbase, const std::vector<WideNode>& sw) {
    anim_free(c);
    if (!d->mesh_boxes) return CTL_OK;
    c->anim = new AnimState();
    AnimState* A = c->anim;
    std::string err;
    auto fail = [&](const std::string& m) { c->err = "scene_upload: " + m; anim_free(c); return (int)CTL_ERR_INVALID; };
    A->n_meshes = d->n_meshes;
    A->n_nodes = d->n_nodes;
    for (uint32_t i = 0; i < d->n_nodes; i++) A->node_mesh.push_back(d->nodes[i].mesh_index);
    if (!anim_upload(A, &A->d_mesh_boxes, d->mesh_boxes, 6ull * d->n_meshes) ||
        !anim_alloc(A, &A->d_inst_boxes, 6ull * std::max(1u, d->n_nodes)) || !anim_alloc(A, &A->d_eps, 10) ||
        hipHostMalloc((void**)&A->h_eps, (10 + 6ull * std::max(1u, d->n_nodes)) * sizeof(float), hipHostMallocDefault) !=
            hipSuccess)
        return fail("animation state allocation failed");
    // the instance trees' host copies (ctl_scene_set_transform / animate rebuild them)
    if (d->n_nodes > 0 && d->scene_start_node >= 0 && d->n_scene_bvh_nodes > 0) {
        SceneTrees& T = A->scene;
        T.bin.assign(d->scene_bvh_nodes, d->scene_bvh_nodes + d->n_scene_bvh_nodes);
        T.root = d->scene_start_node;
        T.wide = sw;
        // children before parents: reverse pre-order from node 0
        std::vector<uint32_t> st;
        if (!T.wide.empty()) st.push_back(0);
        while (!st.empty()) {
            const uint32_t k = st.back();
            st.pop_back();
            T.wide_post.push_back(k);
            for (int q = 0; q < 4; q++) {
                const int32_t v = T.wide[k].child[q];
                if (v >= 0 && v != kSent) {
                    if ((size_t)v >= T.wide.size() || T.wide_post.size() > T.wide.size()) return fail("malformed instance 4-wide tree");
                    st.push_back((uint32_t)v);
                }
            }
        }
        std::reverse(T.wide_post.begin(), T.wide_post.end());
    }
    if (d->n_anim_meshes == 0) return CTL_OK;
    if (!anim_upload(A, (ctl_anim_vertex**)&A->d_verts, d->anim_vertices, d->n_anim_vertices) ||
        !anim_upload(A, (uint32_t**)&A->d_tris, d->anim_triangles, 3ull * d->n_anim_triangles))
        return fail("animation upload failed");
    const bool wide = !wn.empty();
    size_t tmp = 0;
    for (uint32_t a = 0; a < d->n_anim_meshes; a++) {
        AnimMeshPlan P;
        P.am = d->anim_meshes[a];
        if (P.am.mesh >= d->n_meshes) return fail("animated mesh index out of range");
        if ((uint64_t)P.am.vertex_first + P.am.vertex_count > d->n_anim_vertices ||
            (uint64_t)P.am.tri_first + P.am.tri_count > d->n_anim_triangles)
            return fail("animated mesh ranges out of range");
        P.km = d->meshes[P.am.mesh];
        const bool last = P.am.mesh + 1 == d->n_meshes;
        const uint64_t n0 = P.km.bvh_node_offset / 4;
        const uint64_t n1 = last ? d->n_bvh_nodes : d->meshes[P.am.mesh + 1].bvh_node_offset / 4;
        const uint64_t e0 = P.km.bvh_indices_offset;
        const uint64_t e1 = last ? d->n_tri_indices : d->meshes[P.am.mesh + 1].bvh_indices_offset;
        const uint64_t t1 = last ? d->n_tri_data : d->meshes[P.am.mesh + 1].triangle_offset;
        if (n1 <= n0 || e1 < e0 || t1 - P.km.triangle_offset != P.am.tri_count || P.km.bvh_triangle_offset != 3 * e0)
            return fail("animated mesh does not match its compiled arrays");
        for (uint64_t i = 0; i < 3ull * P.am.tri_count; i++)
            if (d->anim_triangles[3ull * P.am.tri_first + i] >= P.am.vertex_count) return fail("animated vertex index out of range");
        for (uint64_t e = e0; e < e1; e++)
            if ((d->tri_indices[e] >> 1) >= P.am.tri_count) return fail("animated mesh entry out of range");
        P.n_entries = (uint32_t)(e1 - e0);
        uint32_t wb = 0, we = 0;
        if (wide) {
            wb = wbase[P.am.mesh];
            we = P.am.mesh + 1 < wbase.size() ? wbase[P.am.mesh + 1] : (uint32_t)wn.size();
        }
        P.wide_base = wb;
        if (!plan_mesh(A, P.rb, d->bvh_nodes + n0, (uint32_t)(n1 - n0), P.n_entries, d->tri_indices + e0,
                       wide ? wn.data() + wb : nullptr, we - wb, err))
            return fail(err);
        tmp = std::max<size_t>(tmp, P.am.vertex_count);
        A->meshes.push_back(std::move(P));
    }
    if (!anim_alloc(A, &A->d_P, tmp) || !anim_alloc(A, &A->d_N, tmp))
        return fail("animation buffers allocation failed");
    A->tmp_cap = tmp;
    return CTL_OK;
}

}  // namespace ctl

using namespace ctl;

extern "C" {

CTL_API ctl_status ctl_scene_animate(ctl_ctx* c, uint32_t anim, const ctl_float4x4* frame0, const ctl_float4x4* frame1,
                                     uint32_t n_bones, float lerp, void* stream) {
    if (!c || !frame0 || !frame1 || n_bones == 0) return CTL_ERR_INVALID;
    if (!c->has_scene || !c->anim) { c->err = "scene_animate: no scene uploaded"; return CTL_ERR_STATE; }
    AnimState* A = c->anim;
    if (anim >= A->meshes.size()) { c->err = "scene_animate: animated mesh index out of range"; return CTL_ERR_INVALID; }
    const AnimMeshPlan& P = A->meshes[anim];
    if (P.am.max_bone >= n_bones) { c->err = "scene_animate: a vertex uses a bone index >= n_bones"; return CTL_ERR_INVALID; }
    if (n_bones > 256) { c->err = "scene_animate: more than 256 bones (bone indices are 8-bit)"; return CTL_ERR_INVALID; }
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "scene_animate: hipSetDevice failed"; return CTL_ERR_HIP; }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t nb = 16ull * n_bones;
    if (A->bones_cap < nb) {
        if (hipStreamSynchronize(s) != hipSuccess) { c->err = "scene_animate: sync failed"; return CTL_ERR_HIP; }
        if (!anim_alloc(A, &A->d_bones[0], nb) || !anim_alloc(A, &A->d_bones[1], nb)) {
            c->err = "scene_animate: bone buffer allocation failed";
            return CTL_ERR_NOMEM;
        }
        A->bones_cap = nb;
    }
    if (hipMemcpyAsync(A->d_bones[0], frame0, nb * sizeof(float), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(A->d_bones[1], frame1, nb * sizeof(float), hipMemcpyHostToDevice, s) != hipSuccess) {
        c->err = "scene_animate: bone upload failed";
        return CTL_ERR_HIP;
    }
    DevScene& S = c->scene;
    c->scene_epoch++;   // the geometry moves (render-ahead passes are dropped)
    const uint32_t nv = P.am.vertex_count, nt = P.am.tri_count;
    const uint32_t* tris = A->d_tris + 3ull * P.am.tri_first;
    if (nv) hipLaunchKernelGGL(anim_skin_kernel, dim3((nv + kAB - 1) / kAB), dim3(kAB), 34 * n_bones * sizeof(float), s,
                               A->d_verts + P.am.vertex_first, nv, A->d_bones[0], A->d_bones[1], n_bones, lerp, A->d_P,
                               A->d_N);
    if (nt) hipLaunchKernelGGL(anim_tri_kernel, dim3((nt + kAB - 1) / kAB), dim3(kAB), 0, s, tris, nt, A->d_P, A->d_N,
                               const_cast<ctl_triangle_data*>(S.tri_data) + P.km.triangle_offset);
    if (P.rb.n_leaf) {
        RebuildArgs R;
        R.bin = reinterpret_cast<float*>(const_cast<float4*>(S.bvh)) + 4ull * P.km.bvh_node_offset;
        R.wide = S.wide && P.rb.n_wide ? reinterpret_cast<WideNode*>(const_cast<float4*>(S.wbvh)) + P.wide_base : nullptr;
        R.idx = S.tri_idx + P.km.bvh_indices_offset;
        R.tris = tris;
        R.P = A->d_P;
        R.woop = const_cast<float4*>(S.woop) + P.km.bvh_triangle_offset;
        R.leaf = P.rb.d_leaf;
        R.leaf_of = P.rb.d_leaf_of;
        R.nrec = P.rb.d_nrec;
        R.lrec = P.rb.d_lrec;
        R.wrec = P.rb.d_wrec;
        R.cnt = P.rb.d_cnt;
        R.wup = P.rb.d_wup;
        R.wcnt = P.rb.d_wcnt;
        R.mesh_box = A->d_mesh_boxes + 6 * P.am.mesh;
        R.n_leaf = P.rb.n_leaf;
        hipLaunchKernelGGL(anim_rebuild_kernel, dim3((P.rb.n_leaf + kAB - 1) / kAB), dim3(kAB), 0, s, R);
    }
    if (hipGetLastError() != hipSuccess) { c->err = "scene_animate: launch failed"; return CTL_ERR_HIP; }
    // instances of the mesh, the instance tree, epsilon (DynamicScene::AnimateMesh invalidates the node)
    if (A->n_nodes) {
        std::vector<uint32_t> moved;
        for (uint32_t i = 0; i < A->n_nodes; i++)
            if (A->node_mesh[i] == P.am.mesh) moved.push_back(i);
        const ctl_status r = scene_after_move(c, moved, s, "scene_animate");
        if (r != CTL_OK) return r;
    }
    c->device_edited = true;
    return CTL_OK;
}

CTL_API ctl_status ctl_scene_set_transform(ctl_ctx* c, uint32_t node, const ctl_float4x4* xf, void* stream) {
    if (!c || !xf) return CTL_ERR_INVALID;
    if (!c->has_scene || !c->anim) { c->err = "scene_set_transform: no scene uploaded"; return CTL_ERR_STATE; }
    AnimState* A = c->anim;
    DevScene& S = c->scene;
    if (node >= S.n_nodes) { c->err = "scene_set_transform: node index out of range"; return CTL_ERR_INVALID; }
    if (S.wide && S.quant && A->scene.root >= 0) {
        c->err = "scene_set_transform: 64-B quantized trees are not refit (upload without CTL_SCENE_WIDE_QUANT)";
        return CTL_ERR_STATE;
    }
    for (int k = 0; k < 16; k++)
        if (!std::isfinite(xf->m[k])) { c->err = "scene_set_transform: non-finite transform"; return CTL_ERR_INVALID; }
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "scene_set_transform: hipSetDevice failed"; return CTL_ERR_HIP; }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // SceneBVH::setTransform (SceneBVH.cpp:77-89): the matrix and its inverse, on the host
    m44 M;
    std::memcpy(M.d, xf->m, 64);
    const m44 inv = inverse(M);
    float* dxf = reinterpret_cast<float*>(const_cast<float4*>(S.xf)) + 16 * (size_t)node;
    float* dixf = reinterpret_cast<float*>(const_cast<float4*>(S.inv_xf)) + 16 * (size_t)node;
    if (hipMemcpyAsync(dxf, M.d, 64, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dixf, inv.d, 64, hipMemcpyHostToDevice, s) != hipSuccess) {
        c->err = "scene_set_transform: transform upload failed";
        return CTL_ERR_HIP;
    }
    if (S.n_lights)
        hipLaunchKernelGGL(light_recalc_kernel, dim3(1), dim3(64), 0, s, const_cast<ctl_light*>(S.lights), S.n_lights,
                           const_cast<ctl_light_tri*>(S.light_tris), const_cast<float*>(S.light_tri_cdf), S.woop,
                           S.tri_data, S.xf, node);
    return scene_after_move(c, std::vector<uint32_t>{node}, s, "scene_set_transform");
}

CTL_API ctl_status ctl_scene_read(ctl_ctx* c, uint32_t array, uint64_t first, uint64_t count, void* dst) {
    if (!c || (!dst && count)) return CTL_ERR_INVALID;
    if (!c->has_scene && array != CTL_ARRAY_SAMPLES_1D && array != CTL_ARRAY_SAMPLES_2D) {
        c->err = "scene_read: no scene uploaded";
        return CTL_ERR_STATE;
    }
    const DevScene& S = c->scene;
    const void* src = nullptr;
    size_t elem = 0;
    uint64_t n = 0;
    switch (array) {
        case CTL_ARRAY_TRI_DATA: src = S.tri_data; elem = sizeof(ctl_triangle_data); n = c->n_tri_data; break;
        case CTL_ARRAY_WOOP: src = S.woop; elem = sizeof(ctl_woop_tri); n = c->n_woop; break;
        case CTL_ARRAY_BVH_NODES: src = S.bvh; elem = sizeof(ctl_bvh_node); n = c->n_bvh_nodes; break;
        case CTL_ARRAY_SCENE_BVH: src = S.scene_bvh; elem = sizeof(ctl_bvh_node); n = c->n_scene_bvh; break;
        case CTL_ARRAY_MESH_BOXES:
            if (!c->anim) { c->err = "scene_read: the scene had no mesh boxes"; return CTL_ERR_STATE; }
            src = c->anim->d_mesh_boxes; elem = 6 * sizeof(float); n = c->anim->n_meshes; break;
        case CTL_ARRAY_RAY_EPS:
            if (first != 0 || count > 1) { c->err = "scene_read: ray eps is one value"; return CTL_ERR_INVALID; }
            if (count) memcpy(dst, &S.ray_eps, sizeof(float));
            return CTL_OK;
        case CTL_ARRAY_SAMPLES_1D:
        case CTL_ARRAY_SAMPLES_2D:
            if (c->active < 0) { c->err = "scene_read: no sampler tables (call ctl_sampler_generate)"; return CTL_ERR_STATE; }
            if (array == CTL_ARRAY_SAMPLES_1D) { src = c->d_s1[c->active]; elem = sizeof(float); }
            else { src = c->d_s2[c->active]; elem = sizeof(float2); }
            n = (uint64_t)c->nseq * c->len;
            break;
        case CTL_ARRAY_NODE_XF: src = S.xf; elem = sizeof(ctl_float4x4); n = S.n_nodes; break;
        case CTL_ARRAY_NODE_INV_XF: src = S.inv_xf; elem = sizeof(ctl_float4x4); n = S.n_nodes; break;
        case CTL_ARRAY_LIGHTS: src = S.lights; elem = sizeof(ctl_light); n = c->sarr[SA_LIGHTS].bytes / elem; break;
        case CTL_ARRAY_LIGHT_TRIS: src = S.light_tris; elem = sizeof(ctl_light_tri); n = c->sarr[SA_LTRIS].bytes / elem; break;
        case CTL_ARRAY_LIGHT_CDF: src = S.light_tri_cdf; elem = sizeof(float); n = c->sarr[SA_LCDF].bytes / elem; break;
        case CTL_ARRAY_SCENE_BOX:
            if (!c->anim || !c->device_eps) { c->err = "scene_read: the scene box is derived by set_transform / animate"; return CTL_ERR_STATE; }
            src = c->anim->d_eps; elem = 6 * sizeof(float); n = 1; break;
        case CTL_ARRAY_CULL_BOUND:
            if (first != 0 || count > 1) { c->err = "scene_read: the cull bound is one record of 3 floats"; return CTL_ERR_INVALID; }
            if (count) memcpy(dst, S.cull_m, 3 * sizeof(float));
            return CTL_OK;
        case CTL_ARRAY_ENV:
            if (!S.env) { c->err = "scene_read: no environment light"; return CTL_ERR_STATE; }
            src = S.env; elem = sizeof(ctl_env_light); n = 1; break;
        case CTL_ARRAY_WIDE_BVH:
        case CTL_ARRAY_SCENE_WIDE_BVH:
        case CTL_ARRAY_MESH_WIDE_BASE:
            if (!S.wide) { c->err = "scene_read: the scene has no 4-wide trees (CTL_SCENE_BINARY_BVH)"; return CTL_ERR_STATE; }
            elem = array == CTL_ARRAY_MESH_WIDE_BASE ? sizeof(uint32_t) : (S.quant ? sizeof(QWideNode) : sizeof(WideNode));
            src = array == CTL_ARRAY_WIDE_BVH ? (const void*)S.wbvh
                  : array == CTL_ARRAY_SCENE_WIDE_BVH ? (const void*)S.scene_wbvh : (const void*)S.mesh_wbase;
            n = c->sarr[array == CTL_ARRAY_WIDE_BVH ? SA_WBVH : array == CTL_ARRAY_SCENE_WIDE_BVH ? SA_SWBVH : SA_WBASE].bytes / elem;
            break;
        default: c->err = "scene_read: unknown array"; return CTL_ERR_INVALID;
    }
    if (first > n || count > n - first) { c->err = "scene_read: range out of bounds"; return CTL_ERR_INVALID; }
    if (!count) return CTL_OK;
    if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(dst, (const char*)src + first * elem, count * elem, hipMemcpyDeviceToHost) != hipSuccess) {
        c->err = "scene_read: copy failed";
        return CTL_ERR_HIP;
    }
    return CTL_OK;
}

}  // extern "C"

// anim.hip — animated (skinned) meshes on the device: AnimatedMesh::k_ComputeState
// (Engine/AnimatedMesh.cpp:163-184) as a chain of data-parallel kernels, and the
// instance tree after ctl_scene_animate / ctl_scene_set_transform.
//
//   skin     g_ComputeVertices (AnimatedMesh.cu:29-43): per vertex, two 8-bone
//            matrix blends, TransformPoint / TransformDirection, lerp
//   tris     g_ComputeTriangles -> TriangleData::setData (TriangleData.cu:35-63)
//   rebuild  the mesh tree as BVHRebuilder::Build(&p, true) leaves it
//            (AnimatedMesh.cpp:174-176, BVHRebuilder.cpp:281-340, 365-450): one
//            thread per leaf (or per pair of leaves under one node) writes its
//            entries' Woop data (AnimProvider::setObject, AnimatedMesh.cpp:
//            113-117) and the leaf's box record, then climbs: the last of a
//            node's children to arrive (an atomic counter per node) recomputes
//            the node -- the best of the four child/grandchild rotations by SAH
//            if strictly cheaper (host/bvh_rebuild.h states the rules), the
//            moved subtrees' child and parent words, the box records -- and
//            moves on to its parent, carrying the node's view (box, objects,
//            children and theirs) so that only the sibling's is read back.  A
//            node is recomputed after its whole subtree, as in the reference's
//            post-order recursion, and nodes of disjoint subtrees never touch
//            the same words, so the result is the recursion's.  The tree's
//            shape persists from frame to frame, as the reference's does.
//   slots    every node's two slots from its children's final records, and
//            each leaf's holder and pairing for the next frame (one launch)
//   4-wide   the 4-wide copy keeps the topology the upload collapsed and is
//            refit by height: one launch per height below the top, the top
//            (<= 2048 nodes) in one block through LDS.
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
    uint4* d_leaf = nullptr;            // {holder << 1 | slot, first entry, entries, pairing} (anim_rebuild_kernel)
    uint32_t* d_leaf_of = nullptr;      // per entry of the mesh: the record of the leaf starting there
    float* d_nrec = nullptr;            // per binary node: its box (6) and numLeafs (bvhNodeData), 32 B
    float* d_lrec = nullptr;            // per leaf: its box and entries, 32 B
    uint32_t* d_cnt = nullptr;          // arrival counters per binary node (even between launches)
    uint32_t n_wide = 0;                // 4-wide nodes of the mesh (0: binary scene)
    float* d_wrec = nullptr;            // per 4-wide node: its box, 32 B
    uint32_t* d_worder = nullptr;       // 4-wide nodes by height (children first)
    uint32_t* d_woff = nullptr;         // per height: its first entry of d_worder (and the end)
    std::vector<uint32_t> woff;         // the same on the host
    uint32_t wtop = 0;                  // the first height of the one-block top
    uint4* d_wcode = nullptr;           // per 4-wide node: its child codes (WideArgs)
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
// What one thread of the climb hands to another goes through 32-B records (box
// and objects) per binary node (nrec), written and read with the SC1 cache
// policy (buffer_load / buffer_store dwordx4 sc1: coherent across the XCDs' L2s
// access by access), 16 B per access.  Words two threads of the launch may
// write (a moved subtree's parent word, a rotated node's child words) are
// stored the same way, so the last writer wins whatever the XCDs' write-back
// order.  The leaf records (lrec) come from the leaf launch before and are read
// plain.  The climb writes no node slot and no leaf holder: a later launch
// (anim_slot_kernel) stores every node's two slots from its children's final
// records, plain and whole, and each leaf's holder and pairing, and the 4-wide
// copy is refit by height after that (anim_wide_kernel), all reading what the
// climb left after a launch boundary.  An acquire / release at agent scope
// would instead write back and invalidate the whole L2 at every arrival
// (buffer_wbl2 / buffer_inv sc1): the first version did, 7.85 ms per animate.
// The arrival orders the accesses: a thread's records complete (s_waitcnt
// vmcnt(0)) before its arrival increments the counter, and the last arriver's
// loads are issued after the counter's value came back.
// CTL_REBUILD_DIAG (timing-only builds, never shipped): 1 leaves out the climb,
// 2 drops SC1 from the shared records and every rotation (so no stale read can
// reach a child word), 3 drops the rotations
#ifndef CTL_REBUILD_DIAG
#define CTL_REBUILD_DIAG 0
#endif
constexpr int kSC1 = CTL_REBUILD_DIAG == 2 ? 0 : 16;   // cache-policy operand of the buffer intrinsics: SC1

struct Coh {               // buffer descriptors of the arrays the climb shares
    __amdgpu_buffer_rsrc_t bin, nrec;
};
__device__ __forceinline__ float4 cld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1));
}
__device__ __forceinline__ void cst4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
    using v4u = __attribute__((ext_vector_type(4))) unsigned int;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, off, 0, kSC1);
}
__device__ __forceinline__ void cld_kids(__amdgpu_buffer_rsrc_t bin, uint32_t node, int32_t k[2]) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(bin, node * 64u + 48u, 0, kSC1);
    k[0] = (int32_t)v[0];
    k[1] = (int32_t)v[1];
}
__device__ __forceinline__ void cst_kids(__amdgpu_buffer_rsrc_t bin, uint32_t node, int32_t a, int32_t b) {
    using v2u = __attribute__((ext_vector_type(2))) unsigned int;
    __builtin_amdgcn_raw_buffer_store_b64(v2u{(unsigned)a, (unsigned)b}, bin, node * 64u + 48u, 0, kSC1);
}

// BVHNodeData child slots (TriIntersectorData.h:44-88): {lo.x hi.x lo.y hi.y}
// per slot at 0 / 16 B, {lo.z hi.z} per slot at 32 / 40 B
__device__ __forceinline__ DBox slot_box(const float* nd, int c) {
    const float4 q = reinterpret_cast<const float4*>(nd)[c];
    const float2 z = reinterpret_cast<const float2*>(nd + 8)[c];
    return DBox{{q.x, q.z, z.x}, {q.y, q.w, z.y}};
}
// a node's child words as the last launch left them (the climb reads a node's
// own words before anything of this launch can have moved them)
__device__ __forceinline__ void kids_plain(const float* nd, int32_t k[2]) {
    const float2 v = reinterpret_cast<const float2*>(nd + 12)[0];
    k[0] = __float_as_int(v.x);
    k[1] = __float_as_int(v.y);
}

// A record: getBox and numLeafs (bvhNodeData), {lo xyz, hi.x} {hi.yz, objects, 0}
__device__ __forceinline__ void rec_unpack(float4 a, float4 c, DBox& b, int& n) {
    b = DBox{{a.x, a.y, a.z}, {a.w, c.x, c.y}};
    n = __float_as_int(c.z);
}
__device__ __forceinline__ void rec_store(__amdgpu_buffer_rsrc_t r, uint32_t i, const DBox& b, int n) {
    cst4(r, 32u * i, make_float4(b.lo[0], b.lo[1], b.lo[2], b.hi[0]));
    cst4(r, 32u * i + 16u, make_float4(b.hi[1], b.hi[2], __int_as_float(n), 0.0f));
}

struct RebuildArgs {
    float* bin;                 // the mesh tree's node 0
    const uint32_t* idx;        // the mesh's TriIntersectorData2 entries
    const uint32_t* tris;       // the mesh's triangles (skinned vertex indices)
    const float4* P;            // skinned positions
    float4* woop;               // the mesh's TriIntersectorData entries
    uint4* leaf;
    const uint32_t* leaf_of;
    float* nrec;                // per binary node {lo xyz, hi xyz, objects, 0}: written when the node is rebuilt
    float* lrec;                // per leaf record, the same: written by anim_leaf_kernel
    uint32_t* cnt;
    float* mesh_box;            // m_sLocalBox: 6 floats
    uint32_t n_leaf, n_nodes;
};

__device__ __forceinline__ Coh coh_of(const RebuildArgs& A) {
    return Coh{__builtin_amdgcn_make_buffer_rsrc(A.bin, 0, (int)(64u * A.n_nodes), 0x00020000),
               __builtin_amdgcn_make_buffer_rsrc(A.nrec, 0, (int)(32u * A.n_nodes), 0x00020000)};
}

// The last of `need` (1 or 2, fixed for a node: no rotation moves an empty
// slot) arrivals at counter k goes on.  Every launch adds `need` to the counter,
// so the last arrival is the one that makes it a multiple of `need`; nothing
// resets it.  The caller's coherent stores complete first.
__device__ __forceinline__ bool arrive(uint32_t* cnt, uint32_t k, uint32_t need) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(cnt + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::: "memory");   // no load of the arrivals' records is hoisted above the counter
    return need == 1 || (old & 1u) != 0;
}

// A finished subtree as its parent's recomputation reads it: getBox and numLeafs,
// and for an inner node its children with theirs.  The climbing thread carries
// the one it just finished; the sibling's comes from the records.
struct View {
    DBox b;
    int n;
    int32_t k[2];
    DBox kb[2];
    int kn[2];
};

// field-wise selects (a conditional over whole structs would select their
// addresses and put them in scratch)
__device__ __forceinline__ DBox bsel(bool a, const DBox& x, const DBox& y) {
    DBox r;
    for (int k = 0; k < 3; k++) { r.lo[k] = a ? x.lo[k] : y.lo[k]; r.hi[k] = a ? x.hi[k] : y.hi[k]; }
    return r;
}
__device__ __forceinline__ View vsel(bool a, const View& x, const View& y) {
    View r;
    r.b = bsel(a, x.b, y.b);
    r.n = a ? x.n : y.n;
    for (int j = 0; j < 2; j++) {
        r.k[j] = a ? x.k[j] : y.k[j];
        r.kb[j] = bsel(a, x.kb[j], y.kb[j]);
        r.kn[j] = a ? x.kn[j] : y.kn[j];
    }
    return r;
}

// getBox / numLeafs of child value v (AABB::Identity and 0 for an empty slot)
__device__ __forceinline__ void child_info(const RebuildArgs& A, const Coh& C, int32_t v, DBox& b, int& n) {
    if (v == kSent) { b = dbox_identity(); n = 0; return; }
    if (v < 0) {   // a leaf's record: from the leaf launch, plain
        const float4* r = reinterpret_cast<const float4*>(A.lrec + 8 * (size_t)A.leaf_of[(uint32_t)~v]);
        rec_unpack(r[0], r[1], b, n);
        return;
    }
    const uint32_t i = (uint32_t)v >> 2;
    rec_unpack(cld4(C.nrec, 32u * i), cld4(C.nrec, 32u * i + 16u), b, n);
}
__device__ __forceinline__ View load_view(const RebuildArgs& A, const Coh& C, int32_t v) {
    View w;
    child_info(A, C, v, w.b, w.n);
    w.k[0] = w.k[1] = kSent;
    if (v >= 0 && v != kSent) cld_kids(C.bin, (uint32_t)v >> 2, w.k);   // its own rotation may have moved them
    for (int j = 0; j < 2; j++) child_info(A, C, w.k[j], w.kb[j], w.kn[j]);
    return w;
}

// BVHRebuilder::setChild's parent word of a moved inner child (read by the
// next launch; a child can move twice in one launch).  A moved leaf's holder
// is written by anim_slot_kernel, which sees every leaf's final slot.
__device__ __forceinline__ void moved_to(const RebuildArgs& A, int32_t v, uint32_t node) {
    if (v < 0 || v == kSent) return;
    __hip_atomic_store(reinterpret_cast<int32_t*>(A.bin + 16 * (size_t)((uint32_t)v >> 2) + 14), (int32_t)(node << 2),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// recomputeNode (BVHRebuilder.cpp:281-340) of node x, its subtree done, with
// its children's views v[0], v[1].  Returns x's.
__device__ __forceinline__ View recompute_node(const RebuildArgs& A, const Coh& C, uint32_t x, const int32_t c[2],
                                               const View v[2]) {
    const float* X = A.bin + 16 * (size_t)x;
    bool can[2];
    for (int i = 0; i < 2; i++)
        can[i] = c[i] >= 0 && c[i] != kSent && v[i].k[0] != kSent && v[i].k[1] != kSent;   // numberGrandchildren == 2
    // sah(idx, child, grandchild) (:624-638) for the four rotations
    float rot[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    if (can[0]) {
        rot[0] = dbox_area(dbox_union(v[1].b, v[0].kb[1])) * (float)(v[1].n + v[0].kn[1]) + dbox_area(v[0].kb[0]) * (float)v[0].kn[0];
        rot[1] = dbox_area(dbox_union(v[1].b, v[0].kb[0])) * (float)(v[1].n + v[0].kn[0]) + dbox_area(v[0].kb[1]) * (float)v[0].kn[1];
    }
    if (can[1]) {
        rot[2] = dbox_area(dbox_union(v[0].b, v[1].kb[0])) * (float)(v[0].n + v[1].kn[0]) + dbox_area(v[1].kb[1]) * (float)v[1].kn[1];
        rot[3] = dbox_area(dbox_union(v[0].b, v[1].kb[1])) * (float)(v[0].n + v[1].kn[1]) + dbox_area(v[1].kb[0]) * (float)v[1].kn[0];
    }
    int best = 0;
    float bestv = rot[0];
    for (int i = 1; i < 4; i++)
        if (rot[i] < bestv) { best = i; bestv = rot[i]; }   // std::min_element: the first smallest
    const float now = dbox_area(v[0].b) * (float)v[0].n + dbox_area(v[1].b) * (float)v[1].n;
    View r;
    r.n = v[0].n + v[1].n;   // numLeafs(x): no rotation at x changes it
    if (!(bestv < now) || CTL_REBUILD_DIAG >= 2) {
        // getBox: both stored slots, an empty one as stored (both loaded, then
        // selected: a select of a load and a register became a scratch round trip)
        r.b = dbox_union(v[0].b, v[1].b);
        if (c[0] == kSent || c[1] == kSent) {
            const DBox s0 = slot_box(X, 0), s1 = slot_box(X, 1);
            r.b = dbox_union(bsel(c[0] == kSent, s0, v[0].b), bsel(c[1] == kSent, s1, v[1].b));
        }
        for (int i = 0; i < 2; i++) { r.k[i] = c[i]; r.kb[i] = v[i].b; r.kn[i] = v[i].n; }
        rec_store(C.nrec, x, r.b, r.n);
        return r;
    }
    // swapChildren(idx, lc, lg) (:691-702): child c[lc] and grandchild (c[o]'s lg) trade places
    const int lc = best < 2 ? 1 : 0, lg = (best == 1 || best == 2) ? 1 : 0;
    const View L = vsel(lc == 0, v[0], v[1]);   // the child pushed down
    const View O = vsel(lc == 0, v[1], v[0]);   // the other child
    const int32_t g = lg == 0 ? O.k[0] : O.k[1], og = lg == 0 ? O.k[1] : O.k[0];
    const DBox gb = bsel(lg == 0, O.kb[0], O.kb[1]), ogb = bsel(lg == 0, O.kb[1], O.kb[0]);
    const int gn = lg == 0 ? O.kn[0] : O.kn[1];
    const int32_t cl = lc == 0 ? c[0] : c[1], co = lc == 0 ? c[1] : c[0];
    const uint32_t other = (uint32_t)co >> 2;
    cst_kids(C.bin, other, lg == 0 ? cl : og, lg == 0 ? og : cl);
    moved_to(A, cl, other);
    // propagateBBChange(other -> x): the other child's box, its slots in order
    const DBox ob = bsel(lg == 0, dbox_union(L.b, ogb), dbox_union(ogb, L.b));
    const int on = O.n + L.n - gn;   // BVHNodeInfo::changeCount, net
    cst_kids(C.bin, x, lc == 0 ? g : co, lc == 0 ? co : g);
    moved_to(A, g, x);
    rec_store(C.nrec, other, ob, on);
    r.b = bsel(lc == 0, dbox_union(gb, ob), dbox_union(ob, gb));
    r.k[0] = lc == 0 ? g : co;   r.k[1] = lc == 0 ? co : g;
    r.kb[0] = bsel(lc == 0, gb, ob); r.kb[1] = bsel(lc == 0, ob, gb);
    r.kn[0] = lc == 0 ? gn : on; r.kn[1] = lc == 0 ? on : gn;
    rec_store(C.nrec, x, r.b, r.n);
    return r;
}

// The same, the thread having arrived from child slot `from` with that child's
// view; the sibling's comes from the records.
__device__ __forceinline__ View rebuild_node(const RebuildArgs& A, const Coh& C, uint32_t x, const int32_t c[2], int from,
                                             const View& me) {
    const View sib = load_view(A, C, from == 0 ? c[1] : c[0]);
    View v[2];
    v[0] = vsel(from == 0, me, sib);
    v[1] = vsel(from == 0, sib, me);
    return recompute_node(A, C, x, c, v);
}

// A leaf record: {holder << 1 | slot, first entry, entries, mode}; the mode
// (set by the plan, then by each launch's anim_slot_kernel for the next one)
// pairs the two leaves of a node whose children are both leaves: the one in
// slot 0 takes both and recomputes their node without an arrival, the other
// has nothing to do.
constexpr uint32_t kLeafSingle = 0xffffffffu, kLeafPartner = 0xfffffffeu;   // else: the partner's record

// A leaf's view: its record, written by anim_leaf_kernel (an earlier launch)
__device__ __forceinline__ View leaf_view(const RebuildArgs& A, uint32_t i) {
    View me;
    const float4* r = reinterpret_cast<const float4*>(A.lrec + 8 * (size_t)i);
    rec_unpack(r[0], r[1], me.b, me.n);
    me.k[0] = me.k[1] = kSent;
    me.kb[0] = me.kb[1] = dbox_identity();
    me.kn[0] = me.kn[1] = 0;
    return me;
}

// After node x: on to its parent (false at the root, whose box is m_sLocalBox =
// BVHNodeData::getBox, both slots).  The parent word is moved only by a
// rotation above x, which comes later.
__device__ __forceinline__ bool climb_up(const RebuildArgs& A, uint32_t& x, int32_t& prev, const View& me) {
    const int32_t p = __float_as_int(A.bin[16 * (size_t)x + 14]);
    if (p < 0) {
        for (int q = 0; q < 3; q++) { A.mesh_box[q] = me.b.lo[q]; A.mesh_box[3 + q] = me.b.hi[q]; }
        return false;
    }
    prev = (int32_t)(x << 2);
    x = (uint32_t)p >> 2;
    return true;
}

// One thread per leaf: AnimProvider::setObject (AnimatedMesh.cpp:113-117) for
// its entries, and its record: the box (its triangles' boxes extended from
// AABB::Identity) and the entries.
__global__ __launch_bounds__(kAB) void anim_leaf_kernel(RebuildArgs A) {
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
    float4* r = reinterpret_cast<float4*>(A.lrec + 8 * (size_t)i);
    r[0] = make_float4(lo[0], lo[1], lo[2], hi[0]);
    r[1] = make_float4(hi[1], hi[2], __int_as_float((int)lf.z), 0.0f);
}

// One thread per leaf (or leaf pair) whose record the leaf launch wrote, up the
// binary tree.  96 VGPRs, 5 waves per SIMD (the compiler's choice was 100 and 4).
__global__ __launch_bounds__(kAB) __attribute__((amdgpu_waves_per_eu(5))) void anim_rebuild_kernel(RebuildArgs A) {
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= A.n_leaf || CTL_REBUILD_DIAG == 1) return;
    const uint4 lf = A.leaf[i];
    if (lf.w == kLeafPartner) return;
    const Coh C = coh_of(A);
    View me = leaf_view(A, i);
    int32_t prev = (int32_t)~lf.y;   // the child value the thread comes from
    uint32_t x = lf.x >> 1;
    if (lf.w != kLeafSingle) {   // both children of x: no arrival, no records to read
        const uint4 pf = A.leaf[lf.w];
        View v[2];
        v[0] = me;
        v[1] = leaf_view(A, lf.w);
        const int32_t c[2] = {(int32_t)~lf.y, (int32_t)~pf.y};
        me = recompute_node(A, C, x, c, v);
        if (!climb_up(A, x, prev, me)) return;
    }
    // each node whose children have all arrived, recomputed by the last arrival
    for (;;) {
        int32_t k[2];
        kids_plain(A.bin + 16 * (size_t)x, k);   // unchanged until this node is rebuilt (by the last arrival)
        const uint32_t need = (k[0] != kSent) + (k[1] != kSent);
        if (!arrive(A.cnt, x, need)) return;
        me = rebuild_node(A, C, x, k, k[0] == prev ? 0 : 1, me);
        if (!climb_up(A, x, prev, me)) return;
    }
}

// node->setLeft / setRight for every node: its two slots from its children's
// final records (an empty slot keeps what it holds), three whole 16-B stores;
// and each leaf child's holder and pairing for the next launch.
__global__ __launch_bounds__(kAB) void anim_slot_kernel(float* bin, const float* nrec, const float* lrec,
                                                       const uint32_t* leaf_of, uint4* leaf, uint32_t n_nodes) {
    const uint32_t x = blockIdx.x * kAB + threadIdx.x;
    if (x >= n_nodes) return;
    float4* X = reinterpret_cast<float4*>(bin + 16 * (size_t)x);
    const int4 k4 = reinterpret_cast<const int4*>(X)[3];
    const int32_t k[2] = {k4.x, k4.y};
    float4 s[2] = {}, z = {};
    if (k[0] == kSent || k[1] == kSent) { s[0] = X[0]; s[1] = X[1]; z = X[2]; }
    float zz[4] = {z.x, z.y, z.z, z.w};
    uint32_t lr[2] = {kLeafSingle, kLeafSingle};
    for (int c = 0; c < 2; c++) {
        if (k[c] == kSent) continue;
        const bool lv = k[c] < 0;
        if (lv) lr[c] = leaf_of[(uint32_t)~k[c]];
        const float* r = lv ? lrec + 8 * (size_t)lr[c] : nrec + 8 * (size_t)((uint32_t)k[c] >> 2);
        const float4 a = reinterpret_cast<const float4*>(r)[0], b = reinterpret_cast<const float4*>(r)[1];
        s[c] = make_float4(a.x, a.w, a.y, b.x);   // {lo.x hi.x lo.y hi.y}
        zz[2 * c] = a.z;
        zz[2 * c + 1] = b.y;
    }
    X[0] = s[0];
    X[1] = s[1];
    X[2] = make_float4(zz[0], zz[1], zz[2], zz[3]);
    const bool pair = lr[0] != kLeafSingle && lr[1] != kLeafSingle;
    for (int c = 0; c < 2; c++) {
        if (lr[c] == kLeafSingle) continue;
        leaf[lr[c]].x = x << 1 | (uint32_t)c;
        leaf[lr[c]].w = !pair ? kLeafSingle : c == 0 ? lr[1] : kLeafPartner;
    }
}

// The 4-wide copy, refit in the topology the upload collapsed.  Per node, the
// plan's child codes: an empty slot 0xffffffff, a leaf its lrec record << 2 | 1,
// an inner child its node << 2 (its box in wrec) or, between nodes of the
// one-block top, its position there << 2 | 2 (its box in LDS).
struct WideArgs {
    WideNode* wide;
    float* wrec;               // per node: the union of its slots, for its parent
    const float* lrec;
    const uint4* code;
    const uint32_t* order;     // nodes by height, children first
};
constexpr uint32_t kNoChild = 0xffffffffu;
__device__ __forceinline__ DBox rec6(const float* base, uint32_t i) {
    const float4* r = reinterpret_cast<const float4*>(base + 8 * (size_t)i);
    const float4 a = r[0], c = r[1];
    return DBox{{a.x, a.y, a.z}, {a.w, c.x, c.y}};
}
// each occupied slot gets its child's box, an empty one keeps what it holds
// (whole 16-B stores: lo_x .. hi_z over the four slots); returns the union of
// the occupied slots in slot order
__device__ __forceinline__ DBox wide_write(WideNode* W, const uint32_t c[4], DBox cb[4]) {
    DBox b = dbox_identity();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (c[q] == kNoChild)
            cb[q] = DBox{{W->lo_x[q], W->lo_y[q], W->lo_z[q]}, {W->hi_x[q], W->hi_y[q], W->hi_z[q]}};
        else
            b = dbox_union(b, cb[q]);
    }
    float4* F = reinterpret_cast<float4*>(W);
    for (int k = 0; k < 3; k++) {
        F[2 * k] = make_float4(cb[0].lo[k], cb[1].lo[k], cb[2].lo[k], cb[3].lo[k]);
        F[2 * k + 1] = make_float4(cb[0].hi[k], cb[1].hi[k], cb[2].hi[k], cb[3].hi[k]);
    }
    return b;
}
// one height below the top (its children are lower: earlier launches)
__global__ __launch_bounds__(kAB) void anim_wide_kernel(WideArgs A, uint32_t first, uint32_t n) {
    const uint32_t j = blockIdx.x * kAB + threadIdx.x;
    if (j >= n) return;
    const uint32_t w = A.order[first + j];
    const uint4 cd = A.code[w];
    const uint32_t c[4] = {cd.x, cd.y, cd.z, cd.w};
    DBox cb[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (c[q] != kNoChild) cb[q] = rec6((c[q] & 1) ? A.lrec : A.wrec, c[q] >> 2);
    const DBox b = wide_write(A.wide + w, c, cb);
    float4* R = reinterpret_cast<float4*>(A.wrec + 8 * (size_t)w);
    R[0] = make_float4(b.lo[0], b.lo[1], b.lo[2], b.hi[0]);
    R[1] = make_float4(b.hi[1], b.hi[2], 0.0f, 0.0f);
}
// the top heights (at most kTopMax nodes), height after height in one block:
// their nodes and child codes staged in LDS first, their boxes handed up there
constexpr int kTopWide = 1024;
constexpr uint32_t kTopMax = 2048;
__global__ __launch_bounds__(kTopWide) void anim_wide_top_kernel(WideArgs A, const uint32_t* off, uint32_t n_heights) {
    __shared__ float box[6 * kTopMax];
    __shared__ uint4 code[kTopMax];
    __shared__ uint32_t node[kTopMax];
    const uint32_t base = off[0], n = off[n_heights] - base;
    for (uint32_t j = threadIdx.x; j < n; j += kTopWide) {
        node[j] = A.order[base + j];
        code[j] = A.code[node[j]];
    }
    __syncthreads();
    for (uint32_t h = 0; h < n_heights; h++) {
        for (uint32_t j = off[h] - base + threadIdx.x; j < off[h + 1] - base; j += kTopWide) {
            const uint4 cd = code[j];
            const uint32_t c[4] = {cd.x, cd.y, cd.z, cd.w};
            DBox cb[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (c[q] == kNoChild) continue;
                if ((c[q] & 3) == 2) {
                    const float* l = box + 6 * (c[q] >> 2);
                    cb[q] = DBox{{l[0], l[1], l[2]}, {l[3], l[4], l[5]}};
                } else {
                    cb[q] = rec6((c[q] & 1) ? A.lrec : A.wrec, c[q] >> 2);
                }
            }
            const DBox b = wide_write(A.wide + node[j], c, cb);
            float* l = box + 6 * j;
            for (int k = 0; k < 3; k++) { l[k] = b.lo[k]; l[3 + k] = b.hi[k]; }
        }
        __syncthreads();
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
// device): its leaves with the slots that hold them, and the 4-wide copy's
// nodes by height.
bool plan_mesh(AnimState* A, MeshRebuild& R, const ctl_bvh_node* nodes, uint32_t n_nodes, uint32_t n_entries,
               const uint32_t* idx, const WideNode* wn, uint32_t n_wide, std::string& err) {
    R.n_nodes = n_nodes;
    if (n_nodes == 0) { err = "rebuild plan: empty tree"; return false; }
    std::vector<uint4> leaves;
    std::vector<uint8_t> seen(n_entries, 0), node_seen(n_nodes, 0);
    // pre-order from the root: every node reached once, its parent word its parent
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
            leaves.push_back(make_uint4(k << 1 | (uint32_t)c, (uint32_t)~v, e + 1 - (uint32_t)~v, kLeafSingle));
        }
    }
    if (rb_parent(nodes[0]) >= 0) { err = "rebuild plan: the root has a parent word"; return false; }
    if (std::find(seen.begin(), seen.end(), 0) != seen.end()) { err = "rebuild plan: an entry lies in no leaf"; return false; }
    if (64ull * n_nodes > 0xffffffffull) { err = "rebuild plan: a mesh tree of more than 64 M nodes"; return false; }
    std::sort(leaves.begin(), leaves.end(), [](uint4 a, uint4 b) { return a.y < b.y; });
    std::vector<uint32_t> leaf_of(n_entries, 0xffffffffu);
    for (size_t i = 0; i < leaves.size(); i++) leaf_of[leaves[i].y] = (uint32_t)i;
    for (uint4& l : leaves) l.w = kLeafSingle;
    for (uint32_t k = 0; k < n_nodes; k++) {   // a node's two leaf children: the pairing of anim_slot_kernel
        const int32_t a = rb_kid(nodes[k], 0), b = rb_kid(nodes[k], 1);
        if (a >= 0 || b >= 0 || a == kSent || b == kSent || !node_seen[k]) continue;
        leaves[leaf_of[(uint32_t)~a]].w = leaf_of[(uint32_t)~b];
        leaves[leaf_of[(uint32_t)~b]].w = kLeafPartner;
    }
    // the 4-wide copy: every leaf slot is one binary leaf (counted: first entry << 3 | count),
    // every node but the root one node's child; its nodes ordered by height
    std::vector<uint32_t> worder;
    std::vector<uint4> wcode;
    R.woff.clear();
    if (n_wide) {
        std::vector<uint32_t> up(n_wide, 0xffffffffu), height(n_wide, 0);
        std::vector<uint8_t> wleaf(n_entries, 0);
        for (uint32_t i = 0; i < n_wide; i++)
            for (int q = 0; q < 4; q++) {
                const int32_t v = wn[i].child[q];
                if (v == kSent) continue;
                if (v >= 0) {
                    if ((uint32_t)v >= n_wide || up[v] != 0xffffffffu || (uint32_t)v == i) {
                        err = "rebuild plan: malformed 4-wide tree";
                        return false;
                    }
                    up[v] = i;
                } else {
                    const uint32_t first = (uint32_t)~v >> 3;
                    if (first >= n_entries || leaf_of[first] == 0xffffffffu || wleaf[first]) {
                        err = "rebuild plan: a 4-wide leaf is no binary leaf, or repeats";
                        return false;
                    }
                    wleaf[first] = 1;
                }
            }
        for (const uint4& l : leaves)
            if (!wleaf[l.y]) { err = "rebuild plan: a binary leaf is in no 4-wide leaf slot"; return false; }
        // heights from one root, children first (iterative post-order)
        uint32_t root = 0xffffffffu;
        for (uint32_t i = 0; i < n_wide; i++)
            if (up[i] == 0xffffffffu) {
                if (root != 0xffffffffu) { err = "rebuild plan: the 4-wide tree has two roots"; return false; }
                root = i;
            }
        if (root == 0xffffffffu) { err = "rebuild plan: the 4-wide tree has no root"; return false; }
        std::vector<uint32_t> post, st{root};
        while (!st.empty()) {
            const uint32_t k = st.back();
            st.pop_back();
            post.push_back(k);
            for (int q = 0; q < 4; q++) {
                const int32_t v = wn[k].child[q];
                if (v >= 0 && v != kSent) st.push_back((uint32_t)v);
            }
        }
        if (post.size() != n_wide) { err = "rebuild plan: 4-wide nodes unreachable from the root"; return false; }
        uint32_t hmax = 0;
        for (size_t j = post.size(); j-- > 0;) {
            const uint32_t k = post[j];
            uint32_t h = 1;
            for (int q = 0; q < 4; q++) {
                const int32_t v = wn[k].child[q];
                if (v >= 0 && v != kSent) h = std::max(h, height[v] + 1);
            }
            height[k] = h;
            hmax = std::max(hmax, h);
        }
        R.woff.assign(hmax + 1, 0);   // heights 1..hmax -> woff[h - 1] .. woff[h]
        for (uint32_t i = 0; i < n_wide; i++) R.woff[height[i]]++;
        for (uint32_t h = 1; h <= hmax; h++) R.woff[h] += R.woff[h - 1];
        worder.resize(n_wide);
        std::vector<uint32_t> fill(R.woff.begin(), R.woff.end() - 1), pos(n_wide);
        for (uint32_t i = 0; i < n_wide; i++) {
            pos[i] = fill[height[i] - 1]++;
            worder[pos[i]] = i;
        }
        // the top: the highest heights while they hold at most kTopMax nodes together
        R.wtop = hmax;
        while (R.wtop > 0 && n_wide - R.woff[R.wtop - 1] <= kTopMax) R.wtop--;
        const uint32_t top0 = R.woff[R.wtop];
        wcode.resize(n_wide);
        for (uint32_t i = 0; i < n_wide; i++) {
            uint32_t c[4];
            for (int q = 0; q < 4; q++) {
                const int32_t v = wn[i].child[q];
                c[q] = v == kSent ? kNoChild
                       : v < 0    ? leaf_of[(uint32_t)~v >> 3] << 2 | 1u
                       : pos[i] >= top0 && pos[v] >= top0 ? (pos[v] - top0) << 2 | 2u
                                                          : (uint32_t)v << 2;
            }
            wcode[i] = make_uint4(c[0], c[1], c[2], c[3]);
        }
    }
    R.n_leaf = (uint32_t)leaves.size();
    R.n_wide = n_wide;
    if (!anim_upload(A, &R.d_leaf, leaves.data(), leaves.size()) ||
        !anim_upload(A, &R.d_leaf_of, leaf_of.data(), leaf_of.size()) || !anim_alloc(A, &R.d_nrec, 8ull * n_nodes) ||
        !anim_alloc(A, &R.d_cnt, n_nodes) || !anim_alloc(A, &R.d_lrec, 8 * std::max<size_t>(1, leaves.size())) ||
        hipMemset(R.d_cnt, 0, n_nodes * sizeof(uint32_t)) != hipSuccess ||
        (n_wide && (!anim_alloc(A, &R.d_wrec, 8ull * n_wide) || !anim_upload(A, &R.d_worder, worder.data(), n_wide) ||
                    !anim_upload(A, &R.d_woff, R.woff.data(), R.woff.size()) ||
                    !anim_upload(A, &R.d_wcode, wcode.data(), n_wide)))) {
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
        R.idx = S.tri_idx + P.km.bvh_indices_offset;
        R.tris = tris;
        R.P = A->d_P;
        R.woop = const_cast<float4*>(S.woop) + P.km.bvh_triangle_offset;
        R.leaf = P.rb.d_leaf;
        R.leaf_of = P.rb.d_leaf_of;
        R.nrec = P.rb.d_nrec;
        R.lrec = P.rb.d_lrec;
        R.cnt = P.rb.d_cnt;
        R.mesh_box = A->d_mesh_boxes + 6 * P.am.mesh;
        R.n_leaf = P.rb.n_leaf;
        R.n_nodes = P.rb.n_nodes;
        hipLaunchKernelGGL(anim_leaf_kernel, dim3((P.rb.n_leaf + kAB - 1) / kAB), dim3(kAB), 0, s, R);
        hipLaunchKernelGGL(anim_rebuild_kernel, dim3((P.rb.n_leaf + kAB - 1) / kAB), dim3(kAB), 0, s, R);
        hipLaunchKernelGGL(anim_slot_kernel, dim3((P.rb.n_nodes + kAB - 1) / kAB), dim3(kAB), 0, s, R.bin, R.nrec, R.lrec,
                           R.leaf_of, R.leaf, P.rb.n_nodes);
        if (S.wide && P.rb.n_wide) {
            // the 4-wide copy: a launch per height below the top, the top in one block
            const WideArgs W{reinterpret_cast<WideNode*>(const_cast<float4*>(S.wbvh)) + P.wide_base, P.rb.d_wrec, R.lrec,
                             P.rb.d_wcode, P.rb.d_worder};
            const uint32_t nh = (uint32_t)P.rb.woff.size() - 1;
            for (uint32_t h = 0; h < P.rb.wtop; h++) {
                const uint32_t n = P.rb.woff[h + 1] - P.rb.woff[h];
                hipLaunchKernelGGL(anim_wide_kernel, dim3((n + kAB - 1) / kAB), dim3(kAB), 0, s, W, P.rb.woff[h], n);
            }
            hipLaunchKernelGGL(anim_wide_top_kernel, dim3(1), dim3(kTopWide), 0, s, W, P.rb.d_woff + P.rb.wtop,
                               nh - P.rb.wtop);
        }
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

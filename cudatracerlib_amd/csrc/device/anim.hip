// anim.hip — animated (skinned) meshes on the device: AnimatedMesh::k_ComputeState
// (Engine/AnimatedMesh.cpp:163-184) as a chain of data-parallel kernels.
//
//   skin     g_ComputeVertices (AnimatedMesh.cu:29-43): per vertex, two 8-bone
//            matrix blends, TransformPoint / TransformDirection, lerp
//   tris     g_ComputeTriangles -> TriangleData::setData (TriangleData.cu:35-63)
//   leaves   per leaf of the mesh tree, its entries' Woop data (AnimProvider::
//            setObject, AnimatedMesh.cpp:113-117) and the union of their
//            triangles' boxes, stored straight into the parent's child slot
//   refit    bottom-up box refit of the mesh's inner children: the subtrees of at
//            most kSubMax inner nodes in one launch, one block each, level by
//            level between block barriers; the nodes above them one launch per
//            wide level (deepest first) and one single-block launch for the
//            narrow top levels; the 4-wide copy then gathers its boxes from the
//            binary children they came from
//   scene    instance boxes (mesh box x node transform), refit of the scene's
//            binary tree + gather into its 4-wide copy, scene box -> m_rayTraceEps
//
// The reference re-derives the mesh tree on the host with BVHRebuilder (refit
// plus subtree rotations, BVHRebuilder.cpp:281-340); the tree shape is not
// observable through traversal, so the compiled topology is kept and only the
// boxes move.  A box is a min/max over the same vertices whatever the order,
// so the refit boxes are exact and the CPU oracle reproduces them bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"
#include "../ctl_anim.h"
#include "../ctl_shade.h"
#include "../host/bvh_wide.h"
#include "../ctl_qnode.h"

namespace ctl {

struct AnimTree {
    uint32_t base = 0;                  // float4 offset of the tree's node 0
    // The nodes refit by one block (refit_block_kernel): a record {node, child 0,
    // child 1} per node, grouped in block sets, each set's levels deepest first.
    struct Blocks {
        uint32_t n_sets = 0, max_nodes = 0, max_levels = 0;
        uint4* d_rec = nullptr;
        uint32_t* d_lvl = nullptr;      // [levels + 1] level offsets into d_rec, all sets
        uint32_t* d_first = nullptr;    // [n_sets + 1] first level of each set
    };
    Blocks sub;                         // the subtrees below the cut, one set each
    Blocks top;                         // the narrow levels at the top of the tree, one set
    // the levels in between, too wide for one block: one launch each, deepest first
    std::vector<uint32_t> level_off;    // [levels + 1] offsets into d_order
    uint32_t* d_order = nullptr;        // node indices relative to base
    // mesh trees: the leaves, boxed by anim_leaf_kernel
    uint32_t n_leaf = 0;
    uint4* d_leaf = nullptr;            // {node << 1 | child, first entry, entries, 0}
    bool valid = false;
};

// A 4-wide copy's boxes after the binary refit: slot q of the wide tree takes
// the box of binary (node, child) src[q] (recorded by collapse_wide).
struct WideGather {
    uint32_t base = 0;                  // wide-node index of the tree's node 0
    uint32_t n_slots = 0;               // 4 x nodes
    uint32_t* d_src = nullptr;
    bool valid = false;
};

struct AnimMeshPlan {
    ctl_anim_mesh am;
    ctl_kernel_mesh km;
    uint32_t n_entries = 0;
    AnimTree bin;
    WideGather wide;
};

struct AnimState {
    std::vector<AnimMeshPlan> meshes;
    AnimTree scene_bin;
    WideGather scene_wide;
    const ctl_anim_vertex* d_verts = nullptr;
    const uint32_t* d_tris = nullptr;
    float* d_mesh_boxes = nullptr;      // 6 per mesh
    float* d_inst_boxes = nullptr;      // 6 per node
    float* d_eps = nullptr;             // scene box (6) + eps + cull_m (3)
    float* h_eps = nullptr;             // pinned
    float4* d_P = nullptr;
    float4* d_N = nullptr;
    size_t tmp_cap = 0;
    float* d_bones[2] = {nullptr, nullptr};
    size_t bones_cap = 0;
    uint32_t n_meshes = 0, n_nodes = 0;
    std::vector<void*> allocs;
};

namespace {

constexpr int32_t kSent = 0x76543210;
constexpr int kAB = 256;
constexpr uint32_t kTopMax = 512;    // levels at most this wide go to the single-block top set ...
constexpr uint32_t kTopLds = 1400;   // ... of at most this many nodes (boxes, records, level offsets in LDS: < 62 KB)
constexpr uint32_t kSubMax = 511;    // inner nodes of a subtree refit by one block
// child references of a block record: an LDS slot (the set's own node), or
constexpr uint32_t kRefGlobal = 0x40000000u;   // | node: a node refit earlier (its child slots in memory)
constexpr uint32_t kRefInst = 0x80000000u;     // | instance: a scene-tree leaf
constexpr uint32_t kRefLeafSlot = 0xfffffffeu; // a mesh leaf, its slot written by anim_leaf_kernel
constexpr uint32_t kRefNone = 0xffffffffu;     // an empty child

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

// BVHNodeData child boxes (the reference layout, TriIntersectorData.h:44-50)
__device__ __forceinline__ void bin_child_box(const float* nd, int c, float lo[3], float hi[3]) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    lo[0] = nd[o]; hi[0] = nd[o + 1]; lo[1] = nd[o + 2]; hi[1] = nd[o + 3]; lo[2] = nd[z]; hi[2] = nd[z + 1];
}
__device__ __forceinline__ void bin_set_child_box(float* nd, int c, const float lo[3], const float hi[3]) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    nd[o] = lo[0]; nd[o + 1] = hi[0]; nd[o + 2] = lo[1]; nd[o + 3] = hi[1]; nd[z] = lo[2]; nd[z + 1] = hi[2];
}
// Per leaf of a mesh tree (one thread): each entry of its run gets its Woop
// data (AnimProvider::setObject, AnimatedMesh.cpp:113-117), and the union of
// the entries' triangle boxes, in entry order, goes into the parent's child
// slot.  The leaves cover every entry once (checked by the plan), and the plan
// counts each run, so an entry's loads do not wait for the previous end bit.
__global__ __launch_bounds__(kAB) void anim_leaf_kernel(const uint4* __restrict__ leaves, uint32_t n,
                                                       const uint32_t* __restrict__ idx, const uint32_t* __restrict__ tris,
                                                       const float4* __restrict__ P, float4* woop, float* nodes) {
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= n) return;
    const uint4 lf = leaves[i];
    float lo[3], hi[3];
    box_empty(lo, hi);
#pragma unroll 2
    for (uint32_t e = lf.y; e < lf.y + lf.z; e++) {
        const uint32_t t = idx[e] >> 1;
        const f3 a = ld3(P, tris[3 * t]), b = ld3(P, tris[3 * t + 1]), c = ld3(P, tris[3 * t + 2]);
        float w[12];
        woop_set_hd(a, b, c, w);
        woop[3 * e] = make_float4(w[0], w[1], w[2], w[3]);
        woop[3 * e + 1] = make_float4(w[4], w[5], w[6], w[7]);
        woop[3 * e + 2] = make_float4(w[8], w[9], w[10], w[11]);
        const float q0[3] = {tmin(tmin(a.x, b.x), c.x), tmin(tmin(a.y, b.y), c.y), tmin(tmin(a.z, b.z), c.z)};
        const float q1[3] = {tmax(tmax(a.x, b.x), c.x), tmax(tmax(a.y, b.y), c.y), tmax(tmax(a.z, b.z), c.z)};
        box_extend(lo, hi, q0, q1);
    }
    bin_set_child_box(nodes + 16 * (size_t)(lf.x >> 1), (int)(lf.x & 1u), lo, hi);
}

// Leaf boxes of the scene tree: its leaves are instances (~node).  Mesh trees
// (SCENE = false) have their leaf slots written by anim_leaf_kernel.
struct LeafCtx {
    const float* inst;       // instance boxes (scene)
};

// The node's box: the union of its non-empty child slots, in slot order.  The
// whole 64-B node is loaded up front (four 16-B loads in flight, `nd` 16-B
// aligned) rather than a slot after its sentinel test.
__device__ __forceinline__ void bin_node_box(const float* nd, float lo[3], float hi[3]) {
    const float4* n4 = reinterpret_cast<const float4*>(nd);
    const float4 q0 = n4[0], q1 = n4[1], q2 = n4[2], q3 = n4[3];
    box_empty(lo, hi);
    if (__float_as_int(q3.x) != kSent) {
        const float a[3] = {q0.x, q0.z, q2.x}, b[3] = {q0.y, q0.w, q2.y};
        box_extend(lo, hi, a, b);
    }
    if (__float_as_int(q3.y) != kSent) {
        const float a[3] = {q1.x, q1.z, q2.z}, b[3] = {q1.y, q1.w, q2.w};
        box_extend(lo, hi, a, b);
    }
}

// One node: its children's boxes from their leaves or from the children's own
// (already refit) child boxes.
template <bool SCENE>
__device__ __forceinline__ void refit_node(float* nodes, uint32_t k, const LeafCtx& L) {
    float* nd = nodes + 16 * (size_t)k;
    for (int c = 0; c < 2; c++) {
        const int32_t v = __float_as_int(nd[12 + c]);
        if (v == kSent) continue;
        float lo[3], hi[3];
        if (v < 0) {
            if (!SCENE) continue;   // written by anim_leaf_kernel
            const float* b = L.inst + 6 * (uint32_t)~v;
            for (int k = 0; k < 3; k++) { lo[k] = b[k]; hi[k] = b[3 + k]; }
        } else {
            bin_node_box(nodes + 16 * (size_t)(v >> 2), lo, hi);
        }
        bin_set_child_box(nd, c, lo, hi);
    }
}

template <bool SCENE>
__global__ __launch_bounds__(kAB) void refit_bin_kernel(float* nodes, const uint32_t* __restrict__ order, uint32_t n,
                                                       LeafCtx L) {
    const uint32_t i = blockIdx.x * kAB + threadIdx.x;
    if (i >= n) return;
    refit_node<SCENE>(nodes, order[i], L);
}

// One node of a block set: each child slot from its reference, and the node's
// own box (the union of its slots, in slot order as bin_node_box takes it) into
// LDS for its parent in the same set.
template <bool SCENE>
__device__ __forceinline__ void refit_rec(float* nodes, const uint4 q, float* sbox, uint32_t self, const LeafCtx& L) {
    float* nd = nodes + 16 * (size_t)q.x;
    float lo[2][3], hi[2][3];
    bool set[2];
    for (int c = 0; c < 2; c++) {
        const uint32_t r = c ? q.z : q.y;
        set[c] = r != kRefNone && r != kRefLeafSlot;
        if (r == kRefNone) continue;
        if (r == kRefLeafSlot) {
            bin_child_box(nd, c, lo[c], hi[c]);
        } else if (r < kRefGlobal) {
            const float* b = sbox + 6 * r;
            for (int k = 0; k < 3; k++) { lo[c][k] = b[k]; hi[c][k] = b[3 + k]; }
        } else if (r < kRefInst) {
            bin_node_box(nodes + 16 * (size_t)(r - kRefGlobal), lo[c], hi[c]);
        } else {
            const float* b = L.inst + 6 * (size_t)(r - kRefInst);
            for (int k = 0; k < 3; k++) { lo[c][k] = b[k]; hi[c][k] = b[3 + k]; }
        }
    }
    if (set[0] && set[1]) {   // both slots: the node's first 48 B as three whole 16-B stores
        float4* n4 = reinterpret_cast<float4*>(nd);
        n4[0] = make_float4(lo[0][0], hi[0][0], lo[0][1], hi[0][1]);
        n4[1] = make_float4(lo[1][0], hi[1][0], lo[1][1], hi[1][1]);
        n4[2] = make_float4(lo[0][2], hi[0][2], lo[1][2], hi[1][2]);
    } else {
        for (int c = 0; c < 2; c++)
            if (set[c]) bin_set_child_box(nd, c, lo[c], hi[c]);
    }
    float ulo[3], uhi[3];
    box_empty(ulo, uhi);
    if (q.y != kRefNone) box_extend(ulo, uhi, lo[0], hi[0]);
    if (q.z != kRefNone) box_extend(ulo, uhi, lo[1], hi[1]);
    float* o = sbox + 6 * self;
    for (int k = 0; k < 3; k++) { o[k] = ulo[k]; o[3 + k] = uhi[k]; }
}

// Block sets (the subtrees below the cut, one per block; the narrow top of the
// tree in one block): the set's records and level offsets staged in LDS once,
// then level after level with the boxes handed up through LDS.  The barrier
// between levels waits for this wave's LDS traffic only: the node stores are
// read by no one in this launch.  LDS: max_nodes (even) x (6 floats + one
// record) + max_levels + 1 offsets.
template <bool SCENE, int NT>
__global__ __launch_bounds__(NT) void refit_block_kernel(float* nodes, const uint4* __restrict__ rec,
                                                        const uint32_t* __restrict__ lvl,
                                                        const uint32_t* __restrict__ first, uint32_t max_nodes,
                                                        LeafCtx L) {
    extern __shared__ float sbox[];
    uint4* srec = reinterpret_cast<uint4*>(sbox + 6 * max_nodes);
    uint32_t* slvl = reinterpret_cast<uint32_t*>(srec + max_nodes);
    const uint32_t l0 = first[blockIdx.x], nl = first[blockIdx.x + 1] - l0;
    const uint32_t base = lvl[l0], end = lvl[l0 + nl];
    for (uint32_t i = base + threadIdx.x; i < end; i += NT) srec[i - base] = rec[i];
    for (uint32_t l = threadIdx.x; l <= nl; l += NT) slvl[l] = lvl[l0 + l] - base;
    __syncthreads();
    for (uint32_t l = 0; l < nl; l++) {
        const uint32_t e = slvl[l + 1];
        for (uint32_t i = slvl[l] + threadIdx.x; i < e; i += NT) refit_rec<SCENE>(nodes, srec[i], sbox, i, L);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

__global__ __launch_bounds__(kAB) void wide_gather_kernel(WideNode* wide, const uint32_t* __restrict__ src,
                                                         uint32_t n_slots, const float* __restrict__ bin) {
    const uint32_t q = blockIdx.x * kAB + threadIdx.x;
    if (q >= n_slots) return;
    const uint32_t sidx = src[q];
    if (sidx == 0xffffffffu) return;
    float lo[3], hi[3];
    bin_child_box(bin + 16 * (size_t)(sidx >> 1), (int)(sidx & 1u), lo, hi);
    WideNode& w = wide[q >> 2];
    const uint32_t sl = q & 3u;
    w.lo_x[sl] = lo[0]; w.lo_y[sl] = lo[1]; w.lo_z[sl] = lo[2];
    w.hi_x[sl] = hi[0]; w.hi_y[sl] = hi[1]; w.hi_z[sl] = hi[2];
}

// m_sLocalBox of the refit mesh: the union of its root's children.
__global__ void mesh_box_kernel(const float* root, float* out) {
    float lo[3], hi[3];
    bin_node_box(root, lo, hi);
    for (int k = 0; k < 3; k++) { out[k] = lo[k]; out[3 + k] = hi[k]; }
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

bool upload_blocks(AnimState* A, AnimTree::Blocks& B, const std::vector<uint4>& rec, const std::vector<uint32_t>& lvl,
                   const std::vector<uint32_t>& first) {
    B.n_sets = (uint32_t)first.size() - 1;
    B.max_nodes += B.max_nodes & 1u;   // even: the records after the boxes stay 16-B aligned
    return anim_upload(A, &B.d_rec, rec.data(), rec.size()) && anim_upload(A, &B.d_lvl, lvl.data(), lvl.size()) &&
           anim_upload(A, &B.d_first, first.data(), first.size());
}

// Refit plan of a binary tree (BVHNodeData, TriIntersectorData.h:44-50).
//   - the cut: the subtrees of at most kSubMax inner nodes hanging off the
//     nodes above them, one block set each;
//   - above the cut, by depth from the root, deepest first: the narrow levels
//     at the top (each at most kTopMax wide, together at most kTopLds) in one
//     block set, the wider levels below them one launch each.
// A mesh tree (n_entries > 0, `idx` its entries' TriIntersectorData2 words) also
// lists its leaves for anim_leaf_kernel, which writes their slots; a node with
// only leaf children is then in no list.  Every entry must lie in exactly one leaf.
bool plan_binary(AnimState* A, AnimTree& T, const ctl_bvh_node* nodes, uint32_t n_nodes, uint32_t base_f4,
                 uint32_t root, uint32_t n_entries, const uint32_t* idx, std::string& err) {
    T.base = base_f4;
    if (n_nodes == 0 || root >= n_nodes) { err = "refit plan: empty tree"; return false; }
    const bool mesh = n_entries > 0;
    auto child = [&](uint32_t k, int c) {
        int32_t v;
        memcpy(&v, &nodes[k].v[12 + c], 4);
        return v;
    };
    auto kids = [&](uint32_t k, uint32_t* out) {
        int n = 0;
        for (int c = 0; c < 2; c++) {
            const int32_t v = child(k, c);
            if (v >= 0 && v != kSent) out[n++] = (uint32_t)v >> 2;
        }
        return n;
    };
    // depth of every node reachable from the root, and a pre-order
    std::vector<int> depth(n_nodes, -1);
    std::vector<uint32_t> pre, st{root};
    depth[root] = 0;
    while (!st.empty()) {
        const uint32_t k = st.back();
        st.pop_back();
        pre.push_back(k);
        uint32_t ch[2];
        const int nc = kids(k, ch);
        for (int i = 0; i < nc; i++) {
            if (ch[i] >= n_nodes || depth[ch[i]] >= 0) { err = "refit plan: malformed tree"; return false; }
            depth[ch[i]] = depth[k] + 1;
            st.push_back(ch[i]);
        }
    }
    if (pre.size() >= kRefGlobal) { err = "refit plan: tree too large"; return false; }
    // inner nodes per subtree (reverse pre-order: children first)
    std::vector<uint32_t> size(n_nodes, 0);
    for (size_t i = pre.size(); i-- > 0;) {
        uint32_t ch[2];
        const int nc = kids(pre[i], ch);
        size[pre[i]] = 1;
        for (int c = 0; c < nc; c++) size[pre[i]] += size[ch[c]];
    }
    std::vector<int32_t> loc(n_nodes, -1);   // LDS slot of a node of the set being planned
    auto record = [&](uint32_t k) {
        uint32_t r[2];
        for (int c = 0; c < 2; c++) {
            const int32_t v = child(k, c);
            if (v == kSent) r[c] = kRefNone;
            else if (v < 0) r[c] = mesh ? kRefLeafSlot : kRefInst + (uint32_t)~v;
            else if (loc[(uint32_t)v >> 2] >= 0) r[c] = (uint32_t)loc[(uint32_t)v >> 2];
            else r[c] = kRefGlobal + ((uint32_t)v >> 2);
        }
        return make_uint4(k, r[0], r[1], 0u);
    };
    // a block set from its nodes grouped by level, deepest first
    auto add_set = [&](const std::vector<std::vector<uint32_t>>& lv, std::vector<uint4>& rec, std::vector<uint32_t>& lvl,
                       std::vector<uint32_t>& first, uint32_t& max_nodes, uint32_t& max_levels) {
        first.push_back((uint32_t)lvl.size());
        const size_t r0 = rec.size(), v0 = lvl.size();
        for (const auto& level : lv) {
            if (level.empty()) continue;
            lvl.push_back((uint32_t)rec.size());
            for (uint32_t k : level) rec.push_back(record(k));
            for (size_t q = 0; q < level.size(); q++) loc[level[q]] = (int32_t)(rec.size() - level.size() - r0 + q);
        }
        max_nodes = std::max<uint32_t>(max_nodes, (uint32_t)(rec.size() - r0));
        max_levels = std::max<uint32_t>(max_levels, (uint32_t)(lvl.size() - v0));
        for (size_t q = r0; q < rec.size(); q++) loc[rec[q].x] = -1;
    };
    // the cut
    std::vector<uint32_t> top, cuts;
    st.assign(1, root);
    while (!st.empty()) {
        const uint32_t k = st.back();
        st.pop_back();
        if (size[k] <= kSubMax) { cuts.push_back(k); continue; }
        top.push_back(k);   // more than one inner node at and below it: an inner child
        uint32_t ch[2];
        const int nc = kids(k, ch);
        for (int c = 0; c < nc; c++) st.push_back(ch[c]);
    }
    std::sort(cuts.begin(), cuts.end());
    std::vector<uint4> rec;
    std::vector<uint32_t> lvl, first;
    std::vector<std::vector<uint32_t>> lv;
    for (uint32_t r : cuts) {
        lv.clear();
        st.assign(1, r);
        while (!st.empty()) {
            const uint32_t k = st.back();
            st.pop_back();
            uint32_t ch[2];
            const int nc = kids(k, ch);
            for (int c = 0; c < nc; c++) st.push_back(ch[c]);
            if (mesh && nc == 0) continue;   // leaf slots only: anim_leaf_kernel
            const size_t d = (size_t)(depth[k] - depth[r]);
            if (lv.size() <= d) lv.resize(d + 1);
            lv[d].push_back(k);
        }
        if (lv.empty()) continue;
        std::reverse(lv.begin(), lv.end());
        for (auto& level : lv) std::sort(level.begin(), level.end());
        add_set(lv, rec, lvl, first, T.sub.max_nodes, T.sub.max_levels);
    }
    lvl.push_back((uint32_t)rec.size());
    if (first.empty()) first.push_back(0);
    else first.push_back((uint32_t)lvl.size() - 1);
    if (!upload_blocks(A, T.sub, rec, lvl, first)) { err = "refit plan: upload failed"; return false; }
    // above the cut, deepest first; the top levels that fit one block
    std::sort(top.begin(), top.end(), [&](uint32_t a, uint32_t b) {
        return depth[a] != depth[b] ? depth[a] > depth[b] : a < b;
    });
    std::vector<uint32_t> off;
    for (size_t i = 0; i < top.size(); i++)
        if (i == 0 || depth[top[i]] != depth[top[i - 1]]) off.push_back((uint32_t)i);
    off.push_back((uint32_t)top.size());
    size_t split = off.size() - 1;   // levels [split, end) go to the top block set
    while (split > 0 && off[split] - off[split - 1] <= kTopMax && top.size() - off[split - 1] <= kTopLds) split--;
    T.level_off.assign(off.begin(), off.begin() + split + 1);
    lv.clear();
    for (size_t l = split; l + 1 < off.size(); l++) lv.emplace_back(top.begin() + off[l], top.begin() + off[l + 1]);
    rec.clear(); lvl.clear(); first.clear();
    if (!lv.empty()) add_set(lv, rec, lvl, first, T.top.max_nodes, T.top.max_levels);
    lvl.push_back((uint32_t)rec.size());
    first.push_back((uint32_t)lvl.size() - 1);
    if (!upload_blocks(A, T.top, rec, lvl, first) ||
        !anim_upload(A, &T.d_order, top.data(), off[split])) { err = "refit plan: upload failed"; return false; }
    T.valid = true;
    if (!mesh) return true;
    // the leaves of a mesh tree, in entry order
    std::vector<uint4> leaves;
    std::vector<uint8_t> seen(n_entries, 0);
    for (uint32_t k : pre)
        for (int c = 0; c < 2; c++) {
            const int32_t v = child(k, c);
            if (v >= 0 || v == kSent) continue;
            uint32_t e = (uint32_t)~v;
            for (;; e++) {
                if (e >= n_entries || seen[e]) { err = "refit plan: a leaf's entries overrun or overlap"; return false; }
                seen[e] = 1;
                if (idx[e] & 1) break;
            }
            leaves.push_back(make_uint4(k << 1 | (uint32_t)c, (uint32_t)~v, e + 1 - (uint32_t)~v, 0u));
        }
    if (std::find(seen.begin(), seen.end(), 0) != seen.end()) { err = "refit plan: an entry lies in no leaf"; return false; }
    std::sort(leaves.begin(), leaves.end(), [](uint4 a, uint4 b) { return a.y < b.y; });
    T.n_leaf = (uint32_t)leaves.size();
    if (!anim_upload(A, &T.d_leaf, leaves.data(), leaves.size())) { err = "refit plan: upload failed"; return false; }
    return true;
}

bool plan_gather(AnimState* A, WideGather& G, const uint32_t* src, uint32_t n_nodes, uint32_t base, std::string& err) {
    G.base = base;
    G.n_slots = 4 * n_nodes;
    if (!anim_upload(A, &G.d_src, src, G.n_slots)) { err = "refit plan: upload failed"; return false; }
    G.valid = true;
    return true;
}

template <bool SCENE>
void launch_refit(hipStream_t s, const AnimTree& T, float* bin_base, const LeafCtx& L) {
    const size_t per = 6 * sizeof(float) + sizeof(uint4);
    if (T.sub.n_sets)
        hipLaunchKernelGGL((refit_block_kernel<SCENE, kAB>), dim3(T.sub.n_sets), dim3(kAB),
                           per * T.sub.max_nodes + 4 * (T.sub.max_levels + 1), s,
                           bin_base, T.sub.d_rec, T.sub.d_lvl, T.sub.d_first, T.sub.max_nodes, L);
    for (size_t l = 0; l + 1 < T.level_off.size(); l++) {
        const uint32_t first = T.level_off[l], cnt = T.level_off[l + 1] - first;
        hipLaunchKernelGGL(refit_bin_kernel<SCENE>, dim3((cnt + kAB - 1) / kAB), dim3(kAB), 0, s, bin_base,
                           T.d_order + first, cnt, L);
    }
    if (T.top.n_sets)
        hipLaunchKernelGGL((refit_block_kernel<SCENE, 1024>), dim3(1), dim3(1024),
                           per * T.top.max_nodes + 4 * (T.top.max_levels + 1), s,
                           bin_base, T.top.d_rec, T.top.d_lvl, T.top.d_first, T.top.max_nodes, L);
}

void launch_gather(hipStream_t s, const WideGather& G, WideNode* wide_base, const float* bin_base) {
    if (!G.valid || !G.n_slots) return;
    hipLaunchKernelGGL(wide_gather_kernel, dim3((G.n_slots + kAB - 1) / kAB), dim3(kAB), 0, s, wide_base + G.base,
                       G.d_src, G.n_slots, bin_base);
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
               const std::vector<uint32_t>& wbase, const std::vector<WideNode>& sw,
               const std::vector<uint32_t>& wsrc, const std::vector<uint32_t>& ssrc) {
    anim_free(c);
    if (!d->mesh_boxes) return CTL_OK;
    c->anim = new AnimState();
    AnimState* A = c->anim;
    std::string err;
    auto fail = [&](const std::string& m) { c->err = "scene_upload: " + m; anim_free(c); return (int)CTL_ERR_INVALID; };
    A->n_meshes = d->n_meshes;
    A->n_nodes = d->n_nodes;
    if (!anim_upload(A, &A->d_mesh_boxes, d->mesh_boxes, 6ull * d->n_meshes) ||
        !anim_alloc(A, &A->d_inst_boxes, 6ull * std::max(1u, d->n_nodes)) || !anim_alloc(A, &A->d_eps, 10) ||
        hipHostMalloc((void**)&A->h_eps, 10 * sizeof(float), hipHostMallocDefault) != hipSuccess)
        return fail("animation state allocation failed");
    const bool wide = !wn.empty() || !sw.empty();
    // the instance tree's refit plan: animated meshes and moved nodes (ctl_scene_set_transform)
    if (d->n_nodes > 0 && d->scene_start_node >= 0 && d->n_scene_bvh_nodes > 0) {
        if (!plan_binary(A, A->scene_bin, d->scene_bvh_nodes, d->n_scene_bvh_nodes, 0,
                         (uint32_t)d->scene_start_node >> 2, 0, nullptr, err))
            return fail(err);
        if (wide && !sw.empty()) {
            if (ssrc.size() != 4 * sw.size()) return fail("wide source map missing");
            if (!plan_gather(A, A->scene_wide, ssrc.data(), (uint32_t)sw.size(), 0, err)) return fail(err);
        }
    }
    if (d->n_anim_meshes == 0) return CTL_OK;
    if (!anim_upload(A, (ctl_anim_vertex**)&A->d_verts, d->anim_vertices, d->n_anim_vertices) ||
        !anim_upload(A, (uint32_t**)&A->d_tris, d->anim_triangles, 3ull * d->n_anim_triangles))
        return fail("animation upload failed");
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
        if (!plan_binary(A, P.bin, d->bvh_nodes + n0, (uint32_t)(n1 - n0), P.km.bvh_node_offset, 0, P.n_entries,
                         d->tri_indices + e0, err))
            return fail(err);
        if (wide) {
            const uint32_t wb = wbase[P.am.mesh];
            const uint32_t we = P.am.mesh + 1 < wbase.size() ? wbase[P.am.mesh + 1] : (uint32_t)wn.size();
            if (wsrc.size() != 4 * wn.size()) return fail("wide source map missing");
            if (!plan_gather(A, P.wide, wsrc.data() + 4ull * wb, we - wb, wb, err)) return fail(err);
        }
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
    const uint32_t nv = P.am.vertex_count, nt = P.am.tri_count;
    const uint32_t* tris = A->d_tris + 3ull * P.am.tri_first;
    if (nv) hipLaunchKernelGGL(anim_skin_kernel, dim3((nv + kAB - 1) / kAB), dim3(kAB), 34 * n_bones * sizeof(float), s,
                               A->d_verts + P.am.vertex_first, nv, A->d_bones[0], A->d_bones[1], n_bones, lerp, A->d_P,
                               A->d_N);
    if (nt) hipLaunchKernelGGL(anim_tri_kernel, dim3((nt + kAB - 1) / kAB), dim3(kAB), 0, s, tris, nt, A->d_P, A->d_N,
                               const_cast<ctl_triangle_data*>(S.tri_data) + P.km.triangle_offset);
    const uint32_t* idx = S.tri_idx + P.km.bvh_indices_offset;
    float* bin = reinterpret_cast<float*>(const_cast<float4*>(S.bvh) + P.bin.base);
    if (P.bin.n_leaf)
        hipLaunchKernelGGL(anim_leaf_kernel, dim3((P.bin.n_leaf + kAB - 1) / kAB), dim3(kAB), 0, s, P.bin.d_leaf,
                           P.bin.n_leaf, idx, tris, A->d_P, const_cast<float4*>(S.woop) + P.km.bvh_triangle_offset, bin);
    launch_refit<false>(s, P.bin, bin, LeafCtx{nullptr});
    launch_gather(s, P.wide, reinterpret_cast<WideNode*>(const_cast<float4*>(S.wbvh)), bin);
    hipLaunchKernelGGL(mesh_box_kernel, dim3(1), dim3(1), 0, s, bin, A->d_mesh_boxes + 6 * P.am.mesh);
    // instances, scene trees, epsilon
    if (A->n_nodes) {
        hipLaunchKernelGGL(inst_box_kernel, dim3((A->n_nodes + kAB - 1) / kAB), dim3(kAB), 0, s, S.nodes, S.xf,
                           A->n_nodes, A->d_mesh_boxes, A->d_inst_boxes);
        LeafCtx LS{A->d_inst_boxes};
        float* sbin = reinterpret_cast<float*>(const_cast<float4*>(S.scene_bvh));
        if (A->scene_bin.valid) launch_refit<true>(s, A->scene_bin, sbin, LS);
        launch_gather(s, A->scene_wide, reinterpret_cast<WideNode*>(const_cast<float4*>(S.scene_wbvh)), sbin);
        hipLaunchKernelGGL(scene_eps_kernel, dim3(1), dim3(1), 0, s, A->d_inst_boxes, A->n_nodes, A->d_eps,
                           const_cast<ctl_env_light*>(S.env), A->d_mesh_boxes, A->n_meshes);
        if (hipMemcpyAsync(A->h_eps, A->d_eps, 10 * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            c->err = "scene_animate: epsilon readback failed";
            return CTL_ERR_HIP;
        }
        S.ray_eps = A->h_eps[6];
        for (int k = 0; k < 3; k++) S.cull_m[k] = A->h_eps[7 + k];
        // a bound on every mesh box now on the device (cull_bound took them all),
        // kept past an instance-only update (set_constants)
        for (int k = 0; k < 3; k++) c->moved_cull_m[k] = S.cull_m[k];
        c->mesh_moved = true;
        c->device_eps = true;
    }
    c->device_edited = true;
    if (hipGetLastError() != hipSuccess) { c->err = "scene_animate: launch failed"; return CTL_ERR_HIP; }
    return CTL_OK;
}

CTL_API ctl_status ctl_scene_set_transform(ctl_ctx* c, uint32_t node, const ctl_float4x4* xf, void* stream) {
    if (!c || !xf) return CTL_ERR_INVALID;
    if (!c->has_scene || !c->anim) { c->err = "scene_set_transform: no scene uploaded"; return CTL_ERR_STATE; }
    AnimState* A = c->anim;
    DevScene& S = c->scene;
    if (node >= S.n_nodes) { c->err = "scene_set_transform: node index out of range"; return CTL_ERR_INVALID; }
    if (S.wide && S.quant && A->scene_bin.valid) {
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
    hipLaunchKernelGGL(inst_box_kernel, dim3((A->n_nodes + kAB - 1) / kAB), dim3(kAB), 0, s, S.nodes, S.xf, A->n_nodes,
                       A->d_mesh_boxes, A->d_inst_boxes);
    LeafCtx LS{A->d_inst_boxes};
    float* sbin = reinterpret_cast<float*>(const_cast<float4*>(S.scene_bvh));
    if (A->scene_bin.valid) launch_refit<true>(s, A->scene_bin, sbin, LS);
    if (S.wide) launch_gather(s, A->scene_wide, reinterpret_cast<WideNode*>(const_cast<float4*>(S.scene_wbvh)), sbin);
    hipLaunchKernelGGL(scene_eps_kernel, dim3(1), dim3(1), 0, s, A->d_inst_boxes, A->n_nodes, A->d_eps,
                       const_cast<ctl_env_light*>(S.env), A->d_mesh_boxes, A->n_meshes);
    if (hipGetLastError() != hipSuccess) { c->err = "scene_set_transform: launch failed"; return CTL_ERR_HIP; }
    if (hipMemcpyAsync(A->h_eps, A->d_eps, 10 * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        c->err = "scene_set_transform: epsilon readback failed";
        return CTL_ERR_HIP;
    }
    S.ray_eps = A->h_eps[6];
    for (int k = 0; k < 3; k++) S.cull_m[k] = A->h_eps[7 + k];
    c->device_eps = true;
    c->device_edited = true;
    return CTL_OK;
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

// oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference (Ilinite/CudaTracerLib) algorithm for the
// hot path: two-level Aila–Laine BVH traversal + Woop ray/triangle test
// (Kernel/TraceHelper.cu:88-180, Engine/SpatialStructures/BVH/BVHTraversal.h:122-232),
// the batch intersectKernel semantics (TraceHelper.cu:326-746), the
// SequenceSampler / CudaRNG (XORWOW) streams (Kernel/Sampler*.h,
// Base/CudaRandom.{h,cu}), PerspectiveSensor (SceneTypes/Sensor.cu:76-144),
// diffuse BSDF (SceneTypes/BSDF_Simple.cu:7-75), DiffuseLight + ShapeSet
// (SceneTypes/Light.cu:55-155, Engine/ShapeSet.cu:11-68), the PathTrace<true>
// integrator loop (Integrators/PathTracer.cu:10-113,182-194) and
// Image::AddSample (Engine/Image.cu:22-44).
//
// It is the CHECKER for the HIP kernels and the cpu_baseline of bench.py.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it;
// the product library (libctl_trace.so) never links or calls it.
//
// Parity pinning: the reference cannot be built here (it needs the CUDA
// toolkit and empty submodules; a build would need stand-in CUDA headers,
// which this project does not write), and it ships no tests or fixtures.  The
// sampler stream is pinned by the reference outputs recorded in SURVEY.md §8c
// (tests/golden/sampler_reference_values.json); everything else is "parity
// unpinned" against the reference binary and is checked by properties
// (brute-force closest hit, Woop round trip) — see DESIGN.md §Parity.
#include "oracle_math.h"
#include "../include/ctl_trace.h"

#include <vector>
#include <functional>
#include <thread>
#include <atomic>
#include <mutex>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

using namespace oracle;

namespace {

// ---------------------------------------------------------------------------
// Woop unit-triangle transform (Engine/TriIntersectorData.cu:5-32)
// ---------------------------------------------------------------------------
void woop_set(V3 a, V3 b, V3 c, float out[12]) {
    M44 m;
    m.setCol(0, v4(a - c, 0));
    m.setCol(1, v4(b - c, 0));
    m.setCol(2, v4(cross(a - c, b - c), 0));
    m.setCol(3, v4(c, 1));
    m = inverse(m);
    V4 A = v4(m(2, 0), m(2, 1), m(2, 2), -m(2, 3));
    V4 B = m.row(0), C = m.row(1);
    float tmp[12] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, C.x, C.y, C.z, C.w};
    std::memcpy(out, tmp, sizeof(tmp));
}
void woop_get(const float in[12], V3& v0, V3& v1, V3& v2) {
    M44 m = M44::identity();
    m.setRow(0, v4(in[4], in[5], in[6], in[7]));   // b
    m.setRow(1, v4(in[8], in[9], in[10], in[11])); // c
    m.setRow(2, v4(in[0], in[1], in[2], in[3]));   // a
    m(2, 3) *= -1.0f;
    m = inverse(m);
    V3 e02 = xyz(m.col(0)), e12 = xyz(m.col(1));
    v2 = xyz(m.col(3));
    v0 = v2 + e02;
    v1 = v2 + e12;
}

// ---------------------------------------------------------------------------
// kepler_math spans on float bit patterns (Math/MathFunc.h:402-445, host branch)
// ---------------------------------------------------------------------------
inline int imin3(int a, int b, int c) { return omin(omin(a, b), c); }
inline int imax3(int a, int b, int c) { return omax(omax(a, b), c); }
inline int imin_max(int a, int b, int c) { return omax(omin(a, b), c); }
inline int imax_min(int a, int b, int c) { return omin(omax(a, b), c); }
inline float spanBegin(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    return as_float(imax3(as_int(omin(a0, a1)), as_int(omin(b0, b1)), imin_max(as_int(c0), as_int(c1), as_int(d))));
}
inline float spanEnd(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    return as_float(imin3(as_int(omax(a0, a1)), as_int(omax(b0, b1)), imax_min(as_int(c0), as_int(c1), as_int(d))));
}

const int EntrypointSentinel = 0x76543210;

struct Stats { uint64_t nodes = 0, tris = 0, inst = 0; };

// TracerayTemplate, pointer overload (BVHTraversal.h:122-232).  spanTmin is 0
// for traceRay and the ray's tmin for the batch kernel (TraceHelper.cu:469).
// Boxes are culled against rayT, the current hit (the reference), or against
// cullFloor when that is larger: the any-hit shadow query's cull distance,
// which lies past its acceptance bound rayT (occluded(), kShadowCull).
template <class CLB>
bool traceray_template(V3 ori, V3 dir, float& rayT, float spanTmin, const CLB& clb, const float* nodes4,
                       int bvhNodesOffset, int startNode, Stats* st, float cullFloor = 0.0f) {
    if (startNode < 0) return clb(~startNode);
    bool found = false;
    // index 1 holds the sentinel; index 0 only absorbs the pop of an already
    // popped sentinel (the reference would read before its array there)
    int traversalStack[64 + 3];
    traversalStack[0] = EntrypointSentinel;
    traversalStack[1] = EntrypointSentinel;
    const float ooeps = powf(2.0f, -80.0f);   // math::exp2 host branch (MathFunc.h:240-245)
    float idirx = 1.0f / (fabsf(dir.x) > ooeps ? dir.x : o_copysign(ooeps, dir.x));
    float idiry = 1.0f / (fabsf(dir.y) > ooeps ? dir.y : o_copysign(ooeps, dir.y));
    float idirz = 1.0f / (fabsf(dir.z) > ooeps ? dir.z : o_copysign(ooeps, dir.z));
    float origx = ori.x, origy = ori.y, origz = ori.z;
    float oodx = origx * idirx, oody = origy * idiry, oodz = origz * idirz;
    int sp = 1;
    int leafAddr = 0;
    int nodeAddr = startNode;
    while (nodeAddr != EntrypointSentinel) {
        while ((unsigned int)nodeAddr < (unsigned int)EntrypointSentinel) {
            const float* n = nodes4 + 4 * (size_t)(bvhNodesOffset + nodeAddr);
            if (st) st->nodes++;
            const float tc = cullFloor > rayT ? cullFloor : rayT;
            int c0i, c1i;
            std::memcpy(&c0i, n + 12, 4);
            std::memcpy(&c1i, n + 13, 4);
            const float c0lox = n[0] * idirx - oodx;
            const float c0hix = n[1] * idirx - oodx;
            const float c0loy = n[2] * idiry - oody;
            const float c0hiy = n[3] * idiry - oody;
            const float c0loz = n[8] * idirz - oodz;
            const float c0hiz = n[9] * idirz - oodz;
            const float c1loz = n[10] * idirz - oodz;
            const float c1hiz = n[11] * idirz - oodz;
            const float c0min = spanBegin(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, spanTmin);
            const float c0max = spanEnd(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, tc);
            const float c1lox = n[4] * idirx - oodx;
            const float c1hix = n[5] * idirx - oodx;
            const float c1loy = n[6] * idiry - oody;
            const float c1hiy = n[7] * idiry - oody;
            const float c1min = spanBegin(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, spanTmin);
            const float c1max = spanEnd(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, tc);
            bool swp = (c1min < c0min);
            bool traverseChild0 = (c0max >= c0min);
            bool traverseChild1 = (c1max >= c1min);
            if (!traverseChild0 && !traverseChild1) {
                nodeAddr = traversalStack[sp--];
            } else {
                nodeAddr = traverseChild0 ? c0i : c1i;
                if (traverseChild0 && traverseChild1) {
                    if (swp) std::swap(nodeAddr, c1i);
                    traversalStack[++sp] = c1i;
                    if (sp > 65) { std::fprintf(stderr, "oracle: traversal stack overflow\n"); std::abort(); }
                }
            }
            if (nodeAddr < 0 && leafAddr >= 0) {
                leafAddr = nodeAddr;
                nodeAddr = traversalStack[sp--];
            }
            if (!(leafAddr >= 0)) break;   // host branch: mask = leafAddr >= 0
        }
        while (leafAddr < 0) {
            if (leafAddr != -214783648) found |= clb(~leafAddr);   // sic, BVHTraversal.h:221
            leafAddr = nodeAddr;
            if (nodeAddr < 0) nodeAddr = traversalStack[sp--];
        }
    }
    return found;
}

// ---------------------------------------------------------------------------
// Scene view (the ctl_scene_desc arrays)
// ---------------------------------------------------------------------------
struct SceneView {
    const ctl_scene_desc* d;
    M44 xf(uint32_t i) const { M44 m; std::memcpy(m.d, d->node_xf[i].m, 64); return m; }
    M44 inv(uint32_t i) const { M44 m; std::memcpy(m.d, d->node_inv_xf[i].m, 64); return m; }
    bool quirk() const { return (d->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0; }
};

// Traversal modes: TIE_FIRST_FOUND = the reference's binary visit order
// (BVHTraversal.h host branch, TraceHelper.cu:121); TRAVERSE_WIDE = the
// product's 4-wide per-ray order (trace_two_level_wide) over the 4-wide trees
// registered with oracle_set_wide.  (Mode 1, round 3's tie rule, and mode 3,
// round 4's 8-wide order, are retired: probes/round4_variants.patch.)
enum TieMode { TIE_FIRST_FOUND = 0, TRAVERSE_WIDE = 2 };

struct Hit {
    float t; float u, v; uint32_t tri; uint32_t node;
};

// Generic two-level closest/any hit.  traceRay (TraceHelper.cu:88-180):
// spanTmin=0, triTmin=rayEps, t0=FLT_MAX.  Batch (TraceHelper.cu:326-734):
// spanTmin=triTmin=ray.tmin, t0=ray.tmax.
// Material::AlphaTest of a candidate hit (TraceHelper.cu:136-154), defined
// after oracle_c5.h; used by the traceRay flavour only (alpha = true).
bool alpha_survives(const ctl_scene_desc* d, uint32_t gtri, uint32_t nodeIdx, float u, float v);
bool scene_has_alpha(const ctl_scene_desc* d) {   // DynamicScene.cpp:586 doAlphaMapping
    for (uint32_t i = 0; i < d->n_materials; i++)
        if (d->materials[i].alpha_state) return true;
    return false;
}

// Box culling of the any-hit shadow query (occluded_query): CULL_SLAB is the
// product's rule, dist + slab_slack of each level's ray; the others are
// measured alternatives (tests/test_shadow_query.py).
enum ShadowCull { CULL_AT_ACCEPT = 0, CULL_AT_TMAX = 1, CULL_AT_INF = 2, CULL_SLAB = 3 };

// DevScene::cull_m (device/traverse.h cull_bound): per axis, max |coordinate| of
// the scene box and of every mesh's local box.
void cull_bound(const ctl_scene_desc* d, float m[3]) {
    for (int a = 0; a < 3; a++) {
        float v = fabsf(d->box_min[a]) > fabsf(d->box_max[a]) ? fabsf(d->box_min[a]) : fabsf(d->box_max[a]);
        for (uint32_t i = 0; d->mesh_boxes && i < d->n_meshes; i++) {
            const float l = fabsf(d->mesh_boxes[6 * i + a]), hh = fabsf(d->mesh_boxes[6 * i + 3 + a]);
            v = l > v ? l : v;
            v = hh > v ? hh : v;
        }
        m[a] = v;
    }
}

// device/traverse.h slab_slack: 2^-20 max_a (|o_a| + m_a) |idir_a|, a bound (with
// margin) on the rounding of the slab distances lo * idir - o * idir of this ray.
float slab_slack(V3 o, V3 d, const float m[3]) {
    const float ooeps = powf(2.0f, -80.0f);
    const float idx = 1.0f / (fabsf(d.x) > ooeps ? d.x : o_copysign(ooeps, d.x));
    const float idy = 1.0f / (fabsf(d.y) > ooeps ? d.y : o_copysign(ooeps, d.y));
    const float idz = 1.0f / (fabsf(d.z) > ooeps ? d.z : o_copysign(ooeps, d.z));
    const float ex = (fabsf(o.x) + m[0]) * fabsf(idx);
    const float ey = (fabsf(o.y) + m[1]) * fabsf(idy);
    const float ez = (fabsf(o.z) + m[2]) * fabsf(idz);
    const float e = ex > ey ? ex : ey;
    return (e > ez ? e : ez) * powf(2.0f, -20.0f);
}

// The cull distance of an any-hit query's BVH level whose ray is (o, d), at
// least its acceptance bound; mode < 0 (every closest-hit query, a plain
// any-hit query): the acceptance bound itself, i.e. the current hit.
struct AnyCull {
    int mode = -1;
    float dist = 0.0f;
    float m[3] = {0.0f, 0.0f, 0.0f};
    float at(V3 o, V3 d, float accept) const {
        float c = accept;
        switch (mode) {
            case CULL_AT_TMAX: c = dist; break;
            case CULL_AT_INF: c = INFINITY; break;
            case CULL_SLAB: c = dist + slab_slack(o, d, m); break;
            default: break;
        }
        return c > accept ? c : accept;
    }
    // traceray_template's cullFloor: 0 (none) unless this is a shadow query
    float floor(V3 o, V3 d, float accept) const { return mode < 0 ? 0.0f : at(o, d, accept); }
};

bool trace_two_level_wide(const SceneView& S, V3 ori, V3 dir, float spanTmin, float triTmin, Hit& h, bool anyHit,
                          Stats* st, bool alpha, const AnyCull& ac);

// ac (any-hit only): the shadow query's per-level cull distance (AnyCull).
bool trace_two_level(const SceneView& S, V3 ori, V3 dir, float spanTmin, float triTmin, Hit& h, bool anyHit,
                     int tie, Stats* st, bool alpha = false, const AnyCull& ac0 = AnyCull()) {
    const AnyCull ac = anyHit ? ac0 : AnyCull();
    if (tie == TRAVERSE_WIDE) return trace_two_level_wide(S, ori, dir, spanTmin, triTmin, h, anyHit, st, alpha, ac);
    const ctl_scene_desc* d = S.d;
    if (d->n_nodes == 0) return false;
    const float* sceneNodes = reinterpret_cast<const float*>(d->scene_bvh_nodes);
    const float* meshNodes = reinterpret_cast<const float*>(d->bvh_nodes);
    const float* tris = reinterpret_cast<const float*>(d->woop_tris);
    bool done = false;   // any-hit termination
    auto instClb = [&](int nodeIdx) -> bool {
        if (done) return false;
        if (st) st->inst++;
        const ctl_node& N = d->nodes[nodeIdx];
        const ctl_kernel_mesh& mesh = d->meshes[N.mesh_index];
        M44 modl = S.inv(nodeIdx);
        V3 dl = transformDirection(modl, dir), ol = transformPoint(modl, ori);
        auto triClb = [&](int triIdx) -> bool {
            bool found = false;
            for (int triAddr = triIdx;; triAddr++) {
                if (done) break;
                const float* v = tris + 4 * ((size_t)mesh.bvh_triangle_offset + (size_t)triAddr * 3);
                unsigned int index = d->tri_indices[mesh.bvh_indices_offset + triAddr];
                if (st) st->tris++;
                float Oz = v[3] - ol.x * v[0] - ol.y * v[1] - ol.z * v[2];
                float invDz = 1.0f / (dl.x * v[0] + dl.y * v[1] + dl.z * v[2]);
                float t = Oz * invDz;
                unsigned int gtri = (index >> 1) + mesh.triangle_offset;
                if (t > triTmin && t < h.t) {
                    float Ox = v[7] + ol.x * v[4] + ol.y * v[5] + ol.z * v[6];
                    float Dx = dl.x * v[4] + dl.y * v[5] + dl.z * v[6];
                    float u = Ox + t * Dx;
                    if (u >= 0.0f) {
                        float Oy = v[11] + ol.x * v[8] + ol.y * v[9] + ol.z * v[10];
                        float Dy = dl.x * v[8] + dl.y * v[9] + dl.z * v[10];
                        float vv = Oy + t * Dy;
                        if (vv >= 0.0f && u + vv <= 1.0f && (!alpha || alpha_survives(d, gtri, (uint32_t)nodeIdx, u, vv))) {
                            h.node = (uint32_t)nodeIdx;
                            h.tri = gtri;
                            h.u = u; h.v = vv;
                            h.t = t;
                            found = true;
                            if (anyHit) { done = true; break; }
                        }
                    }
                }
                if (index & 1) break;
            }
            return found;
        };
        return traceray_template(ol, dl, h.t, spanTmin, triClb, meshNodes, (int)mesh.bvh_node_offset, 0, st,
                                 ac.floor(ol, dl, h.t));
    };
    return traceray_template(ori, dir, h.t, spanTmin, instClb, sceneNodes, 0, d->scene_start_node, st,
                             ac.floor(ori, dir, h.t));
}

// ---------------------------------------------------------------------------
// The product's 4-wide per-ray order (NOT a reference function).
//
// The default device traversal (cudatracerlib_amd/csrc/device/traverse.h,
// Traverser<..., WIDE>) walks 4-wide trees collapsed from the reference's
// binary ones (host/bvh_wide.h) in its own order.  This is a sequential
// statement of that order, so the GPU path can be held to it bit for bit; how
// far it lands from the reference's binary order (trace_two_level, tie 0) is
// measured separately (tests/test_reference_order.py).  The trees themselves
// are inputs, registered per scene with oracle_set_wide (read back from the
// device or built by the library's host collapse), like the binary arrays.
//
// Order: per node the slabs of the four children (near/far plane chosen by the
// sign of idir), entry/exit spans as kepler_math on the fp32 bits, children
// whose span is non-empty against `tcull` sorted near-first by a fixed
// 5-comparator network, the nearest taken, the rest pushed far-to-near, one
// leaf postponed.  Inside a mesh a lane holding a postponed leaf keeps walking
// (with the same tcull) until it reaches its next leaf; then the postponed
// leaf, that leaf and any leaves stacked right behind it are tested, and
// tcull becomes the closest hit.  The instance level stops at its first leaf.
// Woop test and first-found ties exactly as TraceHelper.cu:118-161.
// ---------------------------------------------------------------------------
struct WideTrees {
    const void* key_nodes = nullptr;   // the desc arrays the trees were built for
    const void* key_scene = nullptr;
    uint64_t key_n = 0;
    std::vector<float> mesh;           // 32 floats (128 B) per node: lo_x hi_x lo_y hi_y lo_z hi_z child pad
    std::vector<uint32_t> wbase;       // first node of each mesh's tree
    std::vector<float> scene;          // the instance tree (root at node 0)
    bool set = false;
};
WideTrees g_wide;
std::mutex g_wide_mtx;

const WideTrees& wide_trees_for(const ctl_scene_desc* d) {
    if (!g_wide.set || g_wide.key_nodes != (const void*)d->bvh_nodes || g_wide.key_n != d->n_bvh_nodes ||
        g_wide.key_scene != (const void*)d->scene_bvh_nodes || g_wide.wbase.size() < d->n_meshes) {
        std::fprintf(stderr, "oracle: TRAVERSE_WIDE without 4-wide trees registered for this scene (oracle_set_wide)\n");
        std::abort();
    }
    return g_wide;
}

struct WRay {
    float ox, oy, oz, dx, dy, dz, idx, idy, idz, oodx, oody, oodz;
    void set(V3 o, V3 d) {
        ox = o.x; oy = o.y; oz = o.z; dx = d.x; dy = d.y; dz = d.z;
        const float ooeps = powf(2.0f, -80.0f);   // TraceHelper.cu:412
        idx = 1.0f / (fabsf(d.x) > ooeps ? d.x : o_copysign(ooeps, d.x));
        idy = 1.0f / (fabsf(d.y) > ooeps ? d.y : o_copysign(ooeps, d.y));
        idz = 1.0f / (fabsf(d.z) > ooeps ? d.z : o_copysign(ooeps, d.z));
        oodx = ox * idx; oody = oy * idy; oodz = oz * idz;
    }
};

bool trace_two_level_wide(const SceneView& S, V3 ori, V3 dir, float spanTmin, float triTmin, Hit& h, bool anyHit,
                          Stats* st, bool alpha, const AnyCull& ac) {
    const ctl_scene_desc* d = S.d;
    if (d->n_nodes == 0) return false;
    const WideTrees& W = wide_trees_for(d);
    const float* tris = reinterpret_cast<const float*>(d->woop_tris);
    const bool single = d->scene_start_node < 0;
    std::vector<int> stack;
    stack.reserve(64);
    stack.push_back(EntrypointSentinel);
    auto pop = [&]() -> int {
        if (stack.empty()) return EntrypointSentinel;
        const int v = stack.back();
        stack.pop_back();
        return v;
    };
    WRay world, cur;
    world.set(ori, dir);
    cur = world;
    int level = 0, nodeAddr = 0, leafAddr = 0;
    size_t meshSent = 0;
    uint32_t wnodeBase = 0, triBase = 0, idxBase = 0, triOffset = 0, inst = 0;
    // any-hit: h.t only changes when the query ends; the cull distance is the
    // level's (ac.at of the world ray, then of each instance's ray)
    const float accept = h.t;
    float cullAny = ac.at(v3(world.ox, world.oy, world.oz), v3(world.dx, world.dy, world.dz), accept);
    float tcull = cullAny;
    const int tminBits = as_int(spanTmin);
    bool found = false;
    auto enter = [&](uint32_t node) {   // TraceHelper.cu:91-100
        if (st) st->inst++;
        inst = node;
        const ctl_node& N = d->nodes[node];
        const ctl_kernel_mesh& M = d->meshes[N.mesh_index];
        wnodeBase = W.wbase[N.mesh_index];
        triBase = M.bvh_triangle_offset; idxBase = M.bvh_indices_offset; triOffset = M.triangle_offset;
        M44 modl = S.inv(node);
        cur.set(transformPoint(modl, v3(world.ox, world.oy, world.oz)),
                transformDirection(modl, v3(world.dx, world.dy, world.dz)));
        cullAny = ac.at(v3(cur.ox, cur.oy, cur.oz), v3(cur.dx, cur.dy, cur.dz), accept);   // the mesh's ray
    };
    // one Woop test (TraceHelper.cu:118-161); true = any-hit termination
    auto test = [&](uint32_t e) -> bool {
        const float* v = tris + 4 * ((size_t)triBase + (size_t)e * 3);
        const uint32_t index = d->tri_indices[idxBase + e];
        if (st) st->tris++;
        float Oz = v[3] - cur.ox * v[0] - cur.oy * v[1] - cur.oz * v[2];
        float invDz = 1.0f / (cur.dx * v[0] + cur.dy * v[1] + cur.dz * v[2]);
        float t = Oz * invDz;
        if (t > triTmin && t < h.t) {
            float Ox = v[7] + cur.ox * v[4] + cur.oy * v[5] + cur.oz * v[6];
            float Dx = cur.dx * v[4] + cur.dy * v[5] + cur.dz * v[6];
            float u = Ox + t * Dx;
            if (u >= 0.0f) {
                float Oy = v[11] + cur.ox * v[8] + cur.oy * v[9] + cur.oz * v[10];
                float Dy = cur.dx * v[8] + cur.dy * v[9] + cur.dz * v[10];
                float vv = Oy + t * Dy;
                const uint32_t gtri = (index >> 1) + triOffset;
                if (vv >= 0.0f && u + vv <= 1.0f && (!alpha || alpha_survives(d, gtri, inst, u, vv))) {
                    h.node = inst; h.tri = gtri; h.u = u; h.v = vv; h.t = t;
                    found = true;
                    if (anyHit) return true;
                }
            }
        }
        return false;
    };
    // a counted leaf child ~((first << 3) | count), count 0 = walk the last-in-leaf flags
    auto leaf = [&](int value) -> bool {
        const uint32_t code = (uint32_t)~value;
        const uint32_t first = code >> 3, cnt = code & 7u;
        if (first == 214783647u) return false;   // the reference's skipped leaf value (BVHTraversal.h:221)
        if (cnt == 0) {
            for (uint32_t e = first;; e++) {
                if (test(e)) return true;
                if (d->tri_indices[idxBase + e] & 1u) break;
            }
            return false;
        }
        for (uint32_t i = 0; i < cnt; i++)
            if (test(first + i)) return true;
        return false;
    };
    if (single) {
        enter(~(uint32_t)d->scene_start_node);
        level = 1;
        tcull = cullAny;
    }
    for (;;) {
        const bool spec = level == 1;
        const float* tree = level ? W.mesh.data() + 32 * (size_t)wnodeBase : W.scene.data();
        const int tBits = as_int(tcull);
        const bool nx = as_int(cur.idx) < 0, ny = as_int(cur.idy) < 0, nz = as_int(cur.idz) < 0;
        while ((unsigned)nodeAddr < (unsigned)EntrypointSentinel && (spec || leafAddr >= 0)) {
            if (st) st->nodes++;
            const float* n = tree + 32 * (size_t)nodeAddr;
            int k[4], c[4];
            for (int i = 0; i < 4; i++) {
                const float lx = n[i], hx = n[4 + i], ly = n[8 + i], hy = n[12 + i], lz = n[16 + i], hz = n[20 + i];
                const float nX = (nx ? hx : lx) * cur.idx - cur.oodx, fX = (nx ? lx : hx) * cur.idx - cur.oodx;
                const float nY = (ny ? hy : ly) * cur.idy - cur.oody, fY = (ny ? ly : hy) * cur.idy - cur.oody;
                const float nZ = (nz ? hz : lz) * cur.idz - cur.oodz, fZ = (nz ? lz : hz) * cur.idz - cur.oodz;
                const float cmin = as_float(imax3(as_int(nX), as_int(nY), omax(as_int(nZ), tminBits)));
                const float cmax = as_float(imin3(as_int(fX), as_int(fY), omin(as_int(fZ), tBits)));
                k[i] = (cmax >= cmin) ? as_int(cmin) : 0x7fffffff;
                std::memcpy(&c[i], n + 24 + i, 4);
            }
            auto cx = [&](int a, int b) {
                if (k[b] < k[a]) { std::swap(k[a], k[b]); std::swap(c[a], c[b]); }
            };
            cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
            int m = 0;
            for (int i = 0; i < 4; i++) m += k[i] != 0x7fffffff;
            for (int i = m - 1; i >= 1; i--) stack.push_back(c[i]);
            int next = m > 0 ? c[0] : pop();
            if (next < 0 && leafAddr >= 0) {   // postpone one leaf
                leafAddr = next;
                next = pop();
            }
            nodeAddr = next;
        }
        bool entered = false;
        while (leafAddr < 0) {
            if (level == 1) {
                if (leaf(leafAddr)) return true;
                leafAddr = nodeAddr;
                if (nodeAddr < 0) nodeAddr = pop();
            } else {
                if (leafAddr != -214783648) {
                    enter((uint32_t)~leafAddr);
                    stack.push_back(nodeAddr);   // pending top-level work
                    meshSent = stack.size();
                    stack.push_back(EntrypointSentinel);
                    level = 1;
                    nodeAddr = 0;
                    leafAddr = 0;
                    entered = true;
                    break;
                }
                leafAddr = nodeAddr;
                if (nodeAddr < 0) nodeAddr = pop();
            }
        }
        tcull = anyHit ? cullAny : h.t;
        if (entered) continue;
        if (nodeAddr == EntrypointSentinel) {
            if (level == 1 && !single) {
                stack.resize(meshSent);
                const int saved = pop();
                level = 0;
                cur = world;
                cullAny = ac.at(v3(world.ox, world.oy, world.oz), v3(world.dx, world.dy, world.dz), accept);
                if (anyHit) tcull = cullAny;
                leafAddr = saved;
                nodeAddr = saved;
                if (saved < 0) nodeAddr = pop();
            } else {
                break;
            }
        }
    }
    return found;
}

// traceRay(dir, ori, TraceResult*) (TraceHelper.cu:174-180) on an Init()'ed result
bool trace_ray(const SceneView& S, V3 ori, V3 dir, Hit& h, int tie, Stats* st) {
    h.t = FLT_MAX; h.tri = UINT_MAX; h.node = UINT_MAX; h.u = h.v = 0;
    trace_two_level(S, ori, dir, 0.0f, S.d->ray_eps, h, false, tie, st, scene_has_alpha(S.d));
    return h.tri != UINT_MAX;
}

// ---------------------------------------------------------------------------
// XORWOW / CudaRNG (Base/CudaRandom.h:112-282, CudaRandom.cu:8-36)
// curand_init(1234, subsequence, 0): subsequence jump = 2^67 steps (published
// cuRAND XORWOW definition).  Jumps use powers of the GF(2) step matrix.
// ---------------------------------------------------------------------------
struct Xorwow { uint32_t v[5]; uint32_t d; };

struct Gf2 { uint32_t col[160][5]; };
void gf2_apply(const Gf2& M, const uint32_t x[5], uint32_t y[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < 160; j++)
        if ((x[j >> 5] >> (j & 31)) & 1u)
            for (int k = 0; k < 5; k++) r[k] ^= M.col[j][k];
    for (int k = 0; k < 5; k++) y[k] = r[k];
}
void xorwow_linear_step(uint32_t v[5]) {
    uint32_t t = (v[0] ^ (v[0] >> 2));
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}
const std::vector<Gf2>& gf2_powers() {   // P[k] = M^(2^k), k < 128
    static std::vector<Gf2> P;
    static std::once_flag once;
    std::call_once(once, [] {
        P.resize(128);
        for (int j = 0; j < 160; j++) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j >> 5] = 1u << (j & 31);
            xorwow_linear_step(v);
            for (int k = 0; k < 5; k++) P[0].col[j][k] = v[k];
        }
        for (int p = 1; p < 128; p++)
            for (int j = 0; j < 160; j++) gf2_apply(P[p - 1], P[p - 1].col[j], P[p].col[j]);
    });
    return P;
}
Xorwow curand_init(uint64_t seed, uint64_t subsequence, uint64_t offset) {
    Xorwow s;
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49UL;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddUL;
    uint32_t t0 = 1099087573UL * s0;
    uint32_t t1 = 2591861531UL * s1;
    s.d = 6615241 + t1 + t0;
    s.v[0] = 123456789UL + t0;
    s.v[1] = 362436069UL ^ t0;
    s.v[2] = 521288629UL + t1;
    s.v[3] = 88675123UL ^ t1;
    s.v[4] = 5783321UL + t0;
    const auto& P = gf2_powers();
    for (int b = 0; b < 64; b++)
        if ((subsequence >> b) & 1) gf2_apply(P[67 + b], s.v, s.v);
    for (int b = 0; b < 64; b++)
        if ((offset >> b) & 1) gf2_apply(P[b], s.v, s.v);
    s.d += 362437u * (uint32_t)offset;
    return s;
}
inline uint32_t xorwow_next(Xorwow& s) {   // curand2 (CudaRandom.h:118-129)
    uint32_t t = (s.v[0] ^ (s.v[0] >> 2));
    s.v[0] = s.v[1]; s.v[1] = s.v[2]; s.v[2] = s.v[3]; s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437;
    return s.v[4] + s.d;
}
inline float xorwow_uniform(Xorwow& s) {   // randomFloat (CudaRandom.cu:8-17)
    const float INV = 2.3283064e-10f;       // CURAND_2POW32_INV
    float f = (float)xorwow_next(s) * INV + (INV / 2.0f);
    return f * (1 - 1e-5f);
}

const uint32_t kSamplerSeed = 7539414;       // IndependantSamplingSequenceGenerator (Sampler.h:68)
void sampler_tables(uint64_t pass, uint32_t nseq, uint32_t len, float* seq1d, float* seq2d) {
    // One CudaRNG stream continued across passes (Sampler.h:36-55,63-85):
    // per sequence `len` 1-D draws then `len` 2-D pairs (x drawn first).
    uint64_t perPass = (uint64_t)nseq * len * 3;
    Xorwow s = curand_init(1234, kSamplerSeed, pass * perPass);
    for (uint32_t q = 0; q < nseq; q++) {
        for (uint32_t i = 0; i < len; i++) seq1d[(size_t)i * nseq + q] = xorwow_uniform(s);
        for (uint32_t i = 0; i < len; i++) {
            float x = xorwow_uniform(s);
            float y = xorwow_uniform(s);
            seq2d[2 * ((size_t)i * nseq + q) + 0] = x;
            seq2d[2 * ((size_t)i * nseq + q) + 1] = y;
        }
    }
}

struct Sampler {   // SequenceSampler (Sampler_device.h:59-113)
    const float* s1; const float* s2; uint32_t nseq, len;
    uint32_t idx, d1 = 0, d2 = 0;
    float randomFloat() {
        uint32_t k = d1 % len;
        float val = 0.0f;
        val += s1[(size_t)k * nseq + idx % nseq];
        val += s1[(size_t)k * nseq + (idx / nseq) % nseq];
        d1++;
        return frac(val);
    }
    V2 randomFloat2() {
        uint32_t k = d2 % len;
        size_t a = (size_t)k * nseq + idx % nseq, b = (size_t)k * nseq + (idx / nseq) % nseq;
        float x = 0.0f, y = 0.0f;
        x += s2[2 * a]; y += s2[2 * a + 1];
        x += s2[2 * b]; y += s2[2 * b + 1];
        d2++;
        return v2(frac(x), frac(y));
    }
};

// ---------------------------------------------------------------------------
// Shading (diffuse + DiffuseLight), EXT_TRI TriangleData
// ---------------------------------------------------------------------------
using Spec = V3;   // RGB Spectrum, SPECTRUM_SAMPLES 3 (Math/Spectrum.h:10)
inline float spec_max(Spec s) { float r = s.x; r = omax(r, s.y); r = omax(r, s.z); return r; }
inline bool spec_zero(Spec s) { return s.x == 0.0f && s.y == 0.0f && s.z == 0.0f; }
inline Spec spec_div(Spec s, float f) { float recip = 1.0f / f; return s * recip; }   // Spectrum.h:122-128

struct DG {   // DifferentialGeometry subset
    V3 P; Frame sys; V3 n; V3 dpdu, dpdv; V2 bary;
    V2 uv;                                   // uv[0]
    float dudx = 0, dudy = 0, dvdx = 0, dvdy = 0;
    bool hasUVPartials = false;              // set by computePartials, never reset (PathTracer.cu:16,60)
};

void fill_dg(const SceneView& S, V2 bary, uint32_t triIdx, uint32_t nodeIdx, DG& dg, bool quirk) {
    // TriangleData::fillDG (Engine/TriangleData.cu:75-103) via fillDG (TraceHelper.cu:274-307)
    M44 L2W = S.xf(nodeIdx);
    dg.bary = bary;
    const uint32_t* w = S.d->tri_data[triIdx].w;
    auto hf = [&](uint16_t h) { return quirk ? half_to_float_host(h) : half_to_float_ieee(h); };
    V3 na = normal_decode((uint16_t)(w[0] & 0xffff)), nb = normal_decode((uint16_t)(w[0] >> 16)),
       nc = normal_decode((uint16_t)(w[1] & 0xffff));
    float ww = 1.0f - dg.bary.x - dg.bary.y, u = dg.bary.x, v = dg.bary.y;
    V3 n = normalize(u * na + v * nb + ww * nc);
    V3 dpdu = v3(hf(w[2] & 0xffff), hf(w[2] >> 16), hf(w[3] & 0xffff));
    V3 dpdv = v3(hf(w[3] >> 16), hf(w[4] & 0xffff), hf(w[4] >> 16));
    V3 s = dpdu - n * dot(n, dpdu);
    V3 t = cross(s, n);
    s = transformDirection(L2W, s); t = transformDirection(L2W, t);
    dg.sys.s = normalize(s); dg.sys.t = normalize(t); dg.sys.n = normalize(cross(t, s));
    dg.dpdu = transformDirection(L2W, dpdu);
    dg.dpdv = transformDirection(L2W, dpdv);
    dg.n = normalize(cross(dg.dpdu, dg.dpdv));
    V2 ta = v2(hf(w[5] & 0xffff), hf(w[5] >> 16)), tb = v2(hf(w[6] & 0xffff), hf(w[6] >> 16)),
       tc = v2(hf(w[7] & 0xffff), hf(w[7] >> 16));
    dg.uv = u * ta + v * tb + ww * tc;
    if (dot(dg.n, dg.sys.n) < 0.0f) dg.n = -dg.n;
}

struct BRec {   // BSDFSamplingRecord subset
    DG dg; V3 wi, wo; uint32_t sampledType; uint32_t typeMask;
};

const uint32_t EAll = 0x1ff, EDelta = 0x61, ESmooth = 0x1e;

uint32_t mat_index(const SceneView& S, uint32_t tri, uint32_t node) {   // TraceResult.cu:83-86
    return ((S.d->tri_data[tri].w[1] >> 16) & 0xff) + S.d->nodes[node].material_offset;
}
uint32_t light_index(const SceneView& S, uint32_t tri, uint32_t node) {  // TraceResult.cu:53-59
    const ctl_material& m = S.d->materials[mat_index(S, tri, node)];
    if (m.node_light_index == UINT_MAX) return UINT_MAX;
    return S.d->nodes[node].lights[m.node_light_index];
}

}  // namespace
#include "oracle_c5.h"
namespace {

// Material::AlphaTest (Engine/Material.cu:160-189) with sample_fast (:140-158)
// and KernelMIPMap::SampleAlpha (MIPMap.cu:123-139, index clamped).
bool alpha_survives(const ctl_scene_desc* d, uint32_t gtri, uint32_t nodeIdx, float u, float v) {
    const uint32_t* w = d->tri_data[gtri].w;
    const ctl_material& m = d->materials[((w[1] >> 16) & 0xff) + d->nodes[nodeIdx].material_offset];
    if (!m.alpha_state) return true;
    const bool q = (d->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0;
    auto hf = [&](uint16_t x) { return q ? half_to_float_host(x) : half_to_float_ieee(x); };
    V2 a = v2(hf(w[5] & 0xffff), hf(w[5] >> 16)), b = v2(hf(w[6] & 0xffff), hf(w[6] >> 16)),
       c = v2(hf(w[7] & 0xffff), hf(w[7] >> 16));
    V2 uv = u * a + v * b + (1 - u - v) * c;
    auto mapped = [&](const ctl_texture* t) {
        return v2(t->m11 * uv.x + t->m12 * uv.y, t->m21 * uv.x + t->m22 * uv.y) + v2(t->m13, t->m23);
    };
    const ctl_texture* refl_img = m.texture != UINT_MAX ? d->textures + m.texture : nullptr;
    const ctl_texture* alpha_img = m.alpha_texture != UINT_MAX ? d->textures + m.alpha_texture : nullptr;
    if ((m.alpha_state == 2 && alpha_img) || (m.alpha_state == 6 && refl_img)) {
        const ctl_texture* t = m.alpha_state == 2 ? alpha_img : refl_img;
        V2 l;
        if (!c5::wrap_coords(mapped(t), v2((float)t->width, (float)t->height), t->wrap, &l)) return 0.0f >= m.alpha_threshold;
        uint32_t x = omin((uint32_t)l.x, t->width - 1), y = omin((uint32_t)l.y, t->height - 1);
        float alpha = float(d->tex_data[t->offsets[0] + y * t->width + x] >> 24) / 255.0f;
        return alpha >= m.alpha_threshold;
    }
    const ctl_texture* src = (m.alpha_state & 4) ? refl_img : alpha_img;
    Spec val;
    if (src) {
        c5::Mip M{src, d->tex_data};
        V2 u2 = mapped(src);
        val = (src->filter == CTL_TEX_POINT ? c5::texel(M, 0, u2) : c5::triangle(M, 0, u2)) *
              v3(src->scale[0], src->scale[1], src->scale[2]);
    } else {
        val = v3(m.reflectance[0], m.reflectance[1], m.reflectance[2]);
    }
    if ((m.alpha_state & 3) == 1) return val.x * 0.212671f + val.y * 0.715160f + val.z * 0.072169f >= m.alpha_threshold;
    return true;
}

// diffuse::m_reflectance.Evaluate(bRec.dg): ConstantTexture or ImageTexture
Spec diffuse_R(const ctl_scene_desc* d, const ctl_material& m, const DG& dg) {
    if (m.texture != UINT_MAX) return c5::image_eval(d->textures + m.texture, d->tex_data, dg);
    return v3(m.reflectance[0], m.reflectance[1], m.reflectance[2]);
}

// diffuse (BSDF_Simple.cu:7-75) under BSDFALL two-sided wrapper (BSDF.h:147-208)
Spec diffuse_sample(const ctl_scene_desc* d, const ctl_material& m, BRec& b, float& pdf, V2 sample) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    Spec res;
    if (!(b.typeMask & m.combined_type) || (m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z <= 0)) {
        res = v3s(0.0f);
    } else {
        b.sampledType = m.combined_type;
        // Warp::squareToCosineHemisphere (Warp.h:61-66) + concentric disk (Warp.h:102-125)
        float r1 = 2.0f * sample.x - 1.0f, r2 = 2.0f * sample.y - 1.0f;
        float phi, r;
        if (r1 == 0 && r2 == 0) { r = phi = 0; }
        else if (r1 * r1 > r2 * r2) { r = r1; phi = (O_PI / 4.0f) * (r2 / r1); }
        else { r = r2; phi = (O_PI / 2.0f) - (r1 / r2) * (O_PI / 4.0f); }
        float sinPhi = cr_sin(phi), cosPhi = cr_cos(phi);
        V2 p = v2(r * cosPhi, r * sinPhi);
        float z = sqrtf(1.0f - p.x * p.x - p.y * p.y);
        b.wo = v3(p.x, p.y, z);
        pdf = fabsf(O_INV_PI * b.wo.z) * 1.0f;
        res = diffuse_R(d, m, b.dg) * 1.0f;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}
Spec diffuse_f(const ctl_scene_desc* d, const ctl_material& m, BRec& b) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    Spec res = v3s(0.0f);
    if (b.typeMask & m.combined_type) {
        bool validRefl = m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z > 0 && b.wo.z > 0;
        bool validTrans = m.combined_type == CTL_EDIFFUSE_TRANSMISSION && b.wi.z * b.wo.z < 0;
        Spec s = diffuse_R(d, m, b.dg) * (O_INV_PI * fabsf(b.wo.z));
        if (validRefl || validTrans) res = s;
        else if (m.combined_type == (CTL_EDIFFUSE_REFLECTION | CTL_EDIFFUSE_TRANSMISSION)) res = s * 0.5f;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}
float diffuse_pdf(const ctl_material& m, BRec& b) {
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    float res = 0.0f;
    if (b.typeMask & m.combined_type) {
        bool validRefl = m.combined_type == CTL_EDIFFUSE_REFLECTION && b.wi.z > 0 && b.wo.z > 0;
        bool validTrans = m.combined_type == CTL_EDIFFUSE_TRANSMISSION && b.wi.z * b.wo.z < 0;
        float f = fabsf(O_INV_PI * b.wo.z);
        if (validRefl || validTrans) res = f;
        else if (m.combined_type == (CTL_EDIFFUSE_REFLECTION | CTL_EDIFFUSE_TRANSMISSION)) res = f * 0.5f;
    }
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return res;
}

// BSDFALL::sample / f / pdf (BSDF.h:140-208): the type switch; diffuse does its
// own two-sided flip above, roughdielectric gets the wrapper here.
Spec bsdf_sample(const ctl_scene_desc* d, const ctl_material& m, BRec& b, float& pdf, V2 sample) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) return diffuse_sample(d, m, b, pdf, sample);
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    Spec r = c5::rough_sample(m, b, pdf, sample);
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return r;
}
Spec bsdf_f(const ctl_scene_desc* d, const ctl_material& m, BRec& b) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) return diffuse_f(d, m, b);
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    Spec r = c5::rough_f(m, b);
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return r;
}
float bsdf_pdf(const ctl_scene_desc*, const ctl_material& m, BRec& b) {
    if (m.bsdf_type == CTL_BSDF_DIFFUSE) return diffuse_pdf(m, b);
    bool flip = b.wi.z < 0 && m.two_sided;
    if (flip) b.wi.z *= -1.0f;
    float r = c5::rough_pdf(m, b);
    if (flip) { b.wi.z *= -1.0f; b.wo.z *= -1.0f; }
    return r;
}

struct DRec {   // DirectSamplingRecord
    V3 p; V3 n; float pdf; int measure; V2 uv; V3 ref; V3 refN; V3 d; float dist;
};
const int ESolidAngle = 1, EArea = 3, EDiscrete = 4;

// MonteCarlo::sampleReuse (Math/MonteCarlo.cu:7-14) with STL_lower_bound (Base/STL.h:39-56)
uint32_t sample_reuse(const float* cdf, uint32_t size, float& sample, float& pdf) {
    const float* first = cdf;
    uint32_t count = size + 1;
    while (count > 0) {
        uint32_t c2 = count / 2;
        const float* mid = first + c2;
        if (*mid < sample) { first = ++mid; count -= c2 + 1; }
        else count = c2;
    }
    uint32_t index = (uint32_t)omin(omax(0, int(first - cdf) - 1), int(size - 1));
    pdf = cdf[index + 1] - cdf[index];
    sample = (sample - cdf[index]) / pdf;
    return index;
}

// DiffuseLight::sampleDirect, non-orthogonal (Light.cu:84-135) + ShapeSet::SamplePosition (ShapeSet.cu:51-69)
Spec light_sample_direct(const SceneView& S, const ctl_light& L, DRec& dRec, V2 _sample) {
    V2 sample = _sample;
    const float* cdf = S.d->light_tri_cdf + L.cdf_first;
    float pdf;
    uint32_t index = sample_reuse(cdf, L.tri_count, sample.y, pdf);
    const ctl_light_tri& sn = S.d->light_tris[L.tri_first + index];
    float a = sqrtf(1.0f - sample.x);                      // Warp::squareToUniformTriangle
    V2 bary = v2(1 - a, a * sample.y);
    V3 p0 = v3(sn.p[0][0], sn.p[0][1], sn.p[0][2]), p1 = v3(sn.p[1][0], sn.p[1][1], sn.p[1][2]),
       p2 = v3(sn.p[2][0], sn.p[2][1], sn.p[2][2]);
    dRec.p = bary.x * p0 + bary.y * p1 + (1.f - bary.x - bary.y) * p2;
    dRec.n = v3(sn.n[0], sn.n[1], sn.n[2]);
    dRec.pdf = 1.0f / L.sum_area;
    dRec.measure = EArea;
    dRec.uv = bary;
    V3 dir = dRec.p - dRec.ref;
    float distSquared = lenSqr(dir);
    dRec.dist = sqrtf(distSquared);
    dRec.d = dir / dRec.dist;
    float dp = absdot(dRec.d, dRec.n);
    dRec.pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
    dRec.measure = ESolidAngle;
    if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0 && dRec.pdf != 0) {
        Spec rad = v3(L.radiance[0], L.radiance[1], L.radiance[2]);
        return spec_div(rad, dRec.pdf) * 1.0f;
    }
    dRec.pdf = 0.0f;
    return v3s(0.0f);
}
float light_pdf_direct(const ctl_light& L, const DRec& dRec) {   // Light.cu:137-155
    if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0) {
        float pdfPos = 1.0f / L.sum_area;
        if (dRec.measure == ESolidAngle) return pdfPos * (dRec.dist * dRec.dist) / absdot(dRec.d, dRec.n);
        else if (dRec.measure == EArea) return pdfPos;
        return 0.0f;
    }
    return 0.0f;
}
float pdf_emitter(const SceneView& S, uint32_t idx) {   // KernelDynamicScene.cu:41-45
    return S.d->light_cdf[idx] - (idx == 0 ? 0.0f : S.d->light_cdf[idx - 1]);
}
// ---- InfiniteLight (SceneTypes/Light.h:294-367, Light.cu:350-511,
// Light.cpp:10-58).  The radiance map is S.d->textures[env->texture]; the
// tables are the desc's env_data; env->world is m_worldTransform's rotation.
const float O_EPSILON = 0.000001f;               // MathFunc.h:21
const float O_INV_TWOPI = 1.0f / (2.0f * O_PI);  // MathFunc.h:14
inline float luminance(Spec s) { return s.x * 0.212671f + s.y * 0.715160f + s.z * 0.072169f; }   // Spectrum.cu:174-177
// KernelMIPMap::Sample(float width = 0, int x, int y) (MIPMap.cu:155-172): log2(1e-8) < 0 -> level 0, clamped x/y
Spec env_texel(const ctl_scene_desc* d, int x, int y) {
    const ctl_texture& t = d->textures[d->env->texture];
    x = omin(omax(x, 0), (int)t.width - 1);
    y = omin(omax(y, 0), (int)t.height - 1);
    uint32_t c = d->tex_data[t.offsets[0] + (uint32_t)y * t.width + (uint32_t)x];
    return v3(float(c & 0xff) / 255.0f, float((c >> 8) & 0xff) / 255.0f, float((c >> 16) & 0xff) / 255.0f);
}
float interval_to_tent(float sample) {   // Warp::intervalToTent (Math/Warp.h:13-27)
    float sign = 1;
    if (sample < 0.5f) sample *= 2;
    else { sign = -1; sample = 2 * (sample - 0.5f); }
    return sign * (1 - sqrtf(sample));
}
// m_worldTransform (Light.h:307, an OrthogonalAffineMap with zero translation):
// TransformDirection = float4x4::TransformDirection (float4x4.h:404-408),
// TransformDirectionTranspose = (dot(d, col0), dot(d, col1), dot(d, col2)) (float4x4.h:424-427)
M44 env_world(const ctl_env_light& L) {
    M44 m = M44::zeros();
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m(i, j) = L.world[i][j];
    m(3, 3) = 1.0f;
    return m;
}
V3 env_to_world(const ctl_env_light& L, V3 d) { return transformDirection(env_world(L), d); }
V3 env_to_local(const ctl_env_light& L, V3 d) {
    const M44 m = env_world(L);
    return v3(dot(d, xyz(m.col(0))), dot(d, xyz(m.col(1))), dot(d, xyz(m.col(2))));
}
V2 env_latlong(V3 v) {   // atan2(v.x, -v.z) / 2pi, safe_acos(v.y) / pi
    return v2(cr_atan2(v.x, -v.z) * O_INV_TWOPI, cr_acos(omin(1.0f, omax(-1.0f, v.y))) * O_INV_PI);
}
// the two bilinear rows of (xPos, yPos) and the pdf numerator they give
void env_rows(const ctl_scene_desc* d, int xPos, int yPos, float dx1, float dy1, Spec& value1, Spec& value2, float& pdf) {
    const ctl_env_light& L = *d->env;
    const float* rowWeights = d->env_data + L.row_weights;
    float dx2 = 1.0f - dx1, dy2 = 1.0f - dy1;
    value1 = env_texel(d, xPos, yPos) * dx2 * dy2 + env_texel(d, xPos + 1, yPos) * dx1 * dy2;
    value2 = env_texel(d, xPos, yPos + 1) * dx2 * dy1 + env_texel(d, xPos + 1, yPos + 1) * dx1 * dy1;
    int h = (int)L.size[1];
    pdf = (luminance(value1) * rowWeights[omin(omax(yPos, 0), h - 1)] +
           luminance(value2) * rowWeights[omin(omax(yPos + 1, 0), h - 1)]) * L.normalization;
}
// InfiniteLight::sampleDirect + internalSampleDirection (Light.cu:350-365, 420-457)
Spec env_sample_direct(const ctl_scene_desc* d, DRec& dRec, V2 sample) {
    const ctl_env_light& L = *d->env;
    float qpdf;
    uint32_t row = sample_reuse(d->env_data + L.cdf_rows, (uint32_t)L.size[1], sample.y, qpdf);
    uint32_t col = sample_reuse(d->env_data + L.cdf_cols + row * (uint32_t)(L.size[0] + 1), (uint32_t)L.size[0],
                                sample.x, qpdf);
    V2 pos = v2((float)col + interval_to_tent(sample.x), (float)row + interval_to_tent(sample.y));
    int xPos = omin(omax((int)floorf(pos.x), 0), (int)(L.size[0] - 1));
    int yPos = omin(omax((int)floorf(pos.y), 0), (int)(L.size[1] - 1));
    Spec value1, value2;
    float pdf;
    env_rows(d, xPos, yPos, pos.x - xPos, pos.y - yPos, value1, value2, pdf);
    Spec value = (value1 + value2) * v3(L.scale[0], L.scale[1], L.scale[2]);
    float phi = L.pixel_size[0] * (pos.x + 0.5f), theta = L.pixel_size[1] * (pos.y + 0.5f);
    float sinTheta = cr_sin(theta);
    V3 dir = v3(cr_sin(phi) * sinTheta, cr_cos(theta), -cr_cos(phi) * sinTheta);
    pdf /= omax(std::fabs(sinTheta), O_EPSILON);
    dir = env_to_world(L, dir);   // d = m_worldTransform.TransformDirection(d) (Light.cu:355)
    dRec.pdf = pdf;
    dRec.p = v3(L.scene_center[0], L.scene_center[1], L.scene_center[2]) + dir * L.scene_radius;
    dRec.n = -normalize(dir);
    dRec.dist = L.scene_radius;
    dRec.d = normalize(dir);
    dRec.measure = ESolidAngle;
    return spec_div(value, pdf);
}
// InfiniteLight::pdfDirect + internalPdfDirection (Light.cu:367-377, 459-479)
float env_pdf_direct(const ctl_scene_desc* d, const DRec& dRec) {
    const ctl_env_light& L = *d->env;
    const V3 ld = env_to_local(L, dRec.d);   // internalPdfDirection(TransformDirectionTranspose(dRec.d)) (Light.cu:369)
    V2 uv = env_latlong(ld);
    float u = uv.x * L.size[0] - 0.5f, v = uv.y * L.size[1] - 0.5f;
    int xPos = (int)floorf(u), yPos = (int)floorf(v);
    Spec value1, value2;
    float pdf;
    env_rows(d, xPos, yPos, u - xPos, v - yPos, value1, value2, pdf);
    float sinTheta = sqrtf(omax(0.0f, 1 - ld.y * ld.y));
    float pdfSA = pdf / omax(std::fabs(sinTheta), O_EPSILON);
    if (dRec.measure == ESolidAngle) return pdfSA;
    if (dRec.measure == EArea) return pdfSA * absdot(dRec.d, dRec.n) / (dRec.dist * dRec.dist);
    return 0.0f;
}
// KernelDynamicScene::EvalEnvironment(r) -> InfiniteLight::evalEnvironment: Sample(uv, 0) = triangle(0, uv)
Spec env_eval(const ctl_scene_desc* d, V3 dir) {
    if (d->env_map_index == UINT_MAX) return v3s(0.0f);
    const ctl_env_light& L = *d->env;
    c5::Mip M{d->textures + L.texture, d->tex_data};
    return c5::triangle(M, 0, env_latlong(env_to_local(L, dir))) * v3(L.scale[0], L.scale[1], L.scale[2]);
}
// EvalEnvironment(r, rX, rY): the MIP map filtered over the differentials (Light.cu:496-511)
Spec env_eval_diff(const ctl_scene_desc* d, V3 rd, V3 rxd, V3 ryd) {
    if (d->env_map_index == UINT_MAX) return v3s(0.0f);
    const ctl_env_light& L = *d->env;
    const V3 v = env_to_local(L, rd);
    V2 uv = env_latlong(v);
    V3 dvdx = env_to_local(L, rxd) - v, dvdy = env_to_local(L, ryd) - v;
    float t1 = O_INV_TWOPI / (v.x * v.x + v.z * v.z), t2 = -O_INV_PI / omax(sqrtf(omax(0.0f, 1.0f - v.y * v.y)), 1e-4f);
    V2 dudx = v2(t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y), dudy = v2(t1 * (dvdy.z * v.x - dvdy.x * v.z), t2 * dvdy.y);
    c5::Mip M{d->textures + L.texture, d->tex_data};
    return c5::mip_eval(M, uv, dudx, dudy) * v3(L.scale[0], L.scale[1], L.scale[2]);
}
// Light::sampleDirect dispatch over the light kinds
Spec sample_direct(const SceneView& S, const ctl_light& L, DRec& dRec, V2 sample) {
    if (L.kind == CTL_LIGHT_INFINITE) return env_sample_direct(S.d, dRec, sample);
    return light_sample_direct(S, L, dRec, sample);
}
inline float power_heuristic(float fPdf, float gPdf) {   // MonteCarlo.h:29-33 with nf=ng=1
    float f = 1 * fPdf, g = 1 * gPdf;
    return (f * f) / (f * f + g * g);
}

// The product's any-hit shadow cull rule (device/traverse.h slab_slack).
constexpr int kShadowCull = CULL_SLAB;

struct RenderCtx {
    SceneView S;
    Sampler* rng;
    int tie;
    bool quirk;
    bool anyHitShadow;
    uint64_t rays = 0;
    Stats st;
};

// KernelDynamicScene::Occluded(Ray(ori, dir), 0, tmax) (KernelDynamicScene.cu:70-80).
// Closest-hit form (the reference): traceRay, then eps < t < tmax - eps; a miss
// with an infinite tmax is not occluded (:77-78).  Any-hit form (the product's
// shadow_any_hit = 1): is there a hit with eps < t < tmax - eps.  Its boxes are
// culled past the acceptance bound (kShadowCull = CULL_SLAB: tmax + slab_slack):
// a box whose rounded slab entry lands past tmax - eps, or past tmax, can still
// hold a hit below tmax - eps, which the closest-hit form finds (it culls at its
// current hit, or not at all before the first one).
bool occluded_query(const SceneView& S, V3 ori, V3 dir, float tmax, bool anyHit, int tie, int cull, Stats* st) {
    const float eps = S.d->ray_eps;
    Hit h;
    if (anyHit) {
        h.t = tmax - eps; h.tri = UINT_MAX; h.node = UINT_MAX; h.u = h.v = 0.0f;
        if (S.d->n_nodes == 0) return false;
        AnyCull ac;
        ac.mode = cull;
        ac.dist = tmax;
        cull_bound(S.d, ac.m);
        trace_two_level(S, ori, dir, 0.0f, eps, h, true, tie, st, scene_has_alpha(S.d), ac);
        return h.tri != UINT_MAX;
    }
    trace_ray(S, ori, dir, h, tie, st);
    bool end = h.t < tmax - eps;
    if (std::isinf(tmax) && h.tri == UINT_MAX) end = false;
    return h.t > 0 + eps && end;
}

bool occluded(RenderCtx& C, V3 ori, V3 dir, float tmax) {   // with tmin = 0, as EstimateDirect calls it
    C.rays++;
    return occluded_query(C.S, ori, dir, tmax, C.anyHitShadow, C.tie, kShadowCull, &C.st);
}

Spec estimate_direct(RenderCtx& C, BRec bRec, const ctl_material& mat, const ctl_light& light, float light_pdf) {
    // TraceAlgorithms.cu:44-73 (flags = EAll & ~EDelta, attenuated, use_mis)
    DRec dRec;
    dRec.p = bRec.dg.P; dRec.n = bRec.dg.sys.n; dRec.measure = EArea;
    dRec.ref = bRec.dg.P; dRec.refN = bRec.dg.sys.n;
    Spec value = sample_direct(C.S, light, dRec, C.rng->randomFloat2());
    Spec retVal = v3s(0.0f);
    if (!spec_zero(value)) {
        bRec.wo = toLocal(bRec.dg.sys, dRec.d);
        bRec.typeMask = EAll & ~EDelta;
        Spec bsdfVal = bsdf_f(C.S.d, mat, bRec);
        if (!spec_zero(bsdfVal) && !occluded(C, dRec.ref, dRec.d, dRec.dist)) {
            float weight = 1.0f;
            if (dRec.measure != EDiscrete) {
                const float bsdfPdf = bsdf_pdf(C.S.d, mat, bRec);
                const float directPdf = dRec.pdf * light_pdf;   // measure is ESolidAngle
                weight = power_heuristic(directPdf, bsdfPdf);
            }
            retVal = value * bsdfVal * weight;
            retVal = retVal * v3s(1.0f);   // Transmittance() without volumes
        }
    }
    return retVal;
}

Spec uniform_sample_one_light(RenderCtx& C, const BRec& bRec, const ctl_material& mat) {
    // TraceAlgorithms.cu:92-101 + sampleEmitter (KernelDynamicScene.cu:25-39)
    const ctl_scene_desc* d = C.S.d;
    if (!d->n_lights) return v3s(0.0f);
    V2 sample = C.rng->randomFloat2();
    uint32_t n = omin(d->n_lights, (uint32_t)CTL_MAX_NUM_LIGHTS);
    const float* cdf = d->light_cdf;
    const float* first = cdf; uint32_t count = n;   // STL_upper_bound
    while (count > 0) {
        uint32_t c2 = count / 2; const float* mid = first + c2;
        if (!(sample.x < *mid)) { first = ++mid; count -= c2 + 1; } else count = c2;
    }
    uint32_t idx = (uint32_t)(first - cdf);
    if (idx >= n) idx = n - 1;
    float fU = cdf[idx], fL = idx > 0 ? cdf[idx - 1] : 0.0f;
    sample.x = (sample.x - fL) / (fU - fL);
    float pdf = fU - fL;
    return spec_div(estimate_direct(C, bRec, mat, d->lights[idx], pdf), pdf);
}

// PathTrace<DIRECT> restricted to surfaces without media (PathTracer.cu:10-113);
// DIRECT = false: emission unweighted (:66-67), no UniformSampleOneLight (:82-83)
Spec path_trace(RenderCtx& C, V3 rori, V3 rdir, V3 rXo, V3 rXd, V3 rYo, V3 rYd, int maxPathLength, int rrStartDepth,
                bool direct = true) {
    const ctl_scene_desc* d = C.S.d;
    Spec cl = v3s(0.0f), cf = v3s(1.0f);
    int depth = 0;
    bool specularBounce = false;
    BRec bRec;
    bRec.wo = v3(0, 0, 1);   // reference leaves it uninitialised before the first sample
    float brdf_scattering_pdf = 0;
    V3 last_nor = v3(0, 0, 0);
    Hit r2;
    while (depth++ < maxPathLength) {
        C.rays++;
        trace_ray(C.S, rori, rdir, r2, C.tie, &C.st);
        if (r2.tri != UINT_MAX) {
            // TraceResult::getBsdfSample (TraceResult.cu:16-45)
            bRec.sampledType = 0;
            bRec.typeMask = EAll;
            bRec.dg.P = rori + r2.t * rdir;
            fill_dg(C.S, v2(r2.u, r2.v), r2.tri, r2.node, bRec.dg, C.quirk);
            bRec.wi = toLocal(bRec.dg.sys, -rdir);
            const ctl_material& mat = d->materials[mat_index(C.S, r2.tri, r2.node)];
            if (mat.two_sided && bRec.wi.z < 0) {
                bRec.dg.n = -bRec.dg.n;
                bRec.dg.sys.n = -bRec.dg.sys.n;
                bRec.wi.z *= -1.0f;
            }
            if (depth == 1) c5::compute_partials(bRec.dg, rXo, rXd, rYo, rYd);   // PathTracer.cu:60-61
            uint32_t li = light_index(C.S, r2.tri, r2.node);
            if (li != UINT_MAX) {
                float misWeight = 1.0f;
                const ctl_light& L = d->lights[li];
                if (!(!direct || depth == 1 || specularBounce)) {
                    DRec dRec;   // DirectSamplingRecFromRay (TraceAlgorithms.cu:33-42)
                    dRec.ref = rori; dRec.refN = last_nor; dRec.p = bRec.dg.P; dRec.n = bRec.dg.n;
                    dRec.d = rdir; dRec.dist = r2.t; dRec.measure = ESolidAngle;
                    float direct_pdf = light_pdf_direct(L, dRec) * pdf_emitter(C.S, li);
                    misWeight = power_heuristic(brdf_scattering_pdf, direct_pdf);
                }
                // DiffuseLight::eval (Light.cu:67-82)
                V3 w = -rdir;
                Spec Le = (dot(bRec.dg.sys.n, w) <= 0) ? v3s(0.0f) : v3(L.radiance[0], L.radiance[1], L.radiance[2]);
                cl = cl + (cf * misWeight) * Le;
            }
            Spec f = bsdf_sample(d, mat, bRec, brdf_scattering_pdf, C.rng->randomFloat2());
            last_nor = bRec.dg.sys.n;
            if (direct && (mat.combined_type & ESmooth) != 0) cl = cl + cf * uniform_sample_one_light(C, bRec, mat);
            specularBounce = (bRec.sampledType & EDelta) != 0;
            cf = cf * f;
            rori = bRec.dg.P;
            rdir = toWorld(bRec.dg.sys, bRec.wo);
        }
        if (r2.tri == UINT_MAX) break;
        if (depth > rrStartDepth && !specularBounce) {
            if (C.rng->randomFloat() >= spec_max(cf)) break;
            cf = spec_div(cf, spec_max(cf));
        }
    }
    if (r2.tri == UINT_MAX) {   // PathTracer.cu:98-111
        float misWeight = 1.0f;
        if (!(!direct || depth == 1 || specularBounce) && d->env_map_index != UINT_MAX) {
            DRec dRec;   // DirectSamplingRecFromRay(r, dist, last_nor, 0, 0): solid angle along r
            dRec.ref = rori; dRec.refN = last_nor; dRec.d = rdir; dRec.dist = r2.t; dRec.measure = ESolidAngle;
            float direct_pdf = env_pdf_direct(d, dRec) * pdf_emitter(C.S, d->env_map_index);
            misWeight = power_heuristic(brdf_scattering_pdf, direct_pdf);
        }
        cl = cl + (cf * misWeight) * env_eval(d, rdir);
    }
    return cl;
}

// PerspectiveSensor::sampleRayDifferential's rayX / rayY (Sensor.cu:138-141)
void sensor_ray_diff(const ctl_camera& cam, V2 pixelSample, V3& ori, V3& dX, V3& dY) {
    M44 s2c, tw;
    std::memcpy(s2c.d, cam.sample_to_camera.m, 64);
    std::memcpy(tw.d, cam.to_world.m, 64);
    V3 nearP = transformPoint(s2c, v3(pixelSample.x * cam.inv_resolution[0], pixelSample.y * cam.inv_resolution[1], 0.0f));
    ori = transformPoint(tw, v3s(0.0f));
    dX = transformDirection(tw, normalize(nearP + v3(cam.dx[0], cam.dx[1], cam.dx[2])));
    dY = transformDirection(tw, normalize(nearP + v3(cam.dy[0], cam.dy[1], cam.dy[2])));
}

void sensor_ray(const ctl_camera& cam, V2 pixelSample, V3& ori, V3& dir) {
    // PerspectiveSensor::sampleRayDifferential (Sensor.cu:130-144)
    M44 s2c, tw;
    std::memcpy(s2c.d, cam.sample_to_camera.m, 64);
    std::memcpy(tw.d, cam.to_world.m, 64);
    V3 nearP = transformPoint(s2c, v3(pixelSample.x * cam.inv_resolution[0], pixelSample.y * cam.inv_resolution[1], 0.0f));
    V3 dd = normalize(nearP);
    ori = transformPoint(tw, v3s(0.0f));
    dir = transformDirection(tw, dd);
}

void add_sample(ctl_pixel* fb, uint32_t w, uint32_t h, float sx, float sy, Spec L) {   // Image.cu:22-44
    L.x = omax(0.0f, L.x); L.y = omax(0.0f, L.y); L.z = omax(0.0f, L.z);
    int x = floor2int(sx), y = floor2int(sy);
    auto bad = [](float f) { return std::isnan(f); };
    auto invalid = [](float f) { return !std::isfinite(f) || f < 0.0f; };
    if (x < 0 || x >= (int)w || y < 0 || y >= (int)h || bad(L.x) || bad(L.y) || bad(L.z) || invalid(L.x) ||
        invalid(L.y) || invalid(L.z))
        return;
    ctl_pixel& p = fb[(size_t)y * w + x];
    p.rgb[0] += L.x; p.rgb[1] += L.y; p.rgb[2] += L.z;
    p.weight_sum += 1.0f;
}

// ---------------------------------------------------------------------------
// WavefrontPathTracer::DoRender over DoubleRayBuffer
// (Integrators/PseudoRealtime/WavefrontPathTracer.cu:17-189, Kernel/DoubleRayBuffer.h:13-231),
// run with the queue atomics resolved in fetch order: element j of a bounce
// inserts its shadow ray and then its continuation before element j+1 does.
// ---------------------------------------------------------------------------
struct WptPayload {   // WavefrontPTRayData (WavefrontPathTracer.h:11-22)
    Spec throughput, L, directF;
    float hx = 0, hy = 0;   // half((float)x).ToFloat()
    float dDist = 0;
    uint32_t dIdx = UINT_MAX;
    bool specular_bounce = true;
    float bsdf_pdf = 0;
    uint32_t prev_normal = 0;
};

float half_round_int(uint32_t x) {   // __float2half_rn of a pixel coordinate (half.h:21-24)
    if (x < 2048u) return (float)x;
    uint32_t sh = 0;
    while ((x >> sh) >= 2048u) sh++;
    uint32_t q = x >> sh, r = x & ((1u << sh) - 1u), h = 1u << (sh - 1u);
    if (r > h || (r == h && (q & 1u))) q++;
    return (float)(q << sh);
}

// One DoubleRayBuffer::FinishIteration traversal: closest hit with the ray's
// tmin for spans and triangles (intersectKernel), as traversalResult.
void wpt_batch(const SceneView& S, const std::vector<ctl_ray>& rays, std::vector<ctl_hit>& hits, int tie, int threads) {
    hits.assign(rays.size(), ctl_hit{});
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        for (;;) {
            size_t base = next.fetch_add(256);
            if (base >= rays.size()) break;
            size_t end = std::min(rays.size(), base + 256);
            for (size_t i = base; i < end; i++) {
                const ctl_ray& r = rays[i];
                Hit h;
                h.t = r.tmax; h.tri = UINT_MAX; h.node = UINT_MAX; h.u = h.v = 0;
                trace_two_level(S, v3(r.o[0], r.o[1], r.o[2]), v3(r.d[0], r.d[1], r.d[2]), r.tmin, r.tmin, h, false,
                                tie, nullptr);
                ctl_hit& o = hits[i];
                o.dist = h.t;
                if (h.tri == UINT_MAX) { o.node_idx = -1; o.tri_idx = -1; o.bary = 0; }
                else {
                    o.node_idx = (int32_t)h.node; o.tri_idx = (int32_t)h.tri;
                    uint16_t xd = (uint16_t)(h.u * 65535), yd = (uint16_t)(h.v * 65535);   // fromResult
                    o.bary = (int32_t)(((uint32_t)yd << 16) | (uint32_t)xd);
                }
            }
        }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; i++) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
}

ctl_ray wpt_ray(V3 o, V3 d, float eps) {   // DoubleRayBuffer::convert (DoubleRayBuffer.h:224-230)
    ctl_ray r;
    r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z; r.tmin = eps;
    r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z; r.tmax = FLT_MAX;
    return r;
}

uint64_t wpt_render(const ctl_scene_desc* d, bool nee, int maxPathLength, int rrStartDepth, uint32_t passesDone,
                    uint64_t pass_index, ctl_pixel* fb, int tie, int threads) {
    const uint32_t nseq = 4096, len = 30;
    std::vector<float> s1((size_t)nseq * len), s2((size_t)nseq * len * 2);
    sampler_tables(pass_index, nseq, len, s1.data(), s2.data());
    const ctl_camera& cam = d->camera;
    const uint32_t W = cam.width, H = cam.height;
    const bool quirk = (d->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0;
    const float eps = d->ray_eps;
    SceneView S{d};
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    // pathCreateKernelWPT (WavefrontPathTracer.cu:17-49): one sample per pixel
    std::vector<WptPayload> pay(W * (size_t)H);
    std::vector<ctl_ray> rays(pay.size());
    for (uint32_t i = 0; i < W * H; i++) {
        uint32_t x = i % W, y = i / W;
        Sampler rng{s1.data(), s2.data(), nseq, len, i};
        V2 pX = v2((float)x, (float)y) + rng.randomFloat2();   // arguments of sampleSensorRay, left to right
        (void)rng.randomFloat2();
        V3 o, dd;
        sensor_ray(cam, pX, o, dd);
        WptPayload& p = pay[i];
        p.hx = half_round_int(x); p.hy = half_round_int(y);
        p.throughput = v3s(1.0f);
        p.L = v3s(0.0f);
        p.directF = v3s(0.0f);
        rays[i] = wpt_ray(o, dd, eps);
    }
    std::vector<ctl_ray> sec;            // secondary buffer 2 (inserted this bounce)
    std::vector<ctl_hit> hits, secHits;  // secHits: buffer 1 after the swap
    uint64_t traced = 0;
    for (int pass = 0;; pass++) {
        // FinishIteration
        wpt_batch(S, rays, hits, tie, threads);
        wpt_batch(S, sec, secHits, tie, threads);
        traced += rays.size() + sec.size();
        std::vector<WptPayload> npay;
        std::vector<ctl_ray> nrays, nsec;
        // pathIterateKernel<NEXT_EVENT_EST> (WavefrontPathTracer.cu:51-150)
        for (size_t j = 0; j < pay.size(); j++) {
            WptPayload p = pay[j];
            const ctl_ray& r = rays[j];
            const ctl_hit& h = hits[j];
            V3 rori = v3(r.o[0], r.o[1], r.o[2]), rdir = v3(r.d[0], r.d[1], r.d[2]);
            Sampler rng{s1.data(), s2.data(), nseq, len, (uint32_t)j};
            rng.d1 += passesDone + 2; rng.d2 += passesDone + 2;   // rng.skip(iterationIdx + 2)
            if (nee && pass > 0 && p.dIdx != UINT_MAX) {
                if (secHits[p.dIdx].dist >= p.dDist * (1 - eps)) p.L = p.L + p.directF;
                p.dIdx = UINT_MAX;
                p.directF = v3s(0.0f);
            }
            bool terminated = pass + 1 == maxPathLength;
            if ((uint32_t)h.tri_idx != UINT_MAX) {
                uint32_t bc = (uint32_t)h.bary;
                V2 bary = v2((float)(bc & 0xffffu) / 65535.0f, (float)(bc >> 16) / 65535.0f);   // toResult
                BRec bRec;   // a fresh record each element; wo given (0,0,1) before the first sample
                bRec.wo = v3(0, 0, 1);
                bRec.sampledType = 0;
                bRec.typeMask = EAll;
                bRec.dg.P = rori + h.dist * rdir;
                uint32_t tri = (uint32_t)h.tri_idx, node = (uint32_t)h.node_idx;
                fill_dg(S, bary, tri, node, bRec.dg, quirk);
                bRec.wi = toLocal(bRec.dg.sys, -rdir);
                const ctl_material& mat = d->materials[mat_index(S, tri, node)];
                if (mat.two_sided && bRec.wi.z < 0) {
                    bRec.dg.n = -bRec.dg.n;
                    bRec.dg.sys.n = -bRec.dg.sys.n;
                    bRec.wi.z *= -1.0f;
                }
                uint32_t li = light_index(S, tri, node);
                if (li != UINT_MAX) {
                    float misWeight = 1.0f;
                    const ctl_light& L = d->lights[li];
                    if (nee && !(pass == 0 || p.specular_bounce)) {
                        DRec dRec;   // DirectSamplingRecFromRay with Uchar2ToNormalizedFloat3(prev_normal)
                        dRec.ref = rori; dRec.refN = normal_decode((uint16_t)p.prev_normal); dRec.p = bRec.dg.P;
                        dRec.n = bRec.dg.n; dRec.d = rdir; dRec.dist = h.dist; dRec.measure = ESolidAngle;
                        float direct_pdf = light_pdf_direct(L, dRec) * pdf_emitter(S, li);
                        misWeight = power_heuristic(p.bsdf_pdf, direct_pdf);
                    }
                    V3 w = -rdir;
                    Spec Le = (dot(bRec.dg.sys.n, w) <= 0) ? v3s(0.0f) : v3(L.radiance[0], L.radiance[1], L.radiance[2]);
                    p.L = p.L + (misWeight * Le) * p.throughput;
                }
                bool surviveRR = true;
                if (pass >= rrStartDepth) {
                    if (rng.randomFloat() < spec_max(p.throughput)) p.throughput = spec_div(p.throughput, spec_max(p.throughput));
                    else surviveRR = false;
                }
                if (pass + 1 != maxPathLength && surviveRR) {
                    Spec f = bsdf_sample(d, mat, bRec, p.bsdf_pdf, rng.randomFloat2());
                    p.specular_bounce = (bRec.sampledType & EDelta) != 0;
                    V3 outDir = toWorld(bRec.dg.sys, bRec.wo);
                    p.dIdx = UINT_MAX;
                    if (nee && (mat.combined_type & ESmooth) != 0) {
                        DRec dRec;   // DirectSamplingRecord(P, sys.n)
                        dRec.p = bRec.dg.P; dRec.n = bRec.dg.sys.n; dRec.measure = EArea;
                        dRec.ref = bRec.dg.P; dRec.refN = bRec.dg.sys.n;
                        // sampleEmitterDirect (KernelDynamicScene.cu:98-117) + sampleEmitter (:25-39)
                        V2 sample = rng.randomFloat2();
                        Spec value = v3s(0.0f);
                        if (d->n_lights) {
                            uint32_t n = omin(d->n_lights, (uint32_t)CTL_MAX_NUM_LIGHTS);
                            const float* cdf = d->light_cdf;
                            const float* first = cdf; uint32_t count = n;   // STL_upper_bound
                            while (count > 0) {
                                uint32_t c2 = count / 2; const float* mid = first + c2;
                                if (!(sample.x < *mid)) { first = ++mid; count -= c2 + 1; } else count = c2;
                            }
                            uint32_t idx = (uint32_t)(first - cdf);
                            if (idx >= n) idx = n - 1;
                            float fU = cdf[idx], fL = idx > 0 ? cdf[idx - 1] : 0.0f;
                            sample.x = (sample.x - fL) / (fU - fL);
                            float emPdf = fU - fL;
                            value = sample_direct(S, d->lights[idx], dRec, sample);
                            if (dRec.pdf != 0) {
                                dRec.pdf *= emPdf;
                                value = spec_div(value, emPdf);
                            } else {
                                value = v3s(0.0f);
                            }
                        }
                        if (!spec_zero(value)) {
                            bRec.typeMask = EAll & ~EDelta;
                            bRec.wo = toLocal(bRec.dg.sys, dRec.d);
                            Spec bsdfVal = bsdf_f(d, mat, bRec);
                            const float bsdfPdf = bsdf_pdf(d, mat, bRec);
                            const float directPdf = dRec.pdf;   // ESolidAngle after sampleDirect
                            const float weight = power_heuristic(directPdf, bsdfPdf);
                            p.directF = p.throughput * value * bsdfVal * weight;
                            p.dDist = dRec.dist;
                            p.dIdx = (uint32_t)nsec.size();   // insertSecondaryRay
                            nsec.push_back(wpt_ray(bRec.dg.P, dRec.d, eps));
                        }
                    }
                    p.prev_normal = normal_encode(bRec.dg.sys.n);
                    p.throughput = p.throughput * f;
                    npay.push_back(p);   // insertPayloadElement
                    nrays.push_back(wpt_ray(bRec.dg.P, outDir, eps));
                } else {
                    terminated = true;
                }
            } else {
                terminated = true;
                float misWeight = 1.0f;   // WavefrontPathTracer.cu:144-157
                if (nee && !(pass == 0 || p.specular_bounce) && d->env_map_index != UINT_MAX) {
                    DRec dRec;
                    dRec.ref = rori; dRec.refN = normal_decode((uint16_t)p.prev_normal); dRec.d = rdir;
                    dRec.dist = h.dist; dRec.measure = ESolidAngle;
                    misWeight = power_heuristic(p.bsdf_pdf, env_pdf_direct(d, dRec) * pdf_emitter(S, d->env_map_index));
                }
                p.L = p.L + (misWeight * p.throughput) * env_eval(d, rdir);
            }
            if (terminated) add_sample(fb, W, H, p.hx, p.hy, p.L);
        }
        pay.swap(npay);
        rays.swap(nrays);
        sec.swap(nsec);
        if (pay.empty() || pass + 1 >= maxPathLength) break;
    }
    return traced;
}

// ---------------------------------------------------------------------------
// AnimatedMesh::k_ComputeState (Engine/AnimatedMesh.cpp:163-184) on copies of
// the compiled arrays, with the compiled tree refit (boxes only).
// ---------------------------------------------------------------------------
M44 skin_matrix(const float* bones, uint64_t idx, uint64_t wgt) {   // d_Compute (AnimatedMesh.cu:13-27)
    M44 mat;
    for (int k = 0; k < 16; k++) mat.d[k] = 0.0f;
    for (int i = 0; i < 8; i++) {
        uint32_t j = (uint32_t)(idx & 0xff);
        float w = (float)(uint32_t)(wgt & 0xff) / 255.0f;
        idx >>= 8; wgt >>= 8;
        for (int k = 0; k < 16; k++) mat.d[k] = mat.d[k] + bones[16 * j + k] * w;   // mat + m * w
    }
    return mat;
}

// TriangleData::setData (TriangleData.cu:35-63) as run on the device by
// g_ComputeTriangles: the UV halves are read back with the IEEE decode.
void tri_set_data_device(uint32_t w[8], V3 v0, V3 v1, V3 vv2, V3 n0, V3 n1, V3 n2) {
    V2 t0 = v2(half_to_float_ieee(w[5] & 0xffff), half_to_float_ieee(w[5] >> 16));
    V2 t1 = v2(half_to_float_ieee(w[6] & 0xffff), half_to_float_ieee(w[6] >> 16));
    V2 t2 = v2(half_to_float_ieee(w[7] & 0xffff), half_to_float_ieee(w[7] >> 16));
    V3 dP1 = v1 - v0, dP2 = vv2 - v0;
    V2 dUV1 = t1 - t0, dUV2 = t2 - t0;
    float determinant = dUV1.x * dUV2.y - dUV1.y * dUV2.x;
    V3 dpdu, dpdv;
    if (determinant == 0) {
        V3 a, b, n = normalize(cross(dP1, dP2));
        coordinateSystem(n, a, b);
        dpdu = a; dpdv = b;
    } else {
        float invDet = 1.0f / determinant;
        dpdu = ((dUV2.y * dP1 - dUV1.y * dP2) * invDet);
        dpdv = ((-dUV2.x * dP1 + dUV1.x * dP2) * invDet);
    }
    w[0] = (uint32_t)normal_encode(n0) | ((uint32_t)normal_encode(n1) << 16);
    w[1] = (uint32_t)normal_encode(n2) | (w[1] & 0xffff0000u);
    w[2] = float_to_half(dpdu.x) | ((uint32_t)float_to_half(dpdu.y) << 16);
    w[3] = float_to_half(dpdu.z) | ((uint32_t)float_to_half(dpdv.x) << 16);
    w[4] = float_to_half(dpdv.y) | ((uint32_t)float_to_half(dpdv.z) << 16);
}

struct Box6 { float lo[3], hi[3]; };
Box6 box_empty() { Box6 b; for (int k = 0; k < 3; k++) { b.lo[k] = FLT_MAX; b.hi[k] = -FLT_MAX; } return b; }
void box_add(Box6& b, const Box6& o) {
    for (int k = 0; k < 3; k++) { b.lo[k] = omin(b.lo[k], o.lo[k]); b.hi[k] = omax(b.hi[k], o.hi[k]); }
}
void box_add(Box6& b, V3 p) {
    Box6 q; q.lo[0] = q.hi[0] = p.x; q.lo[1] = q.hi[1] = p.y; q.lo[2] = q.hi[2] = p.z;
    box_add(b, q);
}
// BVHNodeData child boxes (TriIntersectorData.h:44-50)
Box6 node_child(const ctl_bvh_node& n, int c) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    Box6 b;
    b.lo[0] = n.v[o]; b.hi[0] = n.v[o + 1]; b.lo[1] = n.v[o + 2]; b.hi[1] = n.v[o + 3]; b.lo[2] = n.v[z]; b.hi[2] = n.v[z + 1];
    return b;
}
void node_set_child(ctl_bvh_node& n, int c, const Box6& b) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    n.v[o] = b.lo[0]; n.v[o + 1] = b.hi[0]; n.v[o + 2] = b.lo[1]; n.v[o + 3] = b.hi[1]; n.v[z] = b.lo[2]; n.v[z + 1] = b.hi[2];
}
int32_t node_kid(const ctl_bvh_node& n, int c) { int32_t v; std::memcpy(&v, &n.v[12 + c], 4); return v; }

// refits node k's child boxes from its subtree; returns the union of its children
template <class LEAF>
Box6 refit(ctl_bvh_node* nodes, uint32_t k, const LEAF& leaf) {
    Box6 all = box_empty();
    for (int c = 0; c < 2; c++) {
        int32_t v = node_kid(nodes[k], c);
        if (v == 0x76543210) continue;
        Box6 b = v < 0 ? leaf(v) : refit(nodes, (uint32_t)v >> 2, leaf);
        node_set_child(nodes[k], c, b);
        box_add(all, b);
    }
    return all;
}

// ---------------------------------------------------------------------------
// BVHRebuilder::recomputeNode with its tree rotations
// (Engine/SpatialStructures/BVH/BVHRebuilder.cpp:281-340; the rotations of the
// paper cited at :12-13), as AnimatedMesh::k_ComputeState runs it on a mesh
// tree every frame (AnimatedMesh.cpp:174-176: Build(&p, true), recomputeAll)
// and SceneBVH::Build on the instance tree for the nodes DynamicScene
// invalidated (DynamicScene.cpp:447,564; SceneBVH.cpp:43; only the flagged
// path, :431-438).  The tree state persists: each call starts from the tree
// the last one left.
//   getBox (:598-609): NO_NODE = AABB::Identity; a leaf = its objects' boxes
//     extended from the identity; an inner node = BVHNodeData::getBox, the
//     union of BOTH stored child slots (an empty slot's stored box included)
//   numLeafs (:645-657): objects under the node (bvhNodeData, BuildInfoTree)
//   sah (:624-638), numberGrandchildren (:612-622), swapChildren (:691-702),
//     setChild (:665-681): child value, slot box, parent (BVHNodeData d.z,
//     native) of a moved inner node; propagateBBChange's writes to the
//     ancestors are overwritten when the recursion returns to them
//   AABB::Area (Math/AABB.h:19-23): 2 (x y + x z + y z) of max - min
// ---------------------------------------------------------------------------
constexpr int32_t kNoNode = 0x76543210;

float box_area(const Box6& b) {
    const float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
    return 2.0f * (x * y + x * z + y * z);
}
Box6 box_union(Box6 a, const Box6& b) { box_add(a, b); return a; }
void node_set_kid(ctl_bvh_node& n, int c, int32_t v) { std::memcpy(&n.v[12 + c], &v, 4); }
void node_set_parent(ctl_bvh_node& n, int32_t p) { std::memcpy(&n.v[14], &p, 4); }

struct Rebuilder {
    ctl_bvh_node* N;
    std::function<Box6(int32_t)> leaf_box;     // union of the leaf's objects' boxes (from the identity)
    std::function<int(int32_t)> leaf_count;    // objects in the leaf
    std::function<void(int32_t)> leaf_set;     // setObject for the leaf's entries (may be empty)
    const std::vector<uint8_t>* flagged = nullptr;   // inner nodes to recompute; null: recomputeAll
    std::vector<int32_t> nleaf;

    static bool inner(int32_t v) { return v >= 0 && v != kNoNode; }
    int count(int32_t v) {   // BuildInfoTree (:476-495)
        int s = 0;
        for (int c = 0; c < 2; c++) {
            const int32_t k = node_kid(N[v >> 2], c);
            if (k < 0) s += leaf_count(k);
            else if (k != kNoNode) s += count(k);
        }
        return nleaf[v >> 2] = s;
    }
    int num_leafs(int32_t v) { return v == kNoNode ? 0 : v < 0 ? leaf_count(v) : nleaf[v >> 2]; }
    Box6 get_box(int32_t v) {
        if (v == kNoNode) return box_empty();
        if (v < 0) return leaf_box(v);
        return box_union(node_child(N[v >> 2], 0), node_child(N[v >> 2], 1));
    }
    int32_t kid(int32_t v, int c) { return node_kid(N[v >> 2], c); }
    int grandchildren(int32_t v, int c) {
        const int32_t k = kid(v, c);
        if (!inner(k)) return 0;
        return (kid(k, 0) != kNoNode) + (kid(k, 1) != kNoNode);
    }
    float sah(int32_t v, int lc, int lg) {
        const int32_t child = kid(v, lc), other = kid(v, 1 - lc);
        const int32_t grand = kid(other, lg), og = kid(other, 1 - lg);
        const float rhs_area = box_area(get_box(grand));
        const int rhs_num = num_leafs(grand);
        const Box6 lhs = box_union(get_box(child), get_box(og));
        const int n1 = num_leafs(child), n2 = num_leafs(og);
        return box_area(lhs) * (float)(n1 + n2) + rhs_area * (float)rhs_num;
    }
    void set_child(int32_t v, int c, int32_t k) {   // setChild's array writes
        node_set_kid(N[v >> 2], c, k);
        node_set_child(N[v >> 2], c, get_box(k));
        if (inner(k)) node_set_parent(N[k >> 2], v);
    }
    void swap(int32_t v, int lc, int lg) {
        const int32_t child = kid(v, lc), other = kid(v, 1 - lc);
        const int32_t grand = kid(other, lg);
        set_child(other, lg, child);
        node_set_child(N[v >> 2], 1 - lc, get_box(other));   // propagateBBChange(other -> v)
        set_child(v, lc, grand);
        nleaf[other >> 2] += num_leafs(child) - num_leafs(grand);
    }
    Box6 recompute(int32_t v) {
        const int32_t c[2] = {kid(v, 0), kid(v, 1)};
        bool modified = false;
        for (int i = 0; i < 2; i++) {
            if (c[i] < 0 || (c[i] != kNoNode && (!flagged || (*flagged)[c[i] >> 2]))) {
                modified = true;
                Box6 b;
                if (c[i] < 0) {
                    if (leaf_set) leaf_set(c[i]);
                    b = get_box(c[i]);
                } else {
                    b = recompute(c[i]);
                }
                node_set_child(N[v >> 2], i, b);
            }
        }
        if (modified) {
            const bool ab = grandchildren(v, 0) == 2, cd = grandchildren(v, 1) == 2;
            float rot[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
            if (ab) { rot[0] = sah(v, 1, 0); rot[1] = sah(v, 1, 1); }
            if (cd) { rot[2] = sah(v, 0, 1); rot[3] = sah(v, 0, 0); }
            int best = 0;
            for (int i = 1; i < 4; i++)
                if (rot[i] < rot[best]) best = i;   // std::min_element: the first smallest
            const float cur = box_area(get_box(c[0])) * (float)num_leafs(c[0]) +
                              box_area(get_box(c[1])) * (float)num_leafs(c[1]);
            if (rot[best] < cur) {
                static const int lc[4] = {1, 1, 0, 0}, lg[4] = {0, 1, 1, 0};
                swap(v, lc[best], lg[best]);
            }
        }
        return get_box(v);
    }
    Box6 run(int32_t root) {
        nleaf.assign(nleaf.size(), 0);
        count(root);
        return recompute(root);
    }
};

void instance_box(const M44& xf, const float lo[3], const float hi[3], Box6& o) {   // scene compile's node box
    o = box_empty();
    for (int c = 0; c < 8; c++) {
        V3 p = v3((c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]);
        V3 q = transformPoint(xf, p);
        box_add(o, q);
    }
    for (int k = 0; k < 3; k++) {
        float ext = omax(std::fabs(o.lo[k]), std::fabs(o.hi[k])) * 1e-6f + 1e-30f;
        o.lo[k] -= ext; o.hi[k] += ext;
    }
}

// The instance tree after nodes `moved` changed (SceneBVH::Build ->
// BVHRebuilder::Build without invalidateAll: only the flagged path, with
// rotations): instance boxes from the mesh boxes and the transforms (xf16 per
// node, or the desc's), the scene box's epsilon (DynamicScene.cpp:587).
void scene_rebuild(const ctl_scene_desc* d, ctl_bvh_node* scene, const float* mesh_boxes, const float* xf16,
                   const std::vector<uint32_t>& moved, float* eps) {
    std::vector<Box6> inst(d->n_nodes);
    Box6 sb = box_empty();
    for (uint32_t i = 0; i < d->n_nodes; i++) {
        M44 xf; std::memcpy(xf.d, xf16 ? xf16 + 16 * i : d->node_xf[i].m, 64);
        const float* m = mesh_boxes + 6 * d->nodes[i].mesh_index;
        instance_box(xf, m, m + 3, inst[i]);
        box_add(sb, inst[i]);
    }
    if (d->n_nodes && d->scene_start_node >= 0 && d->n_scene_bvh_nodes) {
        const uint32_t ns = d->n_scene_bvh_nodes;
        // propagateFlag (:343-362): each moved instance's holder and its ancestors
        std::vector<uint8_t> flag(ns, 0);
        for (uint32_t k = 0; k < ns; k++)
            for (int c = 0; c < 2; c++) {
                const int32_t v = node_kid(scene[k], c);
                if (v >= 0 || v == kNoNode || std::find(moved.begin(), moved.end(), (uint32_t)~v) == moved.end()) continue;
                for (int32_t a = (int32_t)(k * 4); a != -1 && !flag[a >> 2];) {
                    flag[a >> 2] = 1;
                    std::memcpy(&a, &scene[a >> 2].v[14], 4);
                }
            }
        Rebuilder R;
        R.N = scene;
        R.nleaf.assign(ns, 0);
        R.flagged = &flag;
        R.leaf_box = [&](int32_t v) { return box_union(box_empty(), inst[(uint32_t)~v]); };
        R.leaf_count = [](int32_t) { return 1; };
        const int32_t root = d->scene_start_node;
        R.nleaf.assign(ns, 0);
        R.count(root);
        if (flag[root >> 2]) R.recompute(root);
    }
    V3 size = v3(sb.hi[0] - sb.lo[0], sb.hi[1] - sb.lo[1], sb.hi[2] - sb.lo[2]);
    *eps = 1e-4f * length(size);
}

void animate(const ctl_scene_desc* d, uint32_t anim, const float* b0, const float* b1, float t, ctl_triangle_data* tri,
             float* woop, ctl_bvh_node* nodes, ctl_bvh_node* scene, float* mesh_boxes, float* eps) {
    const ctl_anim_mesh& am = d->anim_meshes[anim];
    const ctl_kernel_mesh& km = d->meshes[am.mesh];
    const bool last = am.mesh + 1 == d->n_meshes;
    const uint64_t e1 = last ? d->n_tri_indices : d->meshes[am.mesh + 1].bvh_indices_offset;
    // g_ComputeVertices (AnimatedMesh.cu:29-43)
    std::vector<V3> P(am.vertex_count), N(am.vertex_count);
    for (uint32_t i = 0; i < am.vertex_count; i++) {
        const ctl_anim_vertex& v = d->anim_vertices[am.vertex_first + i];
        M44 m0 = skin_matrix(b0, v.bone_indices, v.bone_weights), m1 = skin_matrix(b1, v.bone_indices, v.bone_weights);
        V3 p = v3(v.pos[0], v.pos[1], v.pos[2]), n = v3(v.normal[0], v.normal[1], v.normal[2]);
        V3 p0 = transformPoint(m0, p), p1 = transformPoint(m1, p);
        P[i] = p0 * (1.0f - t) + p1 * t;   // math::lerp (MathFunc.h:161)
        V3 n0 = transformDirection(m0, n), n1 = transformDirection(m1, n);
        N[i] = normalize(n0 * (1.0f - t) + n1 * t);
    }
    const uint32_t* T = d->anim_triangles + 3ull * am.tri_first;
    // g_ComputeTriangles
    for (uint32_t i = 0; i < am.tri_count; i++) {
        uint32_t* w = tri[km.triangle_offset + i].w;
        tri_set_data_device(w, P[T[3 * i]], P[T[3 * i + 1]], P[T[3 * i + 2]], N[T[3 * i]], N[T[3 * i + 1]], N[T[3 * i + 2]]);
    }
    // AnimProvider::setObject for every entry
    for (uint64_t e = km.bvh_indices_offset; e < e1; e++) {
        uint32_t i = d->tri_indices[e] >> 1;
        woop_set(P[T[3 * i]], P[T[3 * i + 1]], P[T[3 * i + 2]], woop + 12 * e);
    }
    // BVHRebuilder over the mesh tree (recomputeAll, with rotations); leaves =
    // the triangles of their entry run, each triangle's box from its vertices
    // (AnimProvider::getBox, AnimatedMesh.cpp:106-114)
    const uint32_t* idx = d->tri_indices + km.bvh_indices_offset;
    const uint32_t n0 = km.bvh_node_offset / 4;
    const uint64_t n1 = last ? d->n_bvh_nodes : d->meshes[am.mesh + 1].bvh_node_offset / 4;
    Rebuilder R;
    R.N = nodes + n0;
    R.nleaf.assign(n1 - n0, 0);
    R.leaf_box = [&](int32_t v) {
        Box6 b = box_empty();
        for (uint32_t e = (uint32_t)~v;; e++) {
            uint32_t i = idx[e] >> 1;
            for (int k = 0; k < 3; k++) box_add(b, P[T[3 * i + k]]);
            if (idx[e] & 1) break;
        }
        return b;
    };
    R.leaf_count = [&](int32_t v) {
        int n = 1;
        for (uint32_t e = (uint32_t)~v; !(idx[e] & 1); e++) n++;
        return n;
    };
    Box6 mb = R.run(0);
    for (int k = 0; k < 3; k++) { mesh_boxes[6 * am.mesh + k] = mb.lo[k]; mesh_boxes[6 * am.mesh + 3 + k] = mb.hi[k]; }
    // instances, scene tree (the animated mesh's instances invalidated), epsilon (DynamicScene.cpp:587)
    std::vector<uint32_t> moved;
    for (uint32_t i = 0; i < d->n_nodes; i++)
        if (d->nodes[i].mesh_index == am.mesh) moved.push_back(i);
    scene_rebuild(d, scene, mesh_boxes, nullptr, moved, eps);
}

}  // namespace

// ===========================================================================
// C API for tests (ctypes)
// ===========================================================================
extern "C" {

// Registers the 4-wide trees of scene d for TRAVERSE_WIDE (128-B WideNode
// records, host/bvh_wide.h layout; wbase[mesh] = first node of the mesh's tree;
// the instance tree rooted at node 0).  Replaces the previous registration.
void oracle_set_wide(const ctl_scene_desc* d, const void* mesh_nodes, uint64_t n_mesh_nodes, const uint32_t* wbase,
                     uint32_t n_wbase, const void* scene_nodes, uint64_t n_scene_nodes) {
    std::lock_guard<std::mutex> g(g_wide_mtx);
    g_wide.key_nodes = d->bvh_nodes;
    g_wide.key_scene = d->scene_bvh_nodes;
    g_wide.key_n = d->n_bvh_nodes;
    const float* m = static_cast<const float*>(mesh_nodes);
    const float* sc = static_cast<const float*>(scene_nodes);
    g_wide.mesh.assign(m, m + 32 * n_mesh_nodes);
    g_wide.wbase.assign(wbase, wbase + n_wbase);
    g_wide.scene.assign(sc, sc + 32 * n_scene_nodes);
    g_wide.set = true;
}

void oracle_woop_set(const float* v0, const float* v1, const float* v2, float* out12) {
    woop_set(v3(v0[0], v0[1], v0[2]), v3(v1[0], v1[1], v1[2]), v3(v2[0], v2[1], v2[2]), out12);
}
void oracle_woop_get(const float* in12, float* v0, float* v1, float* v2) {
    V3 a, b, c;
    woop_get(in12, a, b, c);
    v0[0] = a.x; v0[1] = a.y; v0[2] = a.z;
    v1[0] = b.x; v1[1] = b.y; v1[2] = b.z;
    v2[0] = c.x; v2[1] = c.y; v2[2] = c.z;
}

void oracle_xorwow_uniforms(uint64_t subsequence, uint64_t offset, uint64_t n, float* out) {
    Xorwow s = curand_init(1234, subsequence, offset);
    for (uint64_t i = 0; i < n; i++) out[i] = xorwow_uniform(s);
}
void oracle_xorwow_raw(uint64_t seed, uint64_t subsequence, uint64_t offset, uint64_t n, uint32_t* out) {
    Xorwow s = curand_init(seed, subsequence, offset);
    for (uint64_t i = 0; i < n; i++) out[i] = xorwow_next(s);
}
void oracle_sampler_tables(uint64_t pass, uint32_t nseq, uint32_t len, float* seq1d, float* seq2d) {
    sampler_tables(pass, nseq, len, seq1d, seq2d);
}
// Draws of SequenceSampler(idx): n1 randomFloat() then n2 randomFloat2().
void oracle_sampler_draws(const float* seq1d, const float* seq2d, uint32_t nseq, uint32_t len, uint32_t idx,
                          uint32_t n1, float* out1, uint32_t n2, float* out2) {
    Sampler s{seq1d, seq2d, nseq, len, idx};
    for (uint32_t i = 0; i < n1; i++) out1[i] = s.randomFloat();
    for (uint32_t i = 0; i < n2; i++) { V2 v = s.randomFloat2(); out2[2 * i] = v.x; out2[2 * i + 1] = v.y; }
}

// PerspectiveSensor::Update + Sensor::SetToWorld(pos, tar, up) (Sensor.cu:76-96,674-699)
void oracle_camera(const float* pos, const float* tar, const float* up, float fov_deg, float nearc, float farc,
                   uint32_t w, uint32_t h, ctl_camera* out) {
    V3 p = v3(pos[0], pos[1], pos[2]), t = v3(tar[0], tar[1], tar[2]), u = v3(up[0], up[1], up[2]);
    V3 f = normalize(t - p);
    V3 r = normalize(cross(f, u));
    M44 view = M44::identity();
    view.setCol(0, v4(r, 0)); view.setCol(1, v4(u, 0)); view.setCol(2, v4(f, 0));
    view.setCol(3, v4(0, 0, 0, 1)); view.setRow(3, v4(0, 0, 0, 1));
    M44 tr = M44::identity(); tr(0, 3) = p.x; tr(1, 3) = p.y; tr(2, 3) = p.z;
    M44 toWorld = matmul(tr, view);
    float resx = (float)w, resy = (float)h;
    float invx = 1.0f / resx, invy = 1.0f / resy;
    float aspect = resx / resy;
    float fov = ((float)O_PI / 180.f) * fov_deg;
    M44 sc = M44::identity(); sc(0, 0) = -0.5f; sc(1, 1) = -0.5f * aspect; sc(2, 2) = 1.0f;
    M44 tl = M44::identity(); tl(0, 3) = -1.0f; tl(1, 3) = -1.0f / aspect; tl(2, 3) = 0.0f;
    float recip = 1.0f / (farc - nearc);
    float cot = 1.0f / cr_tan(fov / 2.0f);
    M44 pe = M44::zeros();
    pe(0, 0) = cot; pe(1, 1) = cot; pe(2, 2) = farc * recip; pe(2, 3) = -nearc * farc * recip; pe(3, 2) = 1;
    M44 camToSample = matmul(matmul(sc, tl), pe);
    M44 s2c = inverse(camToSample);
    V3 dx = transformPoint(s2c, v3(invx, 0.0f, 0.0f)) - transformPoint(s2c, v3s(0.0f));
    V3 dy = transformPoint(s2c, v3(0.0f, invy, 0.0f)) - transformPoint(s2c, v3s(0.0f));
    std::memcpy(out->to_world.m, toWorld.d, 64);
    std::memcpy(out->sample_to_camera.m, s2c.d, 64);
    out->dx[0] = dx.x; out->dx[1] = dx.y; out->dx[2] = dx.z;
    out->dy[0] = dy.x; out->dy[1] = dy.y; out->dy[2] = dy.z;
    out->inv_resolution[0] = invx; out->inv_resolution[1] = invy;
    out->width = w; out->height = h;
}

// traceRay semantics (mode 0) or batch semantics (mode 1 closest, 2 any-hit).
// Outputs t,u,v,tri,node per ray; stats[0..3] = rays, inner nodes, tri tests, instance entries.
void oracle_trace(const ctl_scene_desc* desc, int64_t n, const ctl_ray* rays, int32_t mode, int32_t tie,
                  float* out_t, float* out_u, float* out_v, uint32_t* out_tri, uint32_t* out_node, uint64_t* stats,
                  int32_t threads) {
    SceneView S{desc};
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    std::atomic<int64_t> next{0};
    std::mutex mtx;
    uint64_t acc[4] = {0, 0, 0, 0};
    auto worker = [&]() {
        Stats st;
        uint64_t nr = 0;
        for (;;) {
            int64_t base = next.fetch_add(256);
            if (base >= n) break;
            int64_t end = std::min<int64_t>(n, base + 256);
            for (int64_t i = base; i < end; i++) {
                const ctl_ray& r = rays[i];
                V3 o = v3(r.o[0], r.o[1], r.o[2]), dd = v3(r.d[0], r.d[1], r.d[2]);
                Hit h;
                if (mode == 0) {
                    trace_ray(S, o, dd, h, tie, &st);
                } else {
                    h.t = r.tmax; h.tri = UINT_MAX; h.node = UINT_MAX; h.u = h.v = 0;
                    trace_two_level(S, o, dd, r.tmin, r.tmin, h, mode == 2, tie, &st);
                }
                nr++;
                out_t[i] = h.t; out_u[i] = h.u; out_v[i] = h.v; out_tri[i] = h.tri; out_node[i] = h.node;
            }
        }
        std::lock_guard<std::mutex> g(mtx);
        acc[0] += nr; acc[1] += st.nodes; acc[2] += st.tris; acc[3] += st.inst;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; i++) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
    if (stats) for (int i = 0; i < 4; i++) stats[i] = acc[i];
}

// Occluded(Ray(o, d), 0, tmax) per ray (rays[i].tmax = tmax, tmin ignored): the
// reference's closest-hit form (any_hit 0) or the any-hit query (any_hit 1)
// with boxes culled at tmax - eps (cull 0, round 4's rule), at tmax (1), not
// past the ray origin (2) or at tmax + slab_slack (3, the product's).
void oracle_occluded(const ctl_scene_desc* desc, int64_t n, const ctl_ray* rays, uint8_t* out, int32_t any_hit,
                     int32_t tie, int32_t cull, int32_t threads) {
    SceneView S{desc};
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        for (;;) {
            const int64_t base = next.fetch_add(256);
            if (base >= n) break;
            const int64_t end = std::min<int64_t>(n, base + 256);
            for (int64_t i = base; i < end; i++) {
                const ctl_ray& r = rays[i];
                out[i] = occluded_query(S, v3(r.o[0], r.o[1], r.o[2]), v3(r.d[0], r.d[1], r.d[2]), r.tmax, any_hit != 0,
                                        tie, cull, nullptr) ? 1 : 0;
            }
        }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; i++) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
}

// Batch kernel output layout (ctl_hit), TraceHelper.cu:722-731.
void oracle_intersect(const ctl_scene_desc* desc, int64_t n, const ctl_ray* rays, ctl_hit* hits, int32_t any_hit,
                      int32_t tie, int32_t threads) {
    std::vector<float> t(n), u(n), v(n);
    std::vector<uint32_t> tri(n), node(n);
    oracle_trace(desc, n, rays, any_hit ? 2 : 1, tie, t.data(), u.data(), v.data(), tri.data(), node.data(), nullptr,
                 threads);
    for (int64_t i = 0; i < n; i++) {
        ctl_hit& h = hits[i];
        h.dist = t[i];
        if (tri[i] == UINT_MAX) { h.node_idx = -1; h.tri_idx = -1; h.bary = 0; }
        else {
            h.node_idx = (int32_t)node[i]; h.tri_idx = (int32_t)tri[i];
            uint16_t xd = (uint16_t)(u[i] * 65535), yd = (uint16_t)(v[i] * 65535);
            h.bary = (int32_t)(((uint32_t)yd << 16) | (uint32_t)xd);
        }
    }
}

// Closest hit by scanning every leaf entry of every node (BVH-independent truth).
void oracle_brute_force(const ctl_scene_desc* d, int64_t n, const ctl_ray* rays, float* out_t, uint32_t* out_tri,
                        int32_t threads) {
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        for (;;) {
            int64_t i = next.fetch_add(1);
            if (i >= n) break;
            const ctl_ray& r = rays[i];
            V3 o = v3(r.o[0], r.o[1], r.o[2]), dd = v3(r.d[0], r.d[1], r.d[2]);
            float best = FLT_MAX; uint32_t bt = UINT_MAX;
            for (uint32_t ni = 0; ni < d->n_nodes; ni++) {
                const ctl_kernel_mesh& mesh = d->meshes[d->nodes[ni].mesh_index];
                M44 modl; std::memcpy(modl.d, d->node_inv_xf[ni].m, 64);
                V3 dl = transformDirection(modl, dd), ol = transformPoint(modl, o);
                // entries of this mesh: [bvh_indices_offset, next mesh offset)
                uint64_t e0 = mesh.bvh_indices_offset, e1 = d->n_tri_indices;
                for (uint32_t m = 0; m < d->n_meshes; m++)
                    if (d->meshes[m].bvh_indices_offset > e0 && d->meshes[m].bvh_indices_offset < e1) e1 = d->meshes[m].bvh_indices_offset;
                for (uint64_t e = e0; e < e1; e++) {
                    const float* v = reinterpret_cast<const float*>(d->woop_tris) + 12 * e;
                    float Oz = v[3] - ol.x * v[0] - ol.y * v[1] - ol.z * v[2];
                    float invDz = 1.0f / (dl.x * v[0] + dl.y * v[1] + dl.z * v[2]);
                    float t = Oz * invDz;
                    uint32_t gtri = (d->tri_indices[e] >> 1) + mesh.triangle_offset;
                    if (t > d->ray_eps && (t < best || (t == best && gtri < bt))) {
                        float u = (v[7] + ol.x * v[4] + ol.y * v[5] + ol.z * v[6]) + t * (dl.x * v[4] + dl.y * v[5] + dl.z * v[6]);
                        if (u >= 0.0f) {
                            float vv = (v[11] + ol.x * v[8] + ol.y * v[9] + ol.z * v[10]) + t * (dl.x * v[8] + dl.y * v[9] + dl.z * v[10]);
                            if (vv >= 0.0f && u + vv <= 1.0f) { best = t; bt = gtri; }
                        }
                    }
                }
            }
            out_t[i] = best; out_tri[i] = bt;
        }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; i++) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
}

// One PathTracer pass (pathKernel2 semantics, PathTracer.cu:182-194) over the
// pixels of the tiles owned by (rank, num_ranks), accumulating into fb.
// Returns the number of traceRay calls.  pixel_stride > 1 renders only every
// pixel_stride-th pixel (bounded CPU-baseline samples); stats may be NULL.
// Paths are traced on worker threads; the samples are then added with
// AddSample one by one in image order (pixel y*W+x), the order of a
// single-threaded pass: a jittered sample can land on the neighbouring pixel
// (floor(x + u) with u close to 1), so adding from the threads would race.
// With num_ranks > 1 the rank sums exactly the samples that land on its own
// pixels, in that order: it also traces another rank's pixel whose sample
// lands on one of its pixels (the product's apron items), and drops its own
// samples that land on another rank's pixel, so the ranks' framebuffers sum to
// the 1-rank framebuffer bit for bit.
uint64_t oracle_render_pass(const ctl_scene_desc* desc, const ctl_pt_params* prm, uint64_t pass_index,
                            ctl_pixel* fb, int32_t tie, int32_t threads, uint32_t pixel_stride, uint64_t* stats) {
    const uint32_t nseq = 4096, len = 30;
    std::vector<float> s1((size_t)nseq * len), s2((size_t)nseq * len * 2);
    sampler_tables(pass_index, nseq, len, s1.data(), s2.data());
    const ctl_camera& cam = desc->camera;
    uint32_t W = cam.width, H = cam.height;
    uint32_t ts = prm->tile_size ? prm->tile_size : 64;
    uint32_t tilesX = (W + ts - 1) / ts;
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (pixel_stride == 0) pixel_stride = 1;
    std::atomic<int64_t> nextRow{0};
    std::mutex mtx;
    uint64_t totalRays = 0, acc[3] = {0, 0, 0};
    struct Smp { float x, y; Spec L; bool set; };
    std::vector<Smp> smp((size_t)W * H);
    const bool multi = prm->num_ranks > 1;
    auto owned = [&](uint32_t px, uint32_t py) {
        return !multi || ((py / ts) * tilesX + px / ts) % prm->num_ranks == prm->rank;
    };
    auto lands_owned = [&](V2 pX) {
        const float lx = std::floor(pX.x), ly = std::floor(pX.y);
        return lx >= 0.0f && ly >= 0.0f && lx < (float)W && ly < (float)H && owned((uint32_t)lx, (uint32_t)ly);
    };
    auto worker = [&]() {
        RenderCtx C{SceneView{desc}, nullptr, tie, (desc->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0,
                    prm->shadow_any_hit != 0};
        for (;;) {
            int64_t y = nextRow.fetch_add(1);
            if (y >= (int64_t)H) break;
            for (uint32_t x = 0; x < W; x++) {
                uint64_t lin = (uint64_t)y * W + x;
                if (lin % pixel_stride) continue;
                Sampler rng{s1.data(), s2.data(), nseq, len, (uint32_t)(y * W + x)};
                C.rng = &rng;
                V2 pX = v2((float)x, (float)y) + rng.randomFloat2();
                if (!owned(x, (uint32_t)y) && !lands_owned(pX)) continue;
                V2 aperture = rng.randomFloat2();
                (void)aperture;
                V3 o, dd, xo, dX, dY;
                sensor_ray(cam, pX, o, dd);
                sensor_ray_diff(cam, pX, xo, dX, dY);
                Spec col = v3s(1.0f) * path_trace(C, o, dd, xo, dX, xo, dY, prm->max_path_length, prm->rr_start_depth,
                                                   prm->direct != 0);
                smp[lin] = Smp{pX.x, pX.y, col, true};
            }
        }
        std::lock_guard<std::mutex> g(mtx);
        totalRays += C.rays;
        acc[0] += C.st.nodes; acc[1] += C.st.tris; acc[2] += C.st.inst;
    };
    std::vector<std::thread> tv;
    for (int i = 0; i < threads; i++) tv.emplace_back(worker);
    for (auto& t : tv) t.join();
    for (size_t i = 0; i < smp.size(); i++)
        if (smp[i].set && (!multi || lands_owned(v2(smp[i].x, smp[i].y)))) add_sample(fb, W, H, smp[i].x, smp[i].y, smp[i].L);
    if (stats) { stats[0] = totalRays; stats[1] = acc[0]; stats[2] = acc[1]; stats[3] = acc[2]; }
    return totalRays;
}

// PrimTracer::DoRender as Tracer<false>::DoPass runs it (Integrators/PrimTracer.cu:19-106,
// 181-233; Kernel/Tracer.h:209-224): clear the image, one primary ray per pixel
// through the pixel corner, the draw mode's first-hit value added at (x, y).
// The supported BSDFs have no delta component, so first_non_delta_X == first_X.
static float depth_d3d(float d, float n, float f) {   // DeviceDepthImage::NormalizeDepthD3D (Tracer.h:26-31)
    float z = omin(omax(d, n), f);
    return (f / (f - n) * z - f * n / (f - n)) / z;
}

uint64_t oracle_prim_pass(const ctl_scene_desc* desc, const ctl_prim_params* prm, uint64_t pass_index, ctl_pixel* fb,
                          float* depth, int32_t tie, int32_t threads) {
    const uint32_t nseq = 4096, len = 30;
    std::vector<float> s1((size_t)nseq * len), s2((size_t)nseq * len * 2);
    sampler_tables(pass_index, nseq, len, s1.data(), s2.data());
    const ctl_camera& cam = desc->camera;
    const uint32_t W = cam.width, H = cam.height;
    std::memset(fb, 0, sizeof(ctl_pixel) * (size_t)W * H);   // Image::Clear
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    const int mode = prm->draw_mode;
    const float nd = prm->near_depth, fd = prm->far_depth;
    std::atomic<int64_t> nextRow{0};
    std::atomic<uint64_t> totalRays{0};
    std::vector<Spec> out((size_t)W * H);
    auto worker = [&]() {
        // UniformSampleOneLight's Occluded: any hit over (eps, dist - eps) decides as the
        // reference's closest hit + distance test does
        RenderCtx C{SceneView{desc}, nullptr, tie, (desc->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0, true};
        for (;;) {
            const int64_t y = nextRow.fetch_add(1);
            if (y >= (int64_t)H) break;
            for (uint32_t x = 0; x < W; x++) {
                Sampler rng{s1.data(), s2.data(), nseq, len, (uint32_t)(y * W + x)};
                C.rng = &rng;
                const V2 pX = v2((float)x, (float)y);
                (void)rng.randomFloat2();   // aperture sample
                V3 o, d, xo, dX, dY;
                sensor_ray(cam, pX, o, d);
                sensor_ray_diff(cam, pX, xo, dX, dY);
                Hit h;
                C.rays++;
                trace_ray(C.S, o, d, h, C.tie, &C.st);
                Spec L = v3s(0.0f);
                if (h.tri != UINT_MAX) {
                    if (mode == CTL_PRIM_LINEAR_DEPTH) {
                        L = v3s((h.t - nd) / (fd - nd));
                    } else if (mode == CTL_PRIM_D3D_DEPTH) {
                        L = v3s(depth_d3d(h.t, nd, fd));
                    } else {
                        BRec bRec;   // TraceResult::getBsdfSample (TraceResult.cu:16-45)
                        bRec.sampledType = 0;
                        bRec.typeMask = EAll;
                        bRec.dg.P = o + h.t * d;
                        fill_dg(C.S, v2(h.u, h.v), h.tri, h.node, bRec.dg, C.quirk);
                        bRec.wi = toLocal(bRec.dg.sys, -d);
                        const ctl_material& mat = desc->materials[mat_index(C.S, h.tri, h.node)];
                        if (mat.two_sided && bRec.wi.z < 0) {
                            bRec.dg.n = -bRec.dg.n;
                            bRec.dg.sys.n = -bRec.dg.sys.n;
                            bRec.wi.z *= -1.0f;
                        }
                        c5::compute_partials(bRec.dg, xo, dX, xo, dY);
                        const V3 w = -d;
                        if (mode == CTL_PRIM_V_ABSDOT_N_GEO) L = v3s(std::fabs(dot(w, bRec.dg.n)));
                        else if (mode == CTL_PRIM_V_DOT_N_GEO) L = v3s(dot(w, bRec.dg.n));
                        else if (mode == CTL_PRIM_V_DOT_N_SHADE) L = v3s(dot(w, bRec.dg.sys.n));
                        else if (mode == CTL_PRIM_N_GEO_COLORED || mode == CTL_PRIM_N_SHADE_COLORED) {
                            const V3 n = mode == CTL_PRIM_N_GEO_COLORED ? bRec.dg.n : bRec.dg.sys.n;
                            const V3 c = n + v3s(1.0f);
                            L = v3(c.x / 2, c.y / 2, c.z / 2);
                        } else if (mode == CTL_PRIM_UV) L = v3(bRec.dg.uv.x, bRec.dg.uv.y, 0.0f);
                        else if (mode == CTL_PRIM_BARY_COORDS) L = v3(bRec.dg.bary.x, bRec.dg.bary.y, 0.0f);
                        else {
                            bRec.wo = v3(0.0f, 0.0f, 1.0f);
                            const Spec f_avg = bsdf_f(desc, mat, bRec);
                            Spec Le = v3s(0.0f);   // TraceResult::Le -> DiffuseLight::eval (Light.cu:67-82)
                            const uint32_t li = light_index(C.S, h.tri, h.node);
                            if (li != UINT_MAX) {
                                const ctl_light& Lt = desc->lights[li];
                                Le = (dot(bRec.dg.sys.n, w) <= 0) ? v3s(0.0f)
                                                                  : v3(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
                            }
                            const Spec through = v3s(1.0f);   // Transmittance without media
                            if (mode == CTL_PRIM_FIRST_LE || mode == CTL_PRIM_FIRST_NON_DELTA_LE) L = through * Le;
                            else if (mode == CTL_PRIM_FIRST_F || mode == CTL_PRIM_FIRST_NON_DELTA_F) L = through * f_avg;
                            else L = Le + through * (uniform_sample_one_light(C, bRec, mat) + f_avg * 0.5f);
                        }
                    }
                } else {
                    L = env_eval_diff(desc, d, dX, dY);   // PrimTracer.cu:102
                }
                out[(size_t)y * W + x] = L;
                if (depth) depth[(size_t)y * W + x] = depth_d3d(h.t, nd, fd);   // g_DepthImage2.Store
            }
        }
        totalRays += C.rays;
    };
    std::vector<std::thread> tv;
    for (int i = 0; i < threads; i++) tv.emplace_back(worker);
    for (auto& t : tv) t.join();
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) add_sample(fb, W, H, (float)x, (float)y, out[(size_t)y * W + x]);
    return totalRays;
}

// Primary rays of pass `pass_index` in image order (pixel y*W+x): the first
// ray path_trace gets in oracle_render_pass (pathKernel2, PathTracer.cu:182-194),
// as traversalRay {o, eps; d, FLT_MAX}.
void oracle_camera_rays(const ctl_scene_desc* desc, uint64_t pass_index, ctl_ray* out) {
    const uint32_t nseq = 4096, len = 30;
    std::vector<float> s1((size_t)nseq * len), s2((size_t)nseq * len * 2);
    sampler_tables(pass_index, nseq, len, s1.data(), s2.data());
    const ctl_camera& cam = desc->camera;
    for (uint32_t y = 0; y < cam.height; y++)
        for (uint32_t x = 0; x < cam.width; x++) {
            Sampler rng{s1.data(), s2.data(), nseq, len, y * cam.width + x};
            V2 pX = v2((float)x, (float)y) + rng.randomFloat2();
            (void)rng.randomFloat2();
            V3 o, d;
            sensor_ray(cam, pX, o, d);
            ctl_ray& r = out[(size_t)y * cam.width + x];
            r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z; r.tmin = desc->ray_eps;
            r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z; r.tmax = FLT_MAX;
        }
}

// WavefrontPathTracer pass (ctl_wpt_render_pass); returns the rays traversed.
uint64_t oracle_wpt_render_pass(const ctl_scene_desc* desc, int32_t direct, int32_t max_path_length,
                                int32_t rr_start_depth, uint32_t passes_done, uint64_t pass_index, ctl_pixel* fb,
                                int32_t tie, int32_t threads) {
    return wpt_render(desc, direct != 0, max_path_length, rr_start_depth, passes_done, pass_index, fb, tie, threads);
}

// AnimatedMesh::k_ComputeState on caller-owned copies of the compiled arrays.
void oracle_animate(const ctl_scene_desc* desc, uint32_t anim, const float* bones0, const float* bones1, float lerp,
                    ctl_triangle_data* tri, float* woop, ctl_bvh_node* nodes, ctl_bvh_node* scene, float* mesh_boxes,
                    float* eps) {
    animate(desc, anim, bones0, bones1, lerp, tri, woop, nodes, scene, mesh_boxes, eps);
}

// SceneBVH::setTransform + SceneBVH::Build for one moved node (SceneBVH.cpp:77-89,
// DynamicScene.cpp:433-447): the instance tree `scene` (in/out, its state kept
// between calls) rebuilt along the node's path with rotations, from the
// transforms xf16 (16 per node) and the mesh boxes; eps out.
void oracle_scene_set_transform(const ctl_scene_desc* desc, ctl_bvh_node* scene, const float* mesh_boxes,
                                const float* xf16, uint32_t node, float* eps) {
    scene_rebuild(desc, scene, mesh_boxes, xf16, std::vector<uint32_t>{node}, eps);
}

// Host-side compile pieces, for checking the product's scene compiler.
void oracle_triangle_data_set(const float* P9, uint8_t mat, const float* T6, const float* N9, uint32_t* out8) {
    // TriangleData::TriangleData + setUvSetData + setData (TriangleData.cu:10-68), EXT_TRI
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // MatIndex byte (byte 6)
    w[1] = (w[1] & 0xff00ffffu) | ((uint32_t)mat << 16);
    uint16_t a0 = float_to_half(T6[0]), a1 = float_to_half(T6[1]);
    uint16_t b0 = float_to_half(T6[2]), b1 = float_to_half(T6[3]);
    uint16_t c0 = float_to_half(T6[4]), c1 = float_to_half(T6[5]);
    w[5] = a0 | ((uint32_t)a1 << 16);
    w[6] = b0 | ((uint32_t)b1 << 16);
    w[7] = c0 | ((uint32_t)c1 << 16);
    V2 t0 = v2(half_to_float_host(w[5] & 0xffff), half_to_float_host(w[5] >> 16));
    V2 t1 = v2(half_to_float_host(w[6] & 0xffff), half_to_float_host(w[6] >> 16));
    V2 t2 = v2(half_to_float_host(w[7] & 0xffff), half_to_float_host(w[7] >> 16));
    V3 v0 = v3(P9[0], P9[1], P9[2]), v1 = v3(P9[3], P9[4], P9[5]), v2_ = v3(P9[6], P9[7], P9[8]);
    V3 dP1 = v1 - v0, dP2 = v2_ - v0;
    V2 dUV1 = t1 - t0, dUV2 = t2 - t0;
    float determinant = dUV1.x * dUV2.y - dUV1.y * dUV2.x;
    V3 dpdu, dpdv;
    if (determinant == 0) {
        V3 a, b, n = normalize(cross(dP1, dP2));
        coordinateSystem(n, a, b);
        dpdu = a; dpdv = b;
    } else {
        float invDet = 1.0f / determinant;
        dpdu = ((dUV2.y * dP1 - dUV1.y * dP2) * invDet);
        dpdv = ((-dUV2.x * dP1 + dUV1.x * dP2) * invDet);
    }
    V3 n0 = v3(N9[0], N9[1], N9[2]), n1 = v3(N9[3], N9[4], N9[5]), n2 = v3(N9[6], N9[7], N9[8]);
    w[0] = (uint32_t)normal_encode(n0) | ((uint32_t)normal_encode(n1) << 16);
    w[1] = (uint32_t)normal_encode(n2) | (w[1] & 0xffff0000u);
    uint16_t ax = float_to_half(dpdu.x), ay = float_to_half(dpdu.y), az = float_to_half(dpdu.z);
    uint16_t bx = float_to_half(dpdv.x), by = float_to_half(dpdv.y), bz = float_to_half(dpdv.z);
    w[2] = ax | ((uint32_t)ay << 16);
    w[3] = az | ((uint32_t)bx << 16);
    w[4] = by | ((uint32_t)bz << 16);
    std::memcpy(out8, w, 32);
}

// ShapeSet::triData::Recalculate (ShapeSet.cu:11-22), host decode.
void oracle_light_tri(const float* woop12, const uint32_t* tri_data8, const float* xf16, float* p9, float* n3,
                      float* area) {
    M44 mat; std::memcpy(mat.d, xf16, 64);
    V3 p[3];
    woop_get(woop12, p[0], p[1], p[2]);
    // fillDG with bary (1/3, 1/3) on the host path
    ctl_triangle_data td; std::memcpy(td.w, tri_data8, 32);
    ctl_scene_desc dd{}; dd.tri_data = &td; dd.n_tri_data = 1;
    ctl_float4x4 xfm; std::memcpy(xfm.m, xf16, 64);
    dd.node_xf = &xfm;
    SceneView S{&dd};
    DG dg;
    fill_dg(S, v2(1.0f / 3.0f, 1.0f / 3.0f), 0, 0, dg, true);
    for (int i = 0; i < 3; i++) p[i] = transformPoint(mat, p[i]);
    float a = 0.5f * length(cross(p[2] - p[0], p[1] - p[0]));
    for (int i = 0; i < 3; i++) { p9[3 * i] = p[i].x; p9[3 * i + 1] = p[i].y; p9[3 * i + 2] = p[i].z; }
    n3[0] = dg.sys.n.x; n3[1] = dg.sys.n.y; n3[2] = dg.sys.n.z;
    *area = a;
}

// InfiniteLight::InfiniteLight (Light.cpp:10-58) over texture `t`: the column
// CDFs ((w + 1) x h), the row CDF (h + 1) and the row weights (h) in out, and
// (normalization, pixel_size.x, pixel_size.y) in out3
void oracle_env_tables(const ctl_texture* t, const uint32_t* tex_data, float* out, float* out3) {
    const uint32_t w = t->width, h = t->height;
    float* cdfCols = out;
    float* cdfRows = out + (size_t)(w + 1) * h;
    float* rowWeights = cdfRows + h + 1;
    auto lum = [&](uint32_t x, uint32_t y) {   // radianceMap.Sample(0, x, y).getLuminance()
        uint32_t c = tex_data[t->offsets[0] + y * w + x];
        Spec v = v3(float(c & 0xff) / 255.0f, float((c >> 8) & 0xff) / 255.0f, float((c >> 16) & 0xff) / 255.0f);
        return luminance(v);
    };
    float rowSum = 0.0f;
    cdfRows[0] = 0;
    for (uint32_t y = 0; y < h; ++y) {
        float* col = cdfCols + (size_t)y * (w + 1);
        float colSum = 0;
        col[0] = 0;
        for (uint32_t x = 0; x < w; ++x) {
            colSum += lum(x, y);
            col[x + 1] = colSum;
        }
        float norm = 1.0f / colSum;
        for (uint32_t x = 1; x < w; ++x) col[x] *= norm;   // entries 1 .. w-1; entry w is set to 1
        col[w] = 1.0f;
        float weight = cr_sin((y + 0.5f) * O_PI / (float)h);
        rowWeights[y] = weight;
        rowSum += colSum * weight;
        cdfRows[y + 1] = rowSum;
    }
    float norm = 1.0f / rowSum;
    for (uint32_t y = 1; y < h; ++y) cdfRows[y] *= norm;
    cdfRows[h] = 1.0f;
    out3[0] = 1.0f / (rowSum * (2 * O_PI / (float)w) * (O_PI / (float)h));
    out3[1] = 2 * O_PI / (float)w;
    out3[2] = O_PI / (float)h;
}

// InfiniteLight::sampleDirect for n 2D samples of the desc's environment light:
// out7 = (d.xyz, pdf, value/pdf rgb); and pdfDirect / evalEnvironment along n
// directions: out4 = (pdf, radiance rgb)
void oracle_env_sample(const ctl_scene_desc* desc, uint64_t n, const float* samples2, float* out7) {
    for (uint64_t i = 0; i < n; i++) {
        DRec dRec;
        Spec v = env_sample_direct(desc, dRec, v2(samples2[2 * i], samples2[2 * i + 1]));
        float* o = out7 + 7 * i;
        o[0] = dRec.d.x; o[1] = dRec.d.y; o[2] = dRec.d.z; o[3] = dRec.pdf; o[4] = v.x; o[5] = v.y; o[6] = v.z;
    }
}
void oracle_env_eval(const ctl_scene_desc* desc, uint64_t n, const float* dirs3, float* out4) {
    for (uint64_t i = 0; i < n; i++) {
        DRec dRec;
        dRec.d = v3(dirs3[3 * i], dirs3[3 * i + 1], dirs3[3 * i + 2]);
        dRec.measure = ESolidAngle;
        Spec v = env_eval(desc, dRec.d);
        float* o = out4 + 4 * i;
        o[0] = env_pdf_direct(desc, dRec); o[1] = v.x; o[2] = v.y; o[3] = v.z;
    }
}

void oracle_matrix_inverse(const float* in16, float* out16) {
    M44 m; std::memcpy(m.d, in16, 64);
    M44 r = inverse(m);
    std::memcpy(out16, r.d, 64);
}

// ---- final-image stage: ImagePipeline.cu copySamplesToOutput + PixelVarianceBuffer ----
static float o_to_srgb(float v) {   // toSRGBComponent (Math/Spectrum.cu:229-234)
    if (v <= (float)0.0031308) return (float)12.92 * v;
    return (float)1.055 * cr_pow(v, (float)(1.0 / 2.4)) - (float)0.055;
}
static unsigned o_to_u8(float x) {  // Float3ToCOLORREF: (unsigned char)(clamp01(x) * 255.0f)
    return (unsigned)(unsigned char)(omin(omax(x, 0.0f), 1.0f) * 255.0f);
}

void oracle_image_resolve(const ctl_pixel* fb, uint32_t w, uint32_t h, float splat, uint32_t* out) {
    for (uint64_t i = 0; i < (uint64_t)w * h; i++) {
        const ctl_pixel& p = fb[i];
        // PixelData::toSpectrum (Engine/Image.h:21-28): s / weight + s2 * splatScale
        float weight = p.weight_sum != 0 ? p.weight_sum : 1;
        Spec s = spec_div(v3(p.rgb[0], p.rgb[1], p.rgb[2]), weight) + v3(p.rgb_splat[0], p.rgb_splat[1], p.rgb_splat[2]) * splat;
        out[i] = o_to_u8(o_to_srgb(s.x)) | (o_to_u8(o_to_srgb(s.y)) << 8) | (o_to_u8(o_to_srgb(s.z)) << 16) | (255u << 24);
    }
}

void oracle_variance_add_pass(const ctl_pixel* fb, uint32_t w, uint32_t h, float splat, uint32_t tile,
                              const uint8_t* flags, ctl_pixel_variance* var) {
    const uint32_t tx = (w + tile - 1) / tile;
    for (uint32_t y = 0; y < h; y++)
        for (uint32_t x = 0; x < w; x++) {
            char f = (char)flags[(y / tile) * tx + x / tile];
            if (!f) continue;   // updateVarianceBuffer: g_BlockFlags[bIdx] (PixelVarianceBuffer.cu:15-19)
            const ctl_pixel& p = fb[(size_t)y * w + x];
            ctl_pixel_variance& v = var[(size_t)y * w + x];
            float samplerPerformed = (float)f;
            // PixelVarianceInfo::updateMoments (PixelVarianceBuffer.h:22-41)
            Spec nps = v3(p.rgb[0], p.rgb[1], p.rgb[2]) + v3(p.rgb_splat[0], p.rgb_splat[1], p.rgb_splat[2]) * splat;
            Spec est = spec_div(nps - v3(v.prev_I[0], v.prev_I[1], v.prev_I[2]), samplerPerformed);
            v.prev_I[0] = nps.x; v.prev_I[1] = nps.y; v.prev_I[2] = nps.z;
            v.weight = p.weight_sum;
            if (v.iterations_done++ % 2 == 1) {
                v.half_buffer[0] += est.x; v.half_buffer[1] += est.y; v.half_buffer[2] += est.z;
            }
            if (samplerPerformed != 0) {
                float L = est.x * 0.212671f + est.y * 0.715160f + est.z * 0.072169f;   // getLuminance (RGB)
                v.sum_x += L;
                v.sum_x2 += L * L;   // math::sqr
                v.num_samples_var++;
            }
        }
}

void oracle_variance_stats(const ctl_pixel_variance* var, uint64_t n, float* err, float* variance, float* average) {
    for (uint64_t i = 0; i < n; i++) {
        const ctl_pixel_variance& v = var[i];
        if (err) {   // computeError (PixelVarianceBuffer.h:55-62)
            Spec I = spec_div(v3(v.prev_I[0], v.prev_I[1], v.prev_I[2]), v.weight);
            Spec A = spec_div(v3(v.half_buffer[0], v.half_buffer[1], v.half_buffer[2]), float(v.iterations_done / 2));
            Spec dd = I - A;
            float sa = 0.0f; sa += fabsf(dd.x); sa += fabsf(dd.y); sa += fabsf(dd.z);
            float si = 0.0f; si += I.x; si += I.y; si += I.z;
            float e_p = sa / sqrtf(si);
            bool zero = I.x == 0.0f && I.y == 0.0f && I.z == 0.0f;
            bool nan = std::isnan(I.x) || std::isnan(I.y) || std::isnan(I.z) || std::isnan(A.x) || std::isnan(A.y) ||
                       std::isnan(A.z);
            err[i] = zero || nan ? 0.0f : omax(e_p, 1e-2f);
        }
        float N = (float)v.num_samples_var;
        if (variance) {   // VarAccumulator::Var -> VarianceFromMoments
            float invN = 1.0f / N;
            variance[i] = (v.sum_x2 - (v.sum_x * v.sum_x) * invN) * invN;
        }
        if (average) average[i] = v.sum_x / N;   // VarAccumulator::E
    }
}

}  // extern "C"

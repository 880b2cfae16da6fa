// bvh_rebuild.h — BVHRebuilder's box recomputation with tree rotations over a
// binary tree in the reference layout (BVHNodeData, TriIntersectorData.h:44-117),
// on the host: the instance tree after ctl_scene_set_transform / ctl_scene_animate
// (SceneBVH::Build -> BVHRebuilder::Build, Engine/SceneBVH.cpp:43,
// Engine/SpatialStructures/BVH/BVHRebuilder.cpp:365-450).  The mesh trees of
// animated meshes take the same steps on the device (anim.hip rebuild kernel).
//
// One node, after its children (recomputeNode, BVHRebuilder.cpp:281-340):
//   - each child slot gets the child's box: a leaf's objects' boxes extended from
//     AABB::Identity, an inner child's two stored slots (BVHNodeData::getBox,
//     both slots, an empty one included);
//   - of the four rotations that swap one child with a grandchild under the other
//     child (possible where that child has two children), the one of least SAH
//     cost (sah, :624-638: area(child + other grandchild) x their objects + area
//     (grandchild) x its objects; AABB::Area = 2 (xy + xz + yz)) replaces the pair
//     if it is strictly cheaper than area(left) x objects(left) + area(right) x
//     objects(right); the first of equal candidates wins (std::min_element).
//   - swapChildren (:691-702) moves the subtrees and the moved inner nodes'
//     parent words (d.z, the parent's float4 offset); the objects under the
//     pushed-down child change by the difference.
// Only the flagged nodes (the paths of the invalidated objects to the root,
// propagateFlag :343-362) are visited unless `all` (recomputeAll).  Leaf
// children of a visited node are always recomputed.
#pragma once
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../../include/ctl_trace.h"

namespace ctl {

struct RbBox {
    float lo[3], hi[3];
};

inline RbBox rb_identity() { return RbBox{{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}}; }
// AABB::Extend (Math/AABB.h:72-78): componentwise min / max, this box first
inline RbBox rb_union(const RbBox& a, const RbBox& b) {
    RbBox r;
    for (int k = 0; k < 3; k++) {
        r.lo[k] = a.lo[k] < b.lo[k] ? a.lo[k] : b.lo[k];
        r.hi[k] = a.hi[k] > b.hi[k] ? a.hi[k] : b.hi[k];
    }
    return r;
}
inline float rb_area(const RbBox& b) {
    const float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
    return 2.0f * (x * y + x * z + y * z);
}
inline RbBox rb_slot(const ctl_bvh_node& n, int c) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    return RbBox{{n.v[o], n.v[o + 2], n.v[z]}, {n.v[o + 1], n.v[o + 3], n.v[z + 1]}};
}
inline void rb_set_slot(ctl_bvh_node& n, int c, const RbBox& b) {
    const int o = c ? 4 : 0, z = c ? 10 : 8;
    n.v[o] = b.lo[0]; n.v[o + 1] = b.hi[0]; n.v[o + 2] = b.lo[1]; n.v[o + 3] = b.hi[1];
    n.v[z] = b.lo[2]; n.v[z + 1] = b.hi[2];
}
inline int32_t rb_kid(const ctl_bvh_node& n, int c) { int32_t v; std::memcpy(&v, &n.v[12 + c], 4); return v; }
inline void rb_set_kid(ctl_bvh_node& n, int c, int32_t v) { std::memcpy(&n.v[12 + c], &v, 4); }
inline int32_t rb_parent(const ctl_bvh_node& n) { int32_t v; std::memcpy(&v, &n.v[14], 4); return v; }
inline void rb_set_parent(ctl_bvh_node& n, int32_t v) { std::memcpy(&n.v[14], &v, 4); }

// LeafBox(int32_t leaf) -> RbBox, LeafCount(int32_t leaf) -> int
template <class LeafBox, class LeafCount>
struct TreeRebuild {
    static constexpr int32_t kNone = 0x76543210;
    ctl_bvh_node* nodes;
    LeafBox leaf_box;
    LeafCount leaf_count;
    const std::vector<uint8_t>* flagged;   // per node; nullptr: every node
    std::vector<int32_t> objects;          // bvhNodeData::numLeafs per node

    static bool inner(int32_t v) { return v >= 0 && v != kNone; }
    ctl_bvh_node& at(int32_t v) { return nodes[v >> 2]; }
    int count_objects(int32_t v) {
        int n = 0;
        for (int c = 0; c < 2; c++) {
            const int32_t k = rb_kid(at(v), c);
            n += k == kNone ? 0 : k < 0 ? leaf_count(k) : count_objects(k);
        }
        return objects[v >> 2] = n;
    }
    int num(int32_t v) { return v == kNone ? 0 : v < 0 ? leaf_count(v) : objects[v >> 2]; }
    RbBox box(int32_t v) {
        if (v == kNone) return rb_identity();
        if (v < 0) return rb_union(rb_identity(), leaf_box(v));
        return rb_union(rb_slot(at(v), 0), rb_slot(at(v), 1));
    }
    int grandchildren(int32_t v, int c) {
        const int32_t k = rb_kid(at(v), c);
        return inner(k) ? (rb_kid(at(k), 0) != kNone) + (rb_kid(at(k), 1) != kNone) : 0;
    }
    float rotation_cost(int32_t v, int lc, int lg) {
        const int32_t child = rb_kid(at(v), lc), other = rb_kid(at(v), 1 - lc);
        const int32_t grand = rb_kid(at(other), lg), og = rb_kid(at(other), 1 - lg);
        const float ga = rb_area(box(grand));
        const int gn = num(grand);
        const RbBox lhs = rb_union(box(child), box(og));
        return rb_area(lhs) * (float)(num(child) + num(og)) + ga * (float)gn;
    }
    void put(int32_t v, int c, int32_t k) {
        rb_set_kid(at(v), c, k);
        rb_set_slot(at(v), c, box(k));
        if (inner(k)) rb_set_parent(at(k), v);
    }
    void rotate(int32_t v, int lc, int lg) {
        const int32_t child = rb_kid(at(v), lc), other = rb_kid(at(v), 1 - lc);
        const int32_t grand = rb_kid(at(other), lg);
        put(other, lg, child);
        rb_set_slot(at(v), 1 - lc, box(other));
        put(v, lc, grand);
        objects[other >> 2] += num(child) - num(grand);
    }
    void visit(int32_t v) {
        const int32_t c[2] = {rb_kid(at(v), 0), rb_kid(at(v), 1)};
        bool modified = false;
        for (int i = 0; i < 2; i++) {
            const bool leaf = c[i] < 0;
            if (!leaf && (c[i] == kNone || (flagged && !(*flagged)[c[i] >> 2]))) continue;
            modified = true;
            if (!leaf) visit(c[i]);
            rb_set_slot(at(v), i, box(c[i]));
        }
        if (!modified) return;
        float cost[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
        if (grandchildren(v, 0) == 2) { cost[0] = rotation_cost(v, 1, 0); cost[1] = rotation_cost(v, 1, 1); }
        if (grandchildren(v, 1) == 2) { cost[2] = rotation_cost(v, 0, 1); cost[3] = rotation_cost(v, 0, 0); }
        int best = 0;
        for (int i = 1; i < 4; i++)
            if (cost[i] < cost[best]) best = i;
        const float now = rb_area(box(c[0])) * (float)num(c[0]) + rb_area(box(c[1])) * (float)num(c[1]);
        if (cost[best] < now) rotate(v, best < 2 ? 1 : 0, best == 1 || best == 2 ? 1 : 0);
    }
    // root: a tree's start node (float4 offset); n_nodes sizes the object counts
    void run(int32_t root, size_t n_nodes) {
        objects.assign(n_nodes, 0);
        count_objects(root);
        if (!flagged || (*flagged)[root >> 2]) visit(root);
    }
};

template <class LeafBox, class LeafCount>
TreeRebuild<LeafBox, LeafCount> make_tree_rebuild(ctl_bvh_node* nodes, LeafBox lb, LeafCount lc,
                                                  const std::vector<uint8_t>* flagged) {
    return TreeRebuild<LeafBox, LeafCount>{nodes, lb, lc, flagged, {}};
}

// The flags of propagateFlag: every node holding one of the leaves `hit(leaf)`
// selects, and its ancestors through the parent words.
template <class Hit>
std::vector<uint8_t> flag_paths(const ctl_bvh_node* nodes, size_t n_nodes, Hit hit) {
    std::vector<uint8_t> f(n_nodes, 0);
    for (size_t k = 0; k < n_nodes; k++)
        for (int c = 0; c < 2; c++) {
            const int32_t v = rb_kid(nodes[k], c);
            if (v >= 0 || !hit(v)) continue;
            for (int32_t a = (int32_t)(k * 4); a >= 0 && (size_t)(a >> 2) < n_nodes && !f[a >> 2];
                 a = rb_parent(nodes[a >> 2]))
                f[a >> 2] = 1;
        }
    return f;
}

}  // namespace ctl

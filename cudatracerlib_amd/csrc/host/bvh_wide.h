// bvh_wide.h — 4-wide BVH collapsed from the reference's binary BVHNodeData.
//
// The boundary takes the reference layout (two children per 64-B node,
// SplitBVHBuilder.cpp:163-203); on upload each binary tree is collapsed into
// 128-B four-child nodes for the device traversal:
//
//   float4 lo_x, hi_x, lo_y, hi_y, lo_z, hi_z   child boxes, one child per lane of the float4
//   int4   child                                >= 0: node index in this tree,
//                                               < 0: ~first leaf entry (unchanged reference
//                                                    TriIntersectorData2 ranges),
//                                               0x76543210: empty slot / reference sentinel
//   int4   pad
//
// Empty slots and sentinel children have quiet-NaN boxes (no ray enters them).
//
// Which binary nodes become wide nodes is chosen by the SAH-optimal dynamic
// program over the fixed leaves (minimum summed surface area of the wide
// nodes; bvh_wide.cpp).  Against the greedy collapse (open the inner child of
// largest surface area until four children) C3 2606 -> 2647 Mrays/s
// (profiles/r02_collapse_dp_vs_greedy.txt).  Leaves, leaf entries and Woop data are shared with
// the binary tree.
#pragma once
#include <cstdint>
#include <vector>
#include "../../../include/ctl_trace.h"

namespace ctl {

struct alignas(16) WideNode {
    float lo_x[4], hi_x[4], lo_y[4], hi_y[4], lo_z[4], hi_z[4];
    int32_t child[4];
    int32_t pad[4];
};
static_assert(sizeof(WideNode) == 128, "wide node is 128 B");

// Collapses the binary tree rooted at `root_value` (a BVHNodeData child value:
// >= 0 inner node float4 offset, i.e. 4 x node index) of `nodes` and appends
// the wide nodes to `out`.  Returns the root's index relative to the first
// node appended; child indices are relative to that first node as well.
// src (optional): for every emitted node's 4 slots, the binary node index << 1 |
// child slot the slot's box was taken from (0xFFFFFFFF for empty / sentinel slots),
// indexed like the appended nodes — what a refit of the binary tree needs to
// refresh the wide boxes with one gather.
// idx (optional, mesh trees): the tree's TriIntersectorData2 entries (n_idx of
// them, indexed by the leaf values).  With it, every leaf child carries its
// entry count: child = ~((first_entry << 3) | count) with count 1..7, or 0 for
// a leaf of 8 or more entries (the traversal then walks the last-in-leaf
// flags, as the reference does); see wide_leaf_code.  Without it (the
// instance tree) leaf children stay ~first value.
int32_t collapse_wide(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, std::vector<WideNode>& out,
                      std::vector<uint32_t>* src = nullptr, const ctl_tri_index* idx = nullptr, size_t n_idx = 0);

// Leaf child of a counted mesh tree: ~((first << 3) | count), count 1..7 or 0 (>= 8).
// Entries are < 2^28 (the upload refuses larger meshes in this mode).
inline int32_t wide_leaf_code(uint32_t first, uint32_t count) {
    return ~(int32_t)((first << 3) | (count <= 7 ? count : 0u));
}
constexpr uint32_t kWideLeafMaxEntry = 1u << 28;

// Worst-case traversal stack of a tree (entries, the bottom sentinel
// included) for the traversal in device/traverse.h: a node pushes every
// child but the one it descends into, so the deepest stack is 1 + the largest
// sum of (children - 1) along a root-to-node path.  Children are counted
// without sentinel / empty slots; leaves count (a leaf child can be pushed).
// Throws on a malformed tree (offset out of range, a node reached twice).
// Stops and returns `cap` + 1 once the bound passes `cap`.
int binary_stack_bound(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, int cap);
int wide_stack_bound(const WideNode* nodes, size_t n_nodes, int32_t root, int cap);

}  // namespace ctl

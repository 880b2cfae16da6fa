// bvh_w8.h — 8-wide compressed BVH ("W8") built on upload from the reference's
// binary BVHNodeData (SplitBVHBuilder.cpp:163-203) of a one-mesh scene.
//
// One 80-B node = five 16-B loads, for eight children (the 4-wide float node
// needs seven for four):
//
//   float  px, py, pz               quantization grid origin (minimum corner of the children)
//   uint8  ex, ey, ez               grid step per axis 2^(e - 127): the fp32 exponent field
//   uint8  imask                    bit s: slot s holds an inner child
//   uint32 child_base               the inner child in slot s is node child_base + s
//   uint32 leaf_base                first leaf entry (relaid arrays) of this node's leaf children
//   uint8  meta[8]                  leaf slot: (entry bits (1 << count) - 1) << 5 | offset from
//                                   leaf_base, count 1..3; inner / empty slot: 0
//   uint8  qlo_x[8], qhi_x[8], qlo_y[8], qhi_y[8], qlo_z[8], qhi_z[8]
//                                   child bounds on the grid, rounded outward
//                                   (p + q s <= lo and p + q s >= hi exactly);
//                                   an empty slot has qlo = 255 > qhi = 0
//
// Children are placed in slots by ray octant (Ylitie, Karras, Laine 2017): the
// child nearest for rays of octant o (direction signs = the bits of o, set =
// negative) sits in slot o, so visiting slots in increasing slot ^ octant
// order is near-to-far without a sort.  Which binary nodes become W8 nodes is
// the SAH-optimal dynamic program of bvh_wide.h with eight slots; the leaves
// are the binary tree's.  Each node's leaf entries are copied next to each
// other (slot order) into relaid TriIntersectorData / TriIntersectorData2
// arrays, so a node's hit leaves are one 24-bit mask over leaf_base.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/ctl_trace.h"

namespace ctl {

struct alignas(16) W8Node {
    float px, py, pz;
    uint8_t ex, ey, ez, imask;
    uint32_t child_base;
    uint32_t leaf_base;
    uint8_t meta[8];
    uint8_t qlo_x[8], qhi_x[8], qlo_y[8], qhi_y[8], qlo_z[8], qhi_z[8];
};
static_assert(sizeof(W8Node) == 80, "W8 node is 80 B");

constexpr uint32_t kW8MaxNodes = 1u << 24;   // a stack group is (24-bit child base, 8-bit hit mask)
constexpr uint32_t kW8MaxLeaf = 3;           // entries per leaf child (3 meta bits)

struct W8Tree {
    std::vector<W8Node> nodes;        // root at node 0
    std::vector<ctl_woop_tri> woop;   // leaf entries in node order (+ nothing past the end)
    std::vector<uint32_t> idx;        // their TriIntersectorData2 words (last-in-leaf flags as given)
    int stack_bound = 0;              // deepest group stack of any ray (entries, sentinel included)
};

// The W8 tree of one mesh: binary nodes `nodes` (root value root_value, a float4
// offset), its Woop data and leaf entries (woop[e], idx[e], e < n_idx).  False,
// with the reason in *why, when the tree cannot be represented (a leaf of more
// than kW8MaxLeaf entries, a root that is a leaf, 2^24 nodes or more, a box that
// is not finite or too wide to quantize); the caller then keeps the 4-wide tree.
bool build_w8(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, const ctl_woop_tri* woop,
              const ctl_tri_index* idx, size_t n_idx, W8Tree& out, std::string* why);

// Traversal visits slot s in increasing key s ^ oct, oct = the sign bits of
// the ray's inverse direction (x: bit 0, y: bit 1, z: bit 2).

}  // namespace ctl

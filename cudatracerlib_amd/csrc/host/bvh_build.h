// bvh_build.h — parallel binned-SAH BVH builder emitting the reference's
// BVHNodeData / TriIntersectorData2 layout (Engine/TriIntersectorData.h:8-117)
// in the DFS order of SplitBVHBuilder's handleNode (SplitBVHBuilder.cpp:163-203):
//   inner node k -> child value 4*k (float4 offset), leaf -> ~first leaf entry,
//   leaf entries numbered in DFS order, last entry of a leaf flagged (bit 0),
//   a root that is a single leaf -> one inner node {leaf, 0x76543210} whose
//   right box is the zero box (handleNode's level-0 branch).
#pragma once
#include <cstdint>
#include <vector>
#include "../../../include/ctl_trace.h"

namespace ctl {

struct Box { float lo[3], hi[3]; };

struct BvhBuildParams {
    uint32_t max_leaf = 8;        // Platform::m_maxLeafSize = 8 (BVHBuilderHelper.cpp:119,136)
    uint32_t bins = 32;           // binned SAH (the reference sweeps sorted refs)
    uint32_t threads = 0;         // 0 = hardware concurrency
    uint32_t median_depth = 40;   // beyond this depth: median splits (bounds depth <= 64)
    bool leaf_size_one = false;   // top-level (instance) BVH: one object per leaf, leaf = ~object
};

struct BvhOutput {
    std::vector<ctl_bvh_node> nodes;     // inner nodes
    std::vector<uint32_t> leaf_objects;  // object id of each leaf entry (DFS order)
    std::vector<uint8_t> leaf_last;      // 1 if entry is the last of its leaf
    int32_t start_node = 0x76543210;     // root value (inner: 0, single object w/ leaf_size_one: ~obj)
    uint32_t max_depth = 0;
    uint64_t duplicates = 0;             // SBVH: references added by spatial splits
    Box root_box;
};

// Builds over `n` references: box `boxes[i]` of object `ids[i]` (ids == NULL:
// object i).  An object may have several references (split triangles); leaf
// entries carry the object id.  Degenerate boxes (min extent < 0 or a
// line/point: sum(size)==max(size)) are dropped like the reference's "Remove
// degenerates" step (SplitBVHBuilder.cpp:296-303).
void build_bvh(const Box* boxes, uint32_t n, const BvhBuildParams& p, BvhOutput& out, const uint32_t* ids = nullptr);

// SBVH of the reference's SplitBVHBuilder (SplitBVHBuilder.cpp:232-597) over
// triangles t = V[9t .. 9t+8]; see bvh_build.cpp.  Platform and BuildParams
// defaults of the reference: leaves of 1..8 references, splitAlpha 1e-5,
// MaxSpatialDepth 48, MaxDepth 64, 128 spatial bins (SplitBVHBuilder.hpp:62-67,117,176).
struct SbvhParams {
    uint32_t max_leaf = 8;
    float split_alpha = 1.0e-5f;
    uint32_t spatial_bins = 128;
    uint32_t max_spatial_depth = 48;
    uint32_t max_depth = 64;
    uint32_t sweep_max = 1u << 14;   // object splits of larger nodes are binned (bins) instead of sorted
    uint32_t bins = 256;
    uint32_t threads = 0;
    float node_cost = 1.0f;          // SAH cost of one child visit relative to one triangle test (reference: 1)
};
void build_sbvh(const float* V, uint32_t ntri, const SbvhParams& p, BvhOutput& out);

}  // namespace ctl

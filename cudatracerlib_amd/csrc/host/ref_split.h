// ref_split.h — spatial splitting of large triangles' references before the
// BVH build ("early split clipping").  The reference's SBVH builder gets the
// same effect with spatial splits inside the build (SplitBVHBuilder.cpp,
// splitAlpha / MaxSpatialDepth, .hpp:62-67): a triangle whose box is large is
// referenced by several leaves, each with the box of the triangle part inside
// one cell, so rays stop entering boxes that are mostly empty.
//
// A triangle whose box surface area exceeds alpha x the mesh's mean is split
// recursively at the middle of the longest axis of its clipped box, at most
// `max_depth` times; each piece's box is the box of the triangle clipped to
// the cell (Sutherland-Hodgman), widened by one ulp and clamped to the cell.
// Output order is triangle order (deterministic for any thread count).
#pragma once
#include <cstdint>
#include <vector>
#include "bvh_build.h"

namespace ctl {

struct RefSplitParams {
    float alpha = 0.0f;        // 0: off
    uint32_t max_depth = 0;    // up to 2^max_depth pieces per triangle
    uint32_t threads = 0;
};

// vertices: 9 floats per triangle (world or mesh space, as the BVH).
void split_refs(const float* tri_vertices, const Box* tri_boxes, uint64_t n_tris, const RefSplitParams& p,
                std::vector<Box>& out_boxes, std::vector<uint32_t>& out_ids);

}  // namespace ctl

// ctl_qnode.h — 64-B quantized 4-wide BVH node (device traversal format).
//
// A WideNode (host/bvh_wide.h, 128 B of float boxes) re-encoded with 8-bit
// child bounds on a per-node power-of-two grid:
//
//   float4 0   px, py, pz, sx        grid origin (the node box minimum), x step
//   float4 1   sy, sz, lo_x, hi_x    y/z steps; x bounds of children 0..3, one byte each
//   float4 2   lo_y, hi_y, lo_z, hi_z
//   int4   3   child[0..3]           as WideNode (>= 0 node, < 0 ~leaf entry, 0x76543210 empty)
//
// Decoding a bound is  p + float(q) * s  in fp32, the same expression on host and
// device (-ffp-contract=off).  The encoder picks, per child and axis, the
// largest q_lo whose decoded value is <= the float box's lower bound and the
// smallest q_hi whose decoded value is >= its upper bound, so every decoded box
// contains its float box.  The slab test is monotone in the box bounds, so a
// ray that enters the float box enters the decoded one: the quantized
// traversal visits a superset of the float traversal's nodes and returns the
// same hits.
#pragma once
#include "ctl_math.h"

namespace ctl {

struct alignas(16) QWideNode {
    float px, py, pz, sx;
    float sy, sz;
    uint32_t lo_x, hi_x;
    uint32_t lo_y, hi_y, lo_z, hi_z;
    int32_t child[4];
};
static_assert(sizeof(QWideNode) == 64, "quantized wide node is 64 B");

CTL_HD float qdecode(float p, uint32_t q, float s) { return p + (float)q * s; }

// One axis: origin and power-of-two step covering [lo_min, hi_max] with 255
// steps; false when the range is not finite or too wide for fp32.
CTL_HD bool qgrid(float lo_min, float hi_max, float& p, float& s) {
    if (!(lo_min <= hi_max) || !(hi_max - lo_min < 3.0e38f) || !(lo_min > -3.0e38f) || !(hi_max < 3.0e38f))
        return false;
    p = lo_min;
    s = 0x1p-100f;
    const float ext = hi_max - lo_min;
    while (s * 255.0f < ext && s < 0x1p100f) s *= 2.0f;
    while (qdecode(p, 255u, s) < hi_max) {
        if (s >= 0x1p100f) return false;
        s *= 2.0f;
    }
    return true;
}

CTL_HD uint32_t qlo(float p, float s, float lo) {   // largest q with decode <= lo
    float g = (lo - p) / s;
    uint32_t q = g <= 0.0f ? 0u : (g >= 255.0f ? 255u : (uint32_t)g);
    while (q > 0 && qdecode(p, q, s) > lo) q--;
    while (q < 255 && qdecode(p, q + 1, s) <= lo) q++;
    return q;
}

CTL_HD uint32_t qhi(float p, float s, float hi) {   // smallest q with decode >= hi
    float g = (hi - p) / s;
    uint32_t q = g <= 0.0f ? 0u : (g >= 255.0f ? 255u : (uint32_t)g);
    while (q < 255 && qdecode(p, q, s) < hi) q++;
    while (q > 0 && qdecode(p, q - 1, s) >= hi) q--;
    return q;
}

// lo/hi[axis][child] float boxes of a wide node, child[i] as stored.  Returns
// false when a box cannot be quantized (non-finite coordinates).
CTL_HD bool quantize_wide(const float lo[3][4], const float hi[3][4], const int32_t child[4], QWideNode& out) {
    float p[3], s[3];
    for (int a = 0; a < 3; a++) {
        float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
        bool any = false;
        for (int i = 0; i < 4; i++) {
            if (child[i] == 0x76543210) continue;
            any = true;
            mn = tmin(mn, lo[a][i]);
            mx = tmax(mx, hi[a][i]);
        }
        if (!any) { mn = 0.0f; mx = 0.0f; }
        if (!qgrid(mn, mx, p[a], s[a])) return false;
    }
    uint32_t qlw[3] = {0, 0, 0}, qhw[3] = {0, 0, 0};
    for (int i = 0; i < 4; i++) {
        for (int a = 0; a < 3; a++) {
            uint32_t l = 255u, h = 0u;   // empty slot
            if (child[i] != 0x76543210) {
                l = qlo(p[a], s[a], lo[a][i]);
                h = qhi(p[a], s[a], hi[a][i]);
            }
            qlw[a] |= l << (8 * i);
            qhw[a] |= h << (8 * i);
        }
        out.child[i] = child[i];
    }
    out.px = p[0]; out.py = p[1]; out.pz = p[2];
    out.sx = s[0]; out.sy = s[1]; out.sz = s[2];
    out.lo_x = qlw[0]; out.hi_x = qhw[0];
    out.lo_y = qlw[1]; out.hi_y = qhw[1];
    out.lo_z = qlw[2]; out.hi_z = qhw[2];
    return true;
}

}  // namespace ctl

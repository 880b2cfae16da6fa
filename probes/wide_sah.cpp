// wide_sah.cpp — host probe: expected inner-node visits per ray of the
// SAH-optimal W-wide collapse of a compiled scene's binary BVH, for W = 2, 4, 8
// (sum of the wide nodes' surface areas over the root's, the quantity the
// collapse DP of host/bvh_wide.cpp minimises; leaves are fixed, so triangle
// tests are the same for every W).  Used to size the 8-wide node experiment.
//   g++ -O2 -std=c++17 probes/wide_sah.cpp -Iinclude -Lcudatracerlib_amd/_lib -lctl_trace \
//       -Wl,-rpath,$PWD/cudatracerlib_amd/_lib -o /tmp/wide_sah && /tmp/wide_sah 3 0.1
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "ctl_trace.h"

namespace {
const int32_t kSent = 0x76543210;
bool inner(int32_t v) { return v >= 0 && v != kSent; }
struct Box { float lo[3], hi[3]; };
float area(const Box& b) {
    float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
    return 2.0f * (x * y + x * z + y * z);
}
void kids(const ctl_bvh_node& n, Box& a, Box& b, int32_t& va, int32_t& vb) {
    a = Box{{n.v[0], n.v[2], n.v[8]}, {n.v[1], n.v[3], n.v[9]}};
    b = Box{{n.v[4], n.v[6], n.v[10]}, {n.v[5], n.v[7], n.v[11]}};
    std::memcpy(&va, &n.v[12], 4);
    std::memcpy(&vb, &n.v[13], 4);
}
}  // namespace

int main(int argc, char** argv) {
    const int config = argc > 1 ? std::atoi(argv[1]) : 3;
    const double scale = argc > 2 ? std::atof(argv[2]) : 0.1;
    ctl_host_scene* s = ctl_host_scene_create();
    ctl_scene_desc d;
    if (ctl_host_scene_generate(s, config, scale, 1920, 1080) != CTL_OK || ctl_host_scene_compile(s, 0, &d) != CTL_OK) {
        std::fprintf(stderr, "%s\n", ctl_host_last_error());
        return 1;
    }
    const size_t n = d.n_bvh_nodes;
    std::printf("config %d scale %.3f: %llu tris, %zu binary nodes, %llu refs\n", config, scale,
                (unsigned long long)d.n_tri_data, n, (unsigned long long)d.n_tri_indices);
    // post order (children before parents) from the mesh root 0
    std::vector<int32_t> order;
    std::vector<int32_t> st{0};
    while (!st.empty()) {
        int32_t v = st.back();
        st.pop_back();
        order.push_back(v);
        Box a, b;
        int32_t va, vb;
        kids(d.bvh_nodes[v / 4], a, b, va, vb);
        if (inner(va)) st.push_back(va);
        if (inner(vb)) st.push_back(vb);
    }
    std::reverse(order.begin(), order.end());
    Box a0, b0;
    int32_t x0, y0;
    kids(d.bvh_nodes[0], a0, b0, x0, y0);
    Box root{{std::min(a0.lo[0], b0.lo[0]), std::min(a0.lo[1], b0.lo[1]), std::min(a0.lo[2], b0.lo[2])},
             {std::max(a0.hi[0], b0.hi[0]), std::max(a0.hi[1], b0.hi[1]), std::max(a0.hi[2], b0.hi[2])}};
    for (int W : {2, 4, 8}) {
        std::vector<float> g(n * W, 0.0f);
        std::vector<int> cnt(n * W, 0);   // wide nodes in the optimal collapse with budget k
        for (int32_t v : order) {
            Box a, b;
            int32_t va, vb;
            kids(d.bvh_nodes[v / 4], a, b, va, vb);
            auto G = [&](int32_t c, int k) { return inner(c) ? g[(size_t)c / 4 * W + (k - 1)] : 0.0f; };
            auto N = [&](int32_t c, int k) { return inner(c) ? cnt[(size_t)c / 4 * W + (k - 1)] : 0; };
            Box u{{std::min(a.lo[0], b.lo[0]), std::min(a.lo[1], b.lo[1]), std::min(a.lo[2], b.lo[2])},
                  {std::max(a.hi[0], b.hi[0]), std::max(a.hi[1], b.hi[1]), std::max(a.hi[2], b.hi[2])}};
            const Box& box = vb == kSent ? a : (va == kSent ? b : u);
            float best = std::numeric_limits<float>::infinity();
            int bn = 0;
            for (int j = 1; j < W; j++) {
                float c = G(va, j) + G(vb, W - j);
                if (c < best) { best = c; bn = N(va, j) + N(vb, W - j); }
            }
            const size_t x = (size_t)v / 4;
            const float f = area(box) + best;
            g[x * W] = f;
            cnt[x * W] = bn + 1;
            for (int k = 2; k <= W; k++) {
                float bk = f;
                int nk = bn + 1;
                for (int j = 1; j < k; j++) {
                    float c = G(va, j) + G(vb, k - j);
                    if (c < bk) { bk = c; nk = N(va, j) + N(vb, k - j); }
                }
                g[x * W + k - 1] = bk;
                cnt[x * W + k - 1] = nk;
            }
        }
        std::printf("W=%d: SAH node visits per ray (area sum / root area) %.3f, wide nodes %d\n", W,
                    g[0] / area(root), cnt[0]);
    }
    ctl_host_scene_destroy(s);
    return 0;
}

// bvh_build.cpp — see bvh_build.h.  Binned SAH with the reference's SAH costs
// (node cost 1 per child, triangle cost 1: SplitBVHBuilder.hpp Platform,
// SplitBVHBuilder.cpp:306-330), parallel over subtrees and over the binning of
// large nodes, then a serial DFS emission into the reference layout.
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cstring>
#include <mutex>
#include <thread>

namespace ctl {
namespace {

const int32_t kSentinel = 0x76543210;

struct Ref {
    float lo[3], hi[3];
    uint32_t id;
};

struct BNode {
    Box box;
    int32_t left, right;    // child node indices (inner)
    uint32_t first, count;  // ref range (leaf)
    uint8_t leaf;
};

inline float box_area(const Box& b) {   // AABB::Area (Math/AABB.h:19-23)
    float ax = b.hi[0] - b.lo[0], ay = b.hi[1] - b.lo[1], az = b.hi[2] - b.lo[2];
    return 2.0f * (ax * ay + ax * az + ay * az);
}
inline void box_empty(Box& b) {
    for (int k = 0; k < 3; k++) { b.lo[k] = FLT_MAX; b.hi[k] = -FLT_MAX; }
}
inline void box_grow(Box& b, const float lo[3], const float hi[3]) {
    for (int k = 0; k < 3; k++) {
        b.lo[k] = std::min(b.lo[k], lo[k]);
        b.hi[k] = std::max(b.hi[k], hi[k]);
    }
}
inline void box_merge(Box& b, const Box& o) { box_grow(b, o.lo, o.hi); }

struct Builder {
    const BvhBuildParams& p;
    std::vector<Ref> refs;
    std::vector<BNode> nodes;
    std::atomic<uint32_t> node_count{0};
    std::atomic<int> active{1};
    int max_threads;
    std::atomic<uint32_t> max_depth{0};

    explicit Builder(const BvhBuildParams& pp) : p(pp) {}

    uint32_t alloc_node() { return node_count.fetch_add(1); }

    struct Bin { Box b; uint32_t n; };

    // bounds of refs and of their centroids (lo+hi, like sortCompare's key)
    void range_bounds(uint32_t b, uint32_t e, Box& bb, Box& cb, int nthreads) {
        auto work = [&](uint32_t s, uint32_t t, Box& ob, Box& oc) {
            box_empty(ob); box_empty(oc);
            for (uint32_t i = s; i < t; i++) {
                const Ref& r = refs[i];
                box_grow(ob, r.lo, r.hi);
                float c[3] = {r.lo[0] + r.hi[0], r.lo[1] + r.hi[1], r.lo[2] + r.hi[2]};
                box_grow(oc, c, c);
            }
        };
        if (nthreads <= 1 || e - b < 65536) { work(b, e, bb, cb); return; }
        std::vector<Box> pb(nthreads), pc(nthreads);
        std::vector<std::thread> ts;
        uint32_t chunk = (e - b + nthreads - 1) / nthreads;
        for (int t = 0; t < nthreads; t++) {
            uint32_t s = std::min(e, b + t * chunk), f = std::min(e, s + chunk);
            ts.emplace_back([&, s, f, t] { work(s, f, pb[t], pc[t]); });
        }
        for (auto& t : ts) t.join();
        box_empty(bb); box_empty(cb);
        for (int t = 0; t < nthreads; t++) { box_merge(bb, pb[t]); box_merge(cb, pc[t]); }
    }

    void bin_range(uint32_t b, uint32_t e, const Box& cb, int nthreads, std::vector<Bin>& bins) {
        const uint32_t B = p.bins;
        bins.assign(3 * B, Bin{});
        for (auto& x : bins) { box_empty(x.b); x.n = 0; }
        auto work = [&](uint32_t s, uint32_t t, std::vector<Bin>& out) {
            float scale[3];
            for (int k = 0; k < 3; k++) {
                float ext = cb.hi[k] - cb.lo[k];
                scale[k] = ext > 0 ? (float)B * (1.0f - 1e-6f) / ext : 0.0f;
            }
            for (uint32_t i = s; i < t; i++) {
                const Ref& r = refs[i];
                for (int k = 0; k < 3; k++) {
                    float c = r.lo[k] + r.hi[k];
                    uint32_t bi = (uint32_t)std::max(0.0f, std::min((float)(B - 1), (c - cb.lo[k]) * scale[k]));
                    Bin& x = out[k * B + bi];
                    box_grow(x.b, r.lo, r.hi);
                    x.n++;
                }
            }
        };
        if (nthreads <= 1 || e - b < 65536) { work(b, e, bins); return; }
        std::vector<std::vector<Bin>> part(nthreads, bins);
        std::vector<std::thread> ts;
        uint32_t chunk = (e - b + nthreads - 1) / nthreads;
        for (int t = 0; t < nthreads; t++) {
            uint32_t s = std::min(e, b + t * chunk), f = std::min(e, s + chunk);
            ts.emplace_back([&, s, f, t] { work(s, f, part[t]); });
        }
        for (auto& t : ts) t.join();
        for (int t = 0; t < nthreads; t++)
            for (size_t i = 0; i < bins.size(); i++) { box_merge(bins[i].b, part[t][i].b); bins[i].n += part[t][i].n; }
    }

    void build(uint32_t nodeIdx, uint32_t b, uint32_t e, uint32_t depth) {
        uint32_t md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
        BNode& nd = nodes[nodeIdx];
        uint32_t count = e - b;
        int par = (count > (1u << 20)) ? max_threads : 1;
        Box bb, cb;
        range_bounds(b, e, bb, cb, par);
        nd.box = bb;
        const uint32_t maxLeaf = p.leaf_size_one ? 1u : p.max_leaf;
        if (count <= 1) { nd.leaf = 1; nd.first = b; nd.count = count; return; }

        float area = box_area(bb);
        float leafSAH = area * (float)count;
        float nodeSAH = area * 2.0f;
        int bestAxis = -1;
        uint32_t bestSplit = 0;
        float bestSAH = FLT_MAX;
        bool median = depth >= p.median_depth;
        if (!median) {
            std::vector<Bin> bins;
            bin_range(b, e, cb, par, bins);
            const uint32_t B = p.bins;
            std::vector<float> rightArea(B);
            std::vector<uint32_t> rightCount(B);
            for (int k = 0; k < 3; k++) {
                if (!(cb.hi[k] > cb.lo[k])) continue;
                Box acc; box_empty(acc); uint32_t n = 0;
                for (int i = (int)B - 1; i > 0; i--) {
                    box_merge(acc, bins[k * B + i].b); n += bins[k * B + i].n;
                    rightArea[i] = n ? box_area(acc) : 0.0f; rightCount[i] = n;
                }
                box_empty(acc); n = 0;
                for (uint32_t i = 1; i < B; i++) {
                    box_merge(acc, bins[k * B + i - 1].b); n += bins[k * B + i - 1].n;
                    if (n == 0 || rightCount[i] == 0) continue;
                    float sah = nodeSAH + box_area(acc) * (float)n + rightArea[i] * (float)rightCount[i];
                    if (sah < bestSAH) { bestSAH = sah; bestAxis = k; bestSplit = i; }
                }
            }
            if (count <= maxLeaf && leafSAH <= bestSAH) { nd.leaf = 1; nd.first = b; nd.count = count; return; }
        } else if (count <= maxLeaf) {
            nd.leaf = 1; nd.first = b; nd.count = count; return;
        }

        uint32_t mid;
        if (bestAxis >= 0) {
            const uint32_t B = p.bins;
            float ext = cb.hi[bestAxis] - cb.lo[bestAxis];
            float scale = (float)B * (1.0f - 1e-6f) / ext;
            float lo = cb.lo[bestAxis];
            int ax = bestAxis;
            auto it = std::partition(refs.begin() + b, refs.begin() + e, [&](const Ref& r) {
                float c = r.lo[ax] + r.hi[ax];
                uint32_t bi = (uint32_t)std::max(0.0f, std::min((float)(B - 1), (c - lo) * scale));
                return bi < bestSplit;
            });
            mid = (uint32_t)(it - refs.begin());
            if (mid == b || mid == e) mid = b + count / 2;   // cannot happen; keep the tree valid
        } else {
            // all centroids coincide (or median mode): split by count along the widest centroid axis
            int ax = 0;
            float w = -1;
            for (int k = 0; k < 3; k++)
                if (cb.hi[k] - cb.lo[k] > w) { w = cb.hi[k] - cb.lo[k]; ax = k; }
            mid = b + count / 2;
            std::nth_element(refs.begin() + b, refs.begin() + mid, refs.begin() + e, [ax](const Ref& x, const Ref& y) {
                float cx = x.lo[ax] + x.hi[ax], cy = y.lo[ax] + y.hi[ax];
                return cx < cy || (cx == cy && x.id < y.id);
            });
        }
        nd.leaf = 0;
        uint32_t l = alloc_node(), r = alloc_node();
        nd.left = (int32_t)l;
        nd.right = (int32_t)r;
        bool spawn = (e - b) > 4096 && active.load() < max_threads;
        if (spawn) {
            active.fetch_add(1);
            std::thread t([this, l, b, mid, depth] { build(l, b, mid, depth + 1); active.fetch_sub(1); });
            build(r, mid, e, depth + 1);
            t.join();
        } else {
            build(l, b, mid, depth + 1);
            build(r, mid, e, depth + 1);
        }
    }
};

void set_box(ctl_bvh_node& n, int side, const Box& b) {   // BVHNodeData::setLeft/setRight
    if (side == 0) {
        n.v[0] = b.lo[0]; n.v[1] = b.hi[0]; n.v[2] = b.lo[1]; n.v[3] = b.hi[1];
        n.v[8] = b.lo[2]; n.v[9] = b.hi[2];
    } else {
        n.v[4] = b.lo[0]; n.v[5] = b.hi[0]; n.v[6] = b.lo[1]; n.v[7] = b.hi[1];
        n.v[10] = b.lo[2]; n.v[11] = b.hi[2];
    }
}
void set_children(ctl_bvh_node& n, int32_t a, int32_t b, uint32_t parent) {
    std::memcpy(&n.v[12], &a, 4);
    std::memcpy(&n.v[13], &b, 4);
    std::memcpy(&n.v[14], &parent, 4);
    n.v[15] = 0.0f;
}

struct Emitter {
    const Builder& B;
    BvhOutput& out;
    bool leafOne;
    int32_t emit_leaf(const BNode& n) {
        if (leafOne) return ~(int32_t)B.refs[n.first].id;
        uint32_t first = (uint32_t)out.leaf_objects.size();
        for (uint32_t i = 0; i < n.count; i++) {
            out.leaf_objects.push_back(B.refs[n.first + i].id);
            out.leaf_last.push_back(i + 1 == n.count ? 1 : 0);
        }
        return ~(int32_t)first;
    }
    int32_t emit(uint32_t idx, int level, uint32_t parent) {
        const BNode& n = B.nodes[idx];
        if (n.leaf) return emit_leaf(n);
        uint32_t k = (uint32_t)out.nodes.size();
        out.nodes.push_back(ctl_bvh_node{});
        int32_t val = (int32_t)(k * 4);
        int32_t a = emit((uint32_t)n.left, level + 1, (uint32_t)val);
        int32_t b = emit((uint32_t)n.right, level + 1, (uint32_t)val);
        ctl_bvh_node& node = out.nodes[k];
        set_children(node, a, b, parent);
        set_box(node, 0, B.nodes[n.left].box);
        set_box(node, 1, B.nodes[n.right].box);
        return val;
    }
};

}  // namespace

void build_bvh(const Box* boxes, uint32_t n, const BvhBuildParams& p, BvhOutput& out, const uint32_t* ids) {
    out = BvhOutput{};
    Builder B(p);
    B.max_threads = (int)(p.threads ? p.threads : std::max(1u, std::thread::hardware_concurrency()));
    B.refs.reserve(n);
    for (uint32_t i = 0; i < n; i++) {
        const Box& bx = boxes[i];
        float sx = bx.hi[0] - bx.lo[0], sy = bx.hi[1] - bx.lo[1], sz = bx.hi[2] - bx.lo[2];
        float mn = std::min(sx, std::min(sy, sz)), mx = std::max(sx, std::max(sy, sz));
        if (!p.leaf_size_one && (mn < 0.0f || sx + sy + sz == mx)) continue;   // degenerate ref
        Ref r;
        std::memcpy(r.lo, bx.lo, 12);
        std::memcpy(r.hi, bx.hi, 12);
        r.id = ids ? ids[i] : i;
        B.refs.push_back(r);
    }
    uint32_t m = (uint32_t)B.refs.size();
    box_empty(out.root_box);
    if (m == 0) {
        ctl_bvh_node node{};
        Box inv; box_empty(inv);
        set_box(node, 0, inv); set_box(node, 1, inv);
        set_children(node, kSentinel, kSentinel, 0xffffffffu);
        out.nodes.push_back(node);
        out.start_node = 0;
        return;
    }
    B.nodes.resize(2 * (size_t)m + 1);
    B.node_count = 1;
    B.build(0, 0, m, 0);
    B.nodes.resize(B.node_count.load());
    out.root_box = B.nodes[0].box;
    out.max_depth = B.max_depth.load();
    Emitter E{B, out, p.leaf_size_one};
    out.nodes.reserve(B.nodes.size() / 2 + 1);
    if (B.nodes[0].leaf) {
        if (p.leaf_size_one) {   // single instance: KernelSceneBVH start node = ~object
            out.start_node = ~(int32_t)B.refs[0].id;
            return;
        }
        // root leaf: handleNode level-0 branch (SplitBVHBuilder.cpp:177-189)
        out.nodes.push_back(ctl_bvh_node{});
        int32_t leaf = E.emit_leaf(B.nodes[0]);
        ctl_bvh_node& node = out.nodes[0];
        set_children(node, leaf, kSentinel, 0xffffffffu);
        set_box(node, 0, B.nodes[0].box);
        Box zero{{0, 0, 0}, {0, 0, 0}};
        set_box(node, 1, zero);
        out.start_node = 0;
        return;
    }
    out.start_node = E.emit(0, 0, 0xffffffffu);
}

}  // namespace ctl

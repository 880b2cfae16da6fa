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

// DFS emission into the reference layout; NodeAt(i) -> const BNode&, refs = leaf references.
template <class NodeAt>
struct Emitter {
    NodeAt at;
    const std::vector<Ref>& refs;
    BvhOutput& out;
    bool leafOne;
    int32_t emit_leaf(const BNode& n) {
        if (leafOne) return ~(int32_t)refs[n.first].id;
        uint32_t first = (uint32_t)out.leaf_objects.size();
        for (uint32_t i = 0; i < n.count; i++) {
            out.leaf_objects.push_back(refs[n.first + i].id);
            out.leaf_last.push_back(i + 1 == n.count ? 1 : 0);
        }
        return ~(int32_t)first;
    }
    int32_t emit(uint32_t idx, int level, uint32_t parent) {
        const BNode& n = at(idx);
        if (n.leaf) return emit_leaf(n);
        uint32_t k = (uint32_t)out.nodes.size();
        out.nodes.push_back(ctl_bvh_node{});
        int32_t val = (int32_t)(k * 4);
        int32_t a = emit((uint32_t)n.left, level + 1, (uint32_t)val);
        int32_t b = emit((uint32_t)n.right, level + 1, (uint32_t)val);
        ctl_bvh_node& node = out.nodes[k];
        set_children(node, a, b, parent);
        set_box(node, 0, at((uint32_t)n.left).box);
        set_box(node, 1, at((uint32_t)n.right).box);
        return val;
    }
    // the whole tree from root node 0 (handleNode's level-0 rules)
    void run(int32_t leafOneRoot) {
        const BNode& root = at(0);
        if (root.leaf) {
            if (leafOne) { out.start_node = leafOneRoot; return; }   // single instance: start node = ~object
            out.nodes.push_back(ctl_bvh_node{});                    // root leaf (SplitBVHBuilder.cpp:177-189)
            int32_t leaf = emit_leaf(root);
            ctl_bvh_node& node = out.nodes[0];
            set_children(node, leaf, kSentinel, 0xffffffffu);
            set_box(node, 0, root.box);
            Box zero{{0, 0, 0}, {0, 0, 0}};
            set_box(node, 1, zero);
            out.start_node = 0;
            return;
        }
        out.start_node = emit(0, 0, 0xffffffffu);
    }
};

// ---- SBVH: the reference's SplitBVHBuilder algorithm --------------------------
// (SplitBVHBuilder.cpp:232-597, Stich et al. 2009), restated as a parallel
// builder: per node the object split (SAH sweep over the references sorted by
// box centre per axis, tie-broken towards balanced counts; binned above
// sweep_max references) and, below MaxSpatialDepth and when the object
// split's children overlap by at least splitAlpha x the root area, the spatial
// split (spatial_bins planes per axis, each reference chopped at the planes it
// crosses with the triangle's exact plane clipping, enter/exit counts); the
// lowest SAH of leaf / object / spatial wins; a spatial split decides per
// straddling reference between unsplitting it to either side and duplicating
// it (SAH of each choice).  Degenerate references (negative extent, or a line /
// point box) are dropped at every node as the reference does.
struct SbvhBuilder {
    const float* V;   // triangle t: vertices V[9t .. 9t+8]
    const SbvhParams& p;
    float min_overlap = 0.0f;
    int max_threads = 1;
    std::atomic<int> active{1};
    std::atomic<uint32_t> max_depth{0};
    std::atomic<uint64_t> duplicates{0};
    // chunked node store: indices stay valid while other threads append
    static constexpr uint32_t kChunkBits = 16;
    std::vector<std::atomic<BNode*>> chunks;
    std::atomic<uint32_t> node_count{0};
    std::mutex mtx;
    std::vector<Ref> leaf_refs;   // guarded by mtx

    struct Task {
        std::vector<Ref> leaves;            // this task's leaf references (local indices)
        std::vector<uint32_t> leaf_nodes;   // its leaf nodes, `first` relative to `leaves`
    };

    SbvhBuilder(const float* v, const SbvhParams& pp) : V(v), p(pp), chunks(1u << 16) {
        for (auto& c : chunks) c.store(nullptr);
    }
    ~SbvhBuilder() {
        for (auto& c : chunks) delete[] c.load();
    }
    BNode& node(uint32_t i) { return chunks[i >> kChunkBits].load(std::memory_order_acquire)[i & ((1u << kChunkBits) - 1)]; }
    uint32_t alloc_node() {
        const uint32_t i = node_count.fetch_add(1);
        const uint32_t c = i >> kChunkBits;
        if (!chunks[c].load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> g(mtx);
            if (!chunks[c].load(std::memory_order_relaxed)) chunks[c].store(new BNode[1u << kChunkBits], std::memory_order_release);
        }
        return i;
    }

    static bool degenerate(const Ref& r) {
        const float sx = r.hi[0] - r.lo[0], sy = r.hi[1] - r.lo[1], sz = r.hi[2] - r.lo[2];
        return std::min(sx, std::min(sy, sz)) < 0.0f || sx + sy + sz == std::max(sx, std::max(sy, sz));
    }

    // SplitNode (BVHBuilderHelper.cpp:78-113): the triangle's part on each side
    // of the plane, intersected with the reference's box.
    void split_ref(const Ref& ref, int dim, float pos, Ref& l, Ref& r) const {
        Box lb, rb;
        box_empty(lb); box_empty(rb);
        const float* T = V + 9 * (size_t)ref.id;
        const float* v1 = T + 6;
        for (int i = 0; i < 3; i++) {
            const float* v0 = v1;
            v1 = T + 3 * i;
            const float v0p = v0[dim], v1p = v1[dim];
            if (v0p <= pos) box_grow(lb, v0, v0);
            if (v0p >= pos) box_grow(rb, v0, v0);
            if ((v0p < pos && v1p > pos) || (v0p > pos && v1p < pos)) {
                const float t = std::min(1.0f, std::max(0.0f, (pos - v0p) / (v1p - v0p)));
                float q[3];
                for (int k = 0; k < 3; k++) q[k] = v0[k] + (v1[k] - v0[k]) * t;
                box_grow(lb, q, q);
                box_grow(rb, q, q);
            }
        }
        lb.hi[dim] = pos;
        rb.lo[dim] = pos;
        for (int k = 0; k < 3; k++) {   // AABB::Intersect(refBox)
            l.lo[k] = std::max(lb.lo[k], ref.lo[k]); l.hi[k] = std::min(lb.hi[k], ref.hi[k]);
            r.lo[k] = std::max(rb.lo[k], ref.lo[k]); r.hi[k] = std::min(rb.hi[k], ref.hi[k]);
        }
        l.id = r.id = ref.id;
    }

    struct ObjectSplit { float sah = FLT_MAX; int dim = -1; uint32_t num_left = 0, split_bin = 0; bool binned = false; Box lb, rb; };
    struct SpatialSplit { float sah = FLT_MAX; int dim = 0; float pos = 0; };

    static float centre(const Ref& r, int d) { return r.lo[d] + r.hi[d]; }

    ObjectSplit object_split(std::vector<Ref>& refs, float nodeSAH, bool sweep = false) {
        ObjectSplit best;
        const uint32_t n = (uint32_t)refs.size();
        if (sweep || n <= p.sweep_max) {
            std::vector<Box> right(n);
            float bestTie = FLT_MAX;
            for (int d = 0; d < 3; d++) {
                std::sort(refs.begin(), refs.end(), [d](const Ref& a, const Ref& b) {
                    const float ca = centre(a, d), cb = centre(b, d);
                    return ca < cb || (ca == cb && a.id < b.id);
                });
                Box acc; box_empty(acc);
                for (uint32_t i = n - 1; i > 0; i--) { box_grow(acc, refs[i].lo, refs[i].hi); right[i - 1] = acc; }
                box_empty(acc);
                for (uint32_t i = 1; i < n; i++) {
                    box_grow(acc, refs[i - 1].lo, refs[i - 1].hi);
                    const float sah = nodeSAH + box_area(acc) * (float)i + box_area(right[i - 1]) * (float)(n - i);
                    const float tie = (float)i * (float)i + (float)(n - i) * (float)(n - i);
                    if (sah < best.sah || (sah == best.sah && tie < bestTie)) {
                        best.sah = sah; best.dim = d; best.num_left = i; best.lb = acc; best.rb = right[i - 1];
                        bestTie = tie;
                    }
                }
            }
            return best;
        }
        // binned over box centres (large nodes)
        Box cb; box_empty(cb);
        for (const Ref& r : refs) { float c[3] = {centre(r, 0), centre(r, 1), centre(r, 2)}; box_grow(cb, c, c); }
        const uint32_t B = std::max(2u, p.bins);
        struct Bin { Box b; uint32_t n; };
        std::vector<Bin> bins(3 * B);
        for (auto& x : bins) { box_empty(x.b); x.n = 0; }
        float scale[3];
        for (int k = 0; k < 3; k++) {
            const float ext = cb.hi[k] - cb.lo[k];
            scale[k] = ext > 0 ? (float)B * (1.0f - 1e-6f) / ext : 0.0f;
        }
        for (const Ref& r : refs)
            for (int k = 0; k < 3; k++) {
                const uint32_t bi = (uint32_t)std::max(0.0f, std::min((float)(B - 1), (centre(r, k) - cb.lo[k]) * scale[k]));
                box_grow(bins[k * B + bi].b, r.lo, r.hi);
                bins[k * B + bi].n++;
            }
        std::vector<Box> rightB(B);
        std::vector<uint32_t> rightN(B);
        for (int k = 0; k < 3; k++) {
            if (!(cb.hi[k] > cb.lo[k])) continue;
            Box acc; box_empty(acc); uint32_t m = 0;
            for (int i = (int)B - 1; i > 0; i--) { box_merge(acc, bins[k * B + i].b); m += bins[k * B + i].n; rightB[i] = acc; rightN[i] = m; }
            box_empty(acc); m = 0;
            for (uint32_t i = 1; i < B; i++) {
                box_merge(acc, bins[k * B + i - 1].b); m += bins[k * B + i - 1].n;
                if (m == 0 || rightN[i] == 0) continue;
                const float sah = nodeSAH + box_area(acc) * (float)m + box_area(rightB[i]) * (float)rightN[i];
                if (sah < best.sah) {
                    best.sah = sah; best.dim = k; best.num_left = m; best.lb = acc; best.rb = rightB[i];
                    best.binned = true; best.split_bin = i;
                }
            }
        }
        if (best.dim < 0) best = object_split(refs, nodeSAH, true);   // all centres coincide: sorted sweep
        return best;
    }

    void perform_object(std::vector<Ref>& refs, const ObjectSplit& os, std::vector<Ref>& L, std::vector<Ref>& R) {
        const int d = os.dim;
        if (!os.binned) {
            std::sort(refs.begin(), refs.end(), [d](const Ref& a, const Ref& b) {
                const float ca = centre(a, d), cb = centre(b, d);
                return ca < cb || (ca == cb && a.id < b.id);
            });
            L.assign(refs.begin(), refs.begin() + os.num_left);
            R.assign(refs.begin() + os.num_left, refs.end());
            return;
        }
        Box cb; box_empty(cb);
        for (const Ref& r : refs) { float c[3] = {centre(r, 0), centre(r, 1), centre(r, 2)}; box_grow(cb, c, c); }
        const uint32_t B = std::max(2u, p.bins);
        const float ext = cb.hi[d] - cb.lo[d];
        const float scale = (float)B * (1.0f - 1e-6f) / ext;
        for (const Ref& r : refs) {   // the same bins as object_split computed
            const uint32_t bi = (uint32_t)std::max(0.0f, std::min((float)(B - 1), (centre(r, d) - cb.lo[d]) * scale));
            (bi < os.split_bin ? L : R).push_back(r);
        }
    }

    SpatialSplit spatial_split(const std::vector<Ref>& refs, const Box& bb, float nodeSAH, int nthreads) {
        SpatialSplit best;
        const int NB = (int)p.spatial_bins;
        float origin[3], size[3], inv[3];
        for (int k = 0; k < 3; k++) {
            origin[k] = bb.lo[k];
            size[k] = (bb.hi[k] - bb.lo[k]) * (1.0f / (float)NB);
            inv[k] = size[k] > 0.0f ? 1.0f / size[k] : 0.0f;
        }
        struct SBin { Box b; uint32_t enter, exit; };
        auto work = [&](size_t s, size_t t, std::vector<SBin>& bins) {
            bins.assign(3 * (size_t)NB, SBin{});
            for (auto& x : bins) { box_empty(x.b); x.enter = x.exit = 0; }
            for (size_t ri = s; ri < t; ri++) {
                const Ref& ref = refs[ri];
                for (int d = 0; d < 3; d++) {
                    if (size[d] <= 0.0f) continue;
                    const int first = std::min(NB - 1, std::max(0, (int)((ref.lo[d] - origin[d]) * inv[d])));
                    const int last = std::min(NB - 1, std::max(first, (int)((ref.hi[d] - origin[d]) * inv[d])));
                    Ref cur = ref;
                    for (int i = first; i < last; i++) {
                        Ref l, r;
                        split_ref(cur, d, origin[d] + size[d] * (float)(i + 1), l, r);
                        box_grow(bins[d * NB + i].b, l.lo, l.hi);
                        cur = r;
                    }
                    box_grow(bins[d * NB + last].b, cur.lo, cur.hi);
                    bins[d * NB + first].enter++;
                    bins[d * NB + last].exit++;
                }
            }
        };
        std::vector<SBin> bins;
        const size_t n = refs.size();
        if (nthreads <= 1 || n < 65536) {
            work(0, n, bins);
        } else {
            std::vector<std::vector<SBin>> part(nthreads);
            std::vector<std::thread> ts;
            const size_t chunk = (n + nthreads - 1) / nthreads;
            for (int t = 0; t < nthreads; t++) {
                const size_t s = std::min(n, t * chunk), f = std::min(n, s + chunk);
                ts.emplace_back([&, s, f, t] { work(s, f, part[t]); });
            }
            for (auto& t : ts) t.join();
            bins = part[0];
            for (int t = 1; t < nthreads; t++)
                for (size_t i = 0; i < bins.size(); i++) {
                    box_merge(bins[i].b, part[t][i].b);
                    bins[i].enter += part[t][i].enter;
                    bins[i].exit += part[t][i].exit;
                }
        }
        std::vector<Box> right(NB);
        for (int d = 0; d < 3; d++) {
            if (size[d] <= 0.0f) continue;
            Box acc; box_empty(acc);
            for (int i = NB - 1; i > 0; i--) { box_merge(acc, bins[d * NB + i].b); right[i - 1] = acc; }
            box_empty(acc);
            uint32_t ln = 0, rn = (uint32_t)n;
            for (int i = 1; i < NB; i++) {
                box_merge(acc, bins[d * NB + i - 1].b);
                ln += bins[d * NB + i - 1].enter;
                rn -= bins[d * NB + i - 1].exit;
                const float sah = nodeSAH + box_area(acc) * (float)ln + box_area(right[i - 1]) * (float)rn;
                if (sah < best.sah) { best.sah = sah; best.dim = d; best.pos = origin[d] + size[d] * (float)i; }
            }
        }
        return best;
    }

    // performSpatialSplit (SplitBVHBuilder.cpp:520-597)
    void perform_spatial(const std::vector<Ref>& refs, const SpatialSplit& ss, std::vector<Ref>& L, std::vector<Ref>& R) {
        const int d = ss.dim;
        const float pos = ss.pos;
        Box lb, rb;
        box_empty(lb); box_empty(rb);
        std::vector<const Ref*> straddle;
        for (const Ref& r : refs) {
            if (r.hi[d] <= pos) { L.push_back(r); box_grow(lb, r.lo, r.hi); }
            else if (r.lo[d] >= pos) { R.push_back(r); box_grow(rb, r.lo, r.hi); }
            else straddle.push_back(&r);
        }
        auto area_or0 = [](const Box& b) { return b.lo[0] <= b.hi[0] ? box_area(b) : 0.0f; };
        for (const Ref* rp : straddle) {
            Ref lr, rr;
            split_ref(*rp, d, pos, lr, rr);
            Box lub = lb, rub = rb, ldb = lb, rdb = rb;
            box_grow(lub, rp->lo, rp->hi);
            box_grow(rub, rp->lo, rp->hi);
            box_grow(ldb, lr.lo, lr.hi);
            box_grow(rdb, rr.lo, rr.hi);
            const float lac = (float)L.size(), rac = (float)R.size(), lbc = lac + 1.0f, rbc = rac + 1.0f;
            const float unsplitL = box_area(lub) * lbc + area_or0(rb) * rac;
            const float unsplitR = area_or0(lb) * lac + box_area(rub) * rbc;
            const float dupl = box_area(ldb) * lbc + box_area(rdb) * rbc;
            const float m = std::min(unsplitL, std::min(unsplitR, dupl));
            if (m == unsplitL) { lb = lub; L.push_back(*rp); }
            else if (m == unsplitR) { rb = rub; R.push_back(*rp); }
            else { lb = ldb; rb = rdb; L.push_back(lr); R.push_back(rr); }
        }
    }

    void make_leaf(uint32_t idx, std::vector<Ref>& refs, Task& T) {
        BNode& nd = node(idx);
        nd.leaf = 1;
        nd.first = (uint32_t)T.leaves.size();
        nd.count = (uint32_t)refs.size();
        T.leaves.insert(T.leaves.end(), refs.begin(), refs.end());
        T.leaf_nodes.push_back(idx);
    }

    void merge(Task& T) {
        std::lock_guard<std::mutex> g(mtx);
        const uint32_t base = (uint32_t)leaf_refs.size();
        leaf_refs.insert(leaf_refs.end(), T.leaves.begin(), T.leaves.end());
        for (uint32_t i : T.leaf_nodes) node(i).first += base;
        T.leaves.clear();
        T.leaf_nodes.clear();
    }

    void build(uint32_t idx, std::vector<Ref> refs, uint32_t depth, Task& T) {
        uint32_t md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
        // remove degenerates (SplitBVHBuilder.cpp:296-303), keeping one if all are
        auto it = std::remove_if(refs.begin(), refs.end(), degenerate);
        if (it == refs.begin() && !refs.empty()) ++it;
        refs.erase(it, refs.end());
        Box bb; box_empty(bb);
        for (const Ref& r : refs) box_grow(bb, r.lo, r.hi);
        node(idx).box = bb;
        const uint32_t n = (uint32_t)refs.size();
        if (n <= 1 || depth >= p.max_depth) { make_leaf(idx, refs, T); return; }
        const float area = box_area(bb);
        const float leafSAH = area * (float)n, nodeSAH = area * 2.0f * p.node_cost;
        const int par = n > (1u << 18) ? max_threads : 1;
        ObjectSplit os = object_split(refs, nodeSAH);
        SpatialSplit ss;
        if (depth < p.max_spatial_depth) {
            Box ov;
            for (int k = 0; k < 3; k++) { ov.lo[k] = std::max(os.lb.lo[k], os.rb.lo[k]); ov.hi[k] = std::min(os.lb.hi[k], os.rb.hi[k]); }
            const bool nonempty = ov.lo[0] <= ov.hi[0] && ov.lo[1] <= ov.hi[1] && ov.lo[2] <= ov.hi[2];
            if (nonempty && box_area(ov) >= min_overlap) ss = spatial_split(refs, bb, nodeSAH, par);
        }
        const float minSAH = std::min(leafSAH, std::min(os.sah, ss.sah));
        if (minSAH == leafSAH && n <= p.max_leaf) { make_leaf(idx, refs, T); return; }
        std::vector<Ref> L, R;
        if (minSAH == ss.sah) perform_spatial(refs, ss, L, R);
        if (L.empty() || R.empty()) {
            L.clear(); R.clear();
            perform_object(refs, os, L, R);
        }
        duplicates += L.size() + R.size() - n;
        std::vector<Ref>().swap(refs);   // the parent's references are no longer needed
        const uint32_t l = alloc_node(), r = alloc_node();
        BNode& nd = node(idx);
        nd.leaf = 0;
        nd.left = (int32_t)l;
        nd.right = (int32_t)r;
        const bool spawn = L.size() > 4096 && R.size() > 4096 && active.load() < max_threads;
        if (spawn) {
            active.fetch_add(1);
            std::thread t([this, l, depth, LL = std::move(L)]() mutable {
                Task T2;
                build(l, std::move(LL), depth + 1, T2);
                merge(T2);
                active.fetch_sub(1);
            });
            build(r, std::move(R), depth + 1, T);
            t.join();
        } else {
            build(l, std::move(L), depth + 1, T);
            build(r, std::move(R), depth + 1, T);
        }
    }
};

}  // namespace

void build_sbvh(const float* V, uint32_t ntri, const SbvhParams& p, BvhOutput& out) {
    out = BvhOutput{};
    SbvhBuilder B(V, p);
    B.max_threads = (int)(p.threads ? p.threads : std::max(1u, std::thread::hardware_concurrency()));
    std::vector<Ref> refs;
    refs.reserve(ntri);
    for (uint32_t t = 0; t < ntri; t++) {
        Ref r;
        for (int k = 0; k < 3; k++) { r.lo[k] = FLT_MAX; r.hi[k] = -FLT_MAX; }
        for (int c = 0; c < 3; c++)
            for (int k = 0; k < 3; k++) {
                r.lo[k] = std::min(r.lo[k], V[9 * (size_t)t + 3 * c + k]);
                r.hi[k] = std::max(r.hi[k], V[9 * (size_t)t + 3 * c + k]);
            }
        r.id = t;
        if (!SbvhBuilder::degenerate(r)) refs.push_back(r);
    }
    box_empty(out.root_box);
    if (refs.empty()) {
        ctl_bvh_node node{};
        Box inv; box_empty(inv);
        set_box(node, 0, inv); set_box(node, 1, inv);
        set_children(node, kSentinel, kSentinel, 0xffffffffu);
        out.nodes.push_back(node);
        out.start_node = 0;
        return;
    }
    Box rb; box_empty(rb);
    for (const Ref& r : refs) box_grow(rb, r.lo, r.hi);
    B.min_overlap = box_area(rb) * p.split_alpha;   // m_minOverlap (SplitBVHBuilder.cpp:238)
    const uint32_t root = B.alloc_node();
    SbvhBuilder::Task T;
    B.build(root, std::move(refs), 0, T);
    B.merge(T);
    out.root_box = B.node(0).box;
    out.max_depth = B.max_depth.load();
    out.duplicates = B.duplicates.load();
    auto at = [&B](uint32_t i) -> const BNode& { return B.node(i); };
    Emitter<decltype(at)> E{at, B.leaf_refs, out, false};
    out.nodes.reserve(B.node_count.load() / 2 + 1);
    E.run(0);
}

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
    auto at = [&B](uint32_t i) -> const BNode& { return B.nodes[i]; };
    Emitter<decltype(at)> E{at, B.refs, out, p.leaf_size_one};
    out.nodes.reserve(B.nodes.size() / 2 + 1);
    E.run(~(int32_t)B.refs[0].id);
}

}  // namespace ctl

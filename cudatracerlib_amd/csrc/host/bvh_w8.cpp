// bvh_w8.cpp — see bvh_w8.h.
#include "bvh_w8.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace ctl {
namespace {

constexpr int32_t kSent = 0x76543210;
constexpr int K = 8;

inline bool inner(int32_t v) { return v >= 0 && v != kSent; }

struct Box {
    float lo[3], hi[3];
};
struct Kid {
    Box b;
    int32_t v;   // binary child value: >= 0 inner node float4 offset, < 0 ~leaf entry, kSent none
};

void kids_of(const ctl_bvh_node& n, Kid& a, Kid& b) {
    a.b.lo[0] = n.v[0]; a.b.hi[0] = n.v[1]; a.b.lo[1] = n.v[2]; a.b.hi[1] = n.v[3]; a.b.lo[2] = n.v[8]; a.b.hi[2] = n.v[9];
    b.b.lo[0] = n.v[4]; b.b.hi[0] = n.v[5]; b.b.lo[1] = n.v[6]; b.b.hi[1] = n.v[7]; b.b.lo[2] = n.v[10]; b.b.hi[2] = n.v[11];
    std::memcpy(&a.v, &n.v[12], 4);
    std::memcpy(&b.v, &n.v[13], 4);
}

float area(const Box& b) {
    const float ax = b.hi[0] - b.lo[0], ay = b.hi[1] - b.lo[1], az = b.hi[2] - b.lo[2];
    return 2.0f * (ax * ay + ax * az + ay * az);
}

struct Builder {
    const ctl_bvh_node* nodes;
    size_t n_nodes;
    const ctl_woop_tri* woop;
    const ctl_tri_index* idx;
    size_t n_idx;
    W8Tree& out;
    // dynamic program (bvh_wide.cpp, eight slots): g(x, k) for k = 1..8
    std::vector<float> g;
    std::vector<uint8_t> choice;   // per (x, k): 0 = x its own node, j = left child gets j slots
    std::vector<uint8_t> fsplit;   // per x: the j of f(x)

    const ctl_bvh_node& node_of(int32_t v) const {
        const size_t i = (size_t)v / 4;
        if ((v & 3) != 0 || i >= n_nodes) throw std::runtime_error("W8: bad child offset");
        return nodes[i];
    }
    float G(const Kid& c, int k) const { return inner(c.v) ? g[(size_t)c.v / 4 * K + (k - 1)] : 0.0f; }

    void plan(int32_t root) {
        g.assign(n_nodes * K, 0.0f);
        choice.assign(n_nodes * K, 0);
        fsplit.assign(n_nodes, 1);
        std::vector<std::pair<int32_t, bool>> st;
        st.push_back({root, false});
        size_t visits = 0;
        while (!st.empty()) {
            auto [v, done] = st.back();
            st.pop_back();
            Kid a, b;
            kids_of(node_of(v), a, b);
            if (!done) {
                if (++visits > n_nodes) throw std::runtime_error("W8: a node is reached twice");
                st.push_back({v, true});
                if (inner(a.v)) st.push_back({a.v, false});
                if (inner(b.v)) st.push_back({b.v, false});
                continue;
            }
            const size_t x = (size_t)v / 4;
            float best = std::numeric_limits<float>::infinity();
            int bj = 1;
            for (int j = 1; j < K; j++) {
                const float c = G(a, j) + G(b, K - j);
                if (c < best) { best = c; bj = j; }
            }
            fsplit[x] = (uint8_t)bj;
            Box u;
            for (int i = 0; i < 3; i++) {
                u.lo[i] = std::min(a.b.lo[i], b.b.lo[i]);
                u.hi[i] = std::max(a.b.hi[i], b.b.hi[i]);
            }
            const Box& box = b.v == kSent ? a.b : (a.v == kSent ? b.b : u);
            const float f = area(box) + best;
            g[K * x] = f;
            choice[K * x] = 0;
            for (int k = 2; k <= K; k++) {
                float bk = f;
                int ck = 0;
                for (int j = 1; j < k; j++) {
                    const float c = G(a, j) + G(b, k - j);
                    if (c < bk) { bk = c; ck = j; }
                }
                g[K * x + k - 1] = bk;
                choice[K * x + k - 1] = (uint8_t)ck;
            }
        }
    }

    void expand(const Kid& x, int k, std::vector<Kid>& o) const {
        const int ck = inner(x.v) ? choice[(size_t)x.v / 4 * K + (k - 1)] : 0;
        if (ck == 0) {
            if (x.v != kSent) o.push_back(x);   // a sentinel sibling takes no slot
            return;
        }
        Kid a, b;
        kids_of(node_of(x.v), a, b);
        expand(a, ck, o);
        expand(b, k - ck, o);
    }

    // Slot assignment by octant: the child with the smallest projection of its
    // centre (relative to the node's) on octant s's direction (the one a ray of
    // that octant reaches first) goes to slot s; greedy over all (child, slot)
    // costs, cheapest first.
    void assign_slots(const std::vector<Kid>& ks, int slot_of[K]) const {
        float pc[3] = {0, 0, 0};
        for (const Kid& c : ks)
            for (int a = 0; a < 3; a++) pc[a] += 0.5f * (c.b.lo[a] + c.b.hi[a]);
        for (int a = 0; a < 3; a++) pc[a] /= (float)ks.size();
        struct C { float cost; int kid, slot; };
        std::vector<C> cs;
        for (int i = 0; i < (int)ks.size(); i++)
            for (int s = 0; s < K; s++) {
                float d = 0.0f;
                for (int a = 0; a < 3; a++) {
                    const float c = 0.5f * (ks[i].b.lo[a] + ks[i].b.hi[a]) - pc[a];
                    d += ((s >> a) & 1) ? -c : c;
                }
                cs.push_back({d, i, s});
            }
        std::stable_sort(cs.begin(), cs.end(), [](const C& x, const C& y) { return x.cost < y.cost; });
        bool kid_done[K] = {}, slot_used[K] = {};
        for (int i = 0; i < K; i++) slot_of[i] = -1;
        for (const C& c : cs) {
            if (kid_done[c.kid] || slot_used[c.slot]) continue;
            kid_done[c.kid] = slot_used[c.slot] = true;
            slot_of[c.kid] = c.slot;
        }
    }

    // Grid of one axis: origin p, step 2^E (E + 127 stored) with p + 255 * 2^E >=
    // hi_max; bounds rounded outward in exact (long double) arithmetic.
    static bool grid(float lo_min, float hi_max, int& E) {
        if (!std::isfinite(lo_min) || !std::isfinite(hi_max) || !(lo_min <= hi_max)) return false;
        const long double ext = (long double)hi_max - (long double)lo_min;
        const float mag = std::max(std::fabs(lo_min), std::fabs(hi_max));
        int ep = 0;
        (void)std::frexp(mag, &ep);            // mag < 2^ep
        // never below 2^(ep - 40) (p + q s stays exact in long double) nor 2^-64
        // (s * idir stays a normal float)
        E = std::max(-64, ep - 40);
        while ((long double)255.0 * std::ldexp(1.0L, E) < ext) E++;
        return E <= 100;
    }
    static void quant(float p, int E, float lo, float hi, uint8_t& ql, uint8_t& qh) {
        const long double s = std::ldexp(1.0L, E);
        long double gl = std::floor(((long double)lo - p) / s), gh = std::ceil(((long double)hi - p) / s);
        gl = std::max((long double)0, std::min((long double)255, gl));
        gh = std::max((long double)0, std::min((long double)255, gh));
        int a = (int)gl, b = (int)gh;
        while (a > 0 && (long double)p + a * s > (long double)lo) a--;
        while (b < 255 && (long double)p + b * s < (long double)hi) b++;
        if ((long double)p + a * s > (long double)lo || (long double)p + b * s < (long double)hi)
            throw std::runtime_error("W8: bound outside the node grid");
        ql = (uint8_t)a;
        qh = (uint8_t)b;
    }

    void fill(W8Node& w, const std::vector<Kid>& ks, const int slot_of[K]) {
        Box u = ks[0].b;
        for (const Kid& c : ks)
            for (int a = 0; a < 3; a++) {
                u.lo[a] = std::min(u.lo[a], c.b.lo[a]);
                u.hi[a] = std::max(u.hi[a], c.b.hi[a]);
            }
        int E[3];
        for (int a = 0; a < 3; a++)
            if (!grid(u.lo[a], u.hi[a], E[a])) throw std::runtime_error("W8: box not quantizable");
        w.px = u.lo[0]; w.py = u.lo[1]; w.pz = u.lo[2];
        w.ex = (uint8_t)(E[0] + 127); w.ey = (uint8_t)(E[1] + 127); w.ez = (uint8_t)(E[2] + 127);
        for (int s = 0; s < K; s++) {
            w.qlo_x[s] = w.qlo_y[s] = w.qlo_z[s] = 255;
            w.qhi_x[s] = w.qhi_y[s] = w.qhi_z[s] = 0;
            w.meta[s] = 0;
        }
        for (size_t i = 0; i < ks.size(); i++) {
            const int s = slot_of[i];
            const float p[3] = {w.px, w.py, w.pz};
            uint8_t* lo[3] = {w.qlo_x, w.qlo_y, w.qlo_z};
            uint8_t* hi[3] = {w.qhi_x, w.qhi_y, w.qhi_z};
            for (int a = 0; a < 3; a++) quant(p[a], E[a], ks[i].b.lo[a], ks[i].b.hi[a], lo[a][s], hi[a][s]);
        }
    }

    // a leaf child's entries, copied to the relaid arrays; returns their count
    uint32_t copy_leaf(int32_t v) {
        const uint32_t first = (uint32_t)~v;
        uint32_t cnt = 0;
        for (size_t e = first;; e++) {
            if (e >= n_idx) throw std::runtime_error("W8: leaf runs past the entries");
            out.woop.push_back(woop[e]);
            out.idx.push_back(idx[e]);
            if (++cnt > kW8MaxLeaf) throw std::runtime_error("W8: a leaf holds more than 3 entries");
            if (idx[e] & 1u) break;
        }
        return cnt;
    }

    void emit(int32_t root) {
        struct Work { int32_t v; uint32_t at; int depth; };
        std::vector<Work> todo;
        out.nodes.assign(1, W8Node{});
        todo.push_back({root, 0, 1});
        int deepest = 1;
        while (!todo.empty()) {
            const Work wk = todo.back();
            todo.pop_back();
            Kid a, b;
            kids_of(node_of(wk.v), a, b);
            std::vector<Kid> ks;
            const int j = fsplit[(size_t)wk.v / 4];
            expand(a, j, ks);
            expand(b, K - j, ks);
            if (ks.empty()) throw std::runtime_error("W8: a node without children");
            int slot_of[K];
            assign_slots(ks, slot_of);
            W8Node w{};
            fill(w, ks, slot_of);
            int max_inner = -1;
            for (size_t i = 0; i < ks.size(); i++)
                if (inner(ks[i].v)) max_inner = std::max(max_inner, slot_of[i]);
            w.child_base = 0;
            if (max_inner >= 0) {
                w.child_base = (uint32_t)out.nodes.size();
                if (out.nodes.size() + (size_t)max_inner + 1 >= kW8MaxNodes) throw std::runtime_error("W8: 2^24 nodes");
                out.nodes.resize(out.nodes.size() + (size_t)max_inner + 1, W8Node{});
            }
            // leaf entries of this node, slot order
            w.leaf_base = (uint32_t)out.woop.size();
            w.imask = 0;
            for (int s = 0; s < K; s++) {
                for (size_t i = 0; i < ks.size(); i++) {
                    if (slot_of[i] != s) continue;
                    if (inner(ks[i].v)) {
                        w.imask |= (uint8_t)(1u << s);
                        todo.push_back({ks[i].v, w.child_base + (uint32_t)s, wk.depth + 1});
                    } else {
                        const uint32_t off = (uint32_t)out.woop.size() - w.leaf_base;
                        const uint32_t cnt = copy_leaf(ks[i].v);
                        if (off + cnt > 24) throw std::runtime_error("W8: more than 24 leaf entries in a node");
                        w.meta[s] = (uint8_t)((((1u << cnt) - 1u) << 5) | off);
                    }
                }
            }
            // the group stack holds at most one group per level above the current node
            deepest = std::max(deepest, wk.depth);
            out.nodes[wk.at] = w;
        }
        out.stack_bound = deepest + 1;
    }
};

}  // namespace

bool build_w8(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, const ctl_woop_tri* woop,
              const ctl_tri_index* idx, size_t n_idx, W8Tree& out, std::string* why) {
    out = W8Tree{};
    try {
        if (!inner(root_value) || n_nodes == 0) throw std::runtime_error("W8: the root is not an inner node");
        Builder b{nodes, n_nodes, woop, idx, n_idx, out, {}, {}, {}};
        b.plan(root_value);
        b.emit(root_value);
    } catch (const std::exception& e) {
        if (why) *why = e.what();
        out = W8Tree{};
        return false;
    }
    return true;
}

}  // namespace ctl

namespace ctl { void set_host_error(const std::string& s); }

// The 8-wide tree ctl_scene_upload builds for a one-mesh scene under
// CTL_SCENE_WIDE8 (the CTL_ARRAY_W8_* layouts); sizes with NULL outputs.
extern "C" CTL_API ctl_status ctl_host_w8_tree(const ctl_scene_desc* d, void* nodes_out, uint64_t nodes_cap,
                                               uint64_t* n_nodes, void* woop_out, uint32_t* idx_out,
                                               uint64_t entries_cap, uint64_t* n_entries) {
    if (!d || !n_nodes || !n_entries) { ctl::set_host_error("host_w8_tree: null argument"); return CTL_ERR_INVALID; }
    if (d->n_nodes == 0 || d->scene_start_node >= 0 || d->n_anim_meshes != 0) {
        ctl::set_host_error("host_w8_tree: not a one-mesh scene without animated meshes");
        return CTL_ERR_INVALID;
    }
    const uint32_t node = ~(uint32_t)d->scene_start_node;
    if (node >= d->n_nodes || d->nodes[node].mesh_index >= d->n_meshes) {
        ctl::set_host_error("host_w8_tree: start node out of range");
        return CTL_ERR_INVALID;
    }
    const ctl_kernel_mesh& M = d->meshes[d->nodes[node].mesh_index];
    if (M.bvh_node_offset / 4 >= d->n_bvh_nodes || M.bvh_indices_offset > d->n_tri_indices ||
        (uint64_t)M.bvh_triangle_offset / 3 > d->n_woop_tris) {
        ctl::set_host_error("host_w8_tree: mesh offsets out of range");
        return CTL_ERR_INVALID;
    }
    ctl::W8Tree t;
    std::string why;
    const size_t first = M.bvh_node_offset / 4;
    const uint64_t e0 = M.bvh_indices_offset, w0 = M.bvh_triangle_offset / 3;
    if (!ctl::build_w8(d->bvh_nodes + first, d->n_bvh_nodes - first, 0, d->woop_tris + w0, d->tri_indices + e0,
                       (size_t)std::min<uint64_t>(d->n_tri_indices - e0, d->n_woop_tris - w0), t, &why)) {
        ctl::set_host_error("host_w8_tree: " + why);
        return CTL_ERR_INVALID;
    }
    *n_nodes = t.nodes.size();
    *n_entries = t.woop.size();
    if ((nodes_out && nodes_cap < t.nodes.size()) || ((woop_out || idx_out) && entries_cap < t.woop.size())) {
        ctl::set_host_error("host_w8_tree: output capacity too small");
        return CTL_ERR_INVALID;
    }
    if (nodes_out) std::memcpy(nodes_out, t.nodes.data(), t.nodes.size() * sizeof(ctl::W8Node));
    if (woop_out && !t.woop.empty()) std::memcpy(woop_out, t.woop.data(), t.woop.size() * sizeof(ctl_woop_tri));
    if (idx_out && !t.idx.empty()) std::memcpy(idx_out, t.idx.data(), t.idx.size() * sizeof(uint32_t));
    return CTL_OK;
}

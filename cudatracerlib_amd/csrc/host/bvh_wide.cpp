// bvh_wide.cpp — see bvh_wide.h.
#include "bvh_wide.h"
#include "../ctl_qnode.h"

#include <algorithm>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>

namespace ctl {
namespace {

const int32_t kSentinel = 0x76543210;

struct Kid {
    float lo[3], hi[3];
    int32_t v;
    uint32_t src;   // binary node index << 1 | child slot holding this box
};

inline bool is_inner(int32_t v) { return v >= 0 && v != kSentinel; }

inline float kid_area(const Kid& k) {
    float ax = k.hi[0] - k.lo[0], ay = k.hi[1] - k.lo[1], az = k.hi[2] - k.lo[2];
    return 2.0f * (ax * ay + ax * az + ay * az);
}

// Children of binary node `idx` with the boxes stored in it (BVHNodeData::getLeft/getRight).
void binary_kids(const ctl_bvh_node& n, uint32_t idx, Kid& a, Kid& b) {
    a.src = idx << 1;
    b.src = (idx << 1) | 1u;
    a.lo[0] = n.v[0]; a.hi[0] = n.v[1]; a.lo[1] = n.v[2]; a.hi[1] = n.v[3]; a.lo[2] = n.v[8]; a.hi[2] = n.v[9];
    b.lo[0] = n.v[4]; b.hi[0] = n.v[5]; b.lo[1] = n.v[6]; b.hi[1] = n.v[7]; b.lo[2] = n.v[10]; b.hi[2] = n.v[11];
    std::memcpy(&a.v, &n.v[12], 4);
    std::memcpy(&b.v, &n.v[13], 4);
}

struct Collapser {
    const ctl_bvh_node* nodes;
    size_t n_nodes;
    std::vector<WideNode>& out;
    size_t base;
    std::vector<uint32_t>* src;
    const ctl_tri_index* idx;   // counted leaves (mesh trees), or null
    size_t n_idx;

    // a leaf value as the wide node stores it (bvh_wide.h: wide_leaf_code)
    int32_t leaf_value(int32_t v) const {
        if (!idx || v == kSentinel || v >= 0) return v;
        const uint32_t first = (uint32_t)~v;
        if (first >= kWideLeafMaxEntry || first >= n_idx) throw std::runtime_error("wide BVH: leaf entry out of range");
        uint32_t cnt = 1;
        for (size_t e = first; e < n_idx && !(idx[e] & 1u) && cnt < 8; e++) cnt++;
        if (cnt < 8 && first + cnt > n_idx) throw std::runtime_error("wide BVH: leaf runs past the entries");
        return wide_leaf_code(first, cnt);
    }

    const ctl_bvh_node& node_of(int32_t v) const {
        size_t i = (size_t)v / 4;
        if ((v & 3) != 0 || i >= n_nodes) throw std::runtime_error("wide BVH: bad child offset");
        return nodes[i];
    }

    // SAH-optimal collapse (the wide-BVH dynamic program of Ylitie, Karras and
    // Laine, HPG 2017, over fixed leaves): every binary inner node is either a
    // wide node of its own or opened into its parent's slots.  With the leaves
    // fixed their intersection cost is the same in every collapse, so the cost
    // to minimise is the summed surface area of the wide nodes (a wide node is
    // visited when a ray hits its box).  Per binary node x and slot budget k:
    //   g(x, 1) = f(x) = A(x) + min_j g(l, j) + g(r, 4 - j)   (x its own node)
    //   g(x, k) = min(g(x, 1), min_j g(l, j) + g(r, k - j))    (x opened)
    // and g = 0 for leaves.  choice[] keeps the argmin per (x, k).
    std::vector<float> g;               // 4 per binary node: g(x, 1..4)
    std::vector<uint8_t> choice;        // 4 per node: 0 = own node, j = left gets j slots
    std::vector<uint8_t> fsplit;        // per node: the j of f(x)

    void plan(int32_t root) {
        g.assign(n_nodes * 4, 0.0f);
        choice.assign(n_nodes * 4, 0);
        fsplit.assign(n_nodes, 1);
        std::vector<std::pair<int32_t, bool>> st;   // post order without recursion
        st.push_back({root, false});
        size_t visits = 0;
        while (!st.empty()) {
            auto [v, done] = st.back();
            st.pop_back();
            const ctl_bvh_node& n = node_of(v);
            Kid a, b;
            binary_kids(n, (uint32_t)v >> 2, a, b);
            if (!done) {
                if (++visits > n_nodes) throw std::runtime_error("wide BVH: a node is reached twice");
                st.push_back({v, true});
                if (is_inner(a.v)) st.push_back({a.v, false});
                if (is_inner(b.v)) st.push_back({b.v, false});
                continue;
            }
            const size_t x = (size_t)v / 4;
            auto G = [&](const Kid& c, int k) { return is_inner(c.v) ? g[(size_t)c.v / 4 * 4 + (k - 1)] : 0.0f; };
            // the node's own box: the union of its children's (the parent's slot holds it)
            float best = std::numeric_limits<float>::infinity();
            int bj = 1;
            for (int j = 1; j <= 3; j++) {
                const float c = G(a, j) + G(b, 4 - j);
                if (c < best) { best = c; bj = j; }
            }
            fsplit[x] = (uint8_t)bj;
            Kid u = a;
            for (int i = 0; i < 3; i++) {
                u.lo[i] = std::min(a.lo[i], b.lo[i]);
                u.hi[i] = std::max(a.hi[i], b.hi[i]);
            }
            // a sentinel sibling has no box: the node's box is its one real child's
            const Kid& box = b.v == kSentinel ? a : (a.v == kSentinel ? b : u);
            const float f = kid_area(box) + best;
            g[4 * x] = f;
            choice[4 * x] = 0;
            for (int k = 2; k <= 4; k++) {
                float bk = f;
                int ck = 0;
                for (int j = 1; j < k; j++) {
                    const float c = G(a, j) + G(b, k - j);
                    if (c < bk) { bk = c; ck = j; }
                }
                g[4 * x + k - 1] = bk;
                choice[4 * x + k - 1] = (uint8_t)ck;
            }
        }
    }

    // the slots subtree x fills with a budget of k (x's box taken from its parent)
    void expand(const Kid& x, int k, Kid* out, int& nk) {
        const int ck = is_inner(x.v) ? choice[(size_t)x.v / 4 * 4 + (k - 1)] : 0;
        if (ck == 0) { out[nk++] = x; return; }
        Kid a, b;
        binary_kids(node_of(x.v), (uint32_t)x.v >> 2, a, b);
        expand(a, ck, out, nk);
        expand(b, k - ck, out, nk);
    }

    int32_t emit(int32_t v, int depth) {
        if (depth > 256) throw std::runtime_error("wide BVH: tree too deep");
        Kid k[4];
        int nk = 2;
        binary_kids(node_of(v), (uint32_t)v >> 2, k[0], k[1]);
        {
            const Kid a = k[0], b = k[1];
            const int j = fsplit[(size_t)v / 4];
            nk = 0;
            expand(a, j, k, nk);
            expand(b, 4 - j, k, nk);
        }
        const size_t me = out.size();
        out.push_back(WideNode{});
        if (src) {
            src->resize(out.size() * 4 - 4 * base, 0xffffffffu);
            for (int i = 0; i < nk; i++)
                if (k[i].v != kSentinel) (*src)[4 * (me - base) + i] = k[i].src;
        }
        int32_t child[4];
        for (int i = 0; i < 4; i++) {
            if (i >= nk) { child[i] = kSentinel; continue; }
            child[i] = is_inner(k[i].v) ? emit(k[i].v, depth + 1) : leaf_value(k[i].v);
        }
        WideNode& w = out[me];
        // empty slots and sentinel children (the right child of a single-leaf
        // root): quiet-NaN boxes, which fail every slab test (traverse.h)
        const float e = std::numeric_limits<float>::quiet_NaN();
        for (int i = 0; i < 4; i++) {
            const bool used = i < nk && k[i].v != kSentinel;
            w.lo_x[i] = used ? k[i].lo[0] : e; w.hi_x[i] = used ? k[i].hi[0] : e;
            w.lo_y[i] = used ? k[i].lo[1] : e; w.hi_y[i] = used ? k[i].hi[1] : e;
            w.lo_z[i] = used ? k[i].lo[2] : e; w.hi_z[i] = used ? k[i].hi[2] : e;
            w.child[i] = child[i];
            w.pad[i] = 0;
        }
        return (int32_t)(me - base);
    }
};

}  // namespace

int32_t collapse_wide(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, std::vector<WideNode>& out,
                      std::vector<uint32_t>* src, const ctl_tri_index* idx, size_t n_idx) {
    if (!is_inner(root_value) || n_nodes == 0) throw std::runtime_error("wide BVH: root is not an inner node");
    if (src) src->clear();
    Collapser c{nodes, n_nodes, out, out.size(), src, idx, n_idx, {}, {}, {}};
    c.plan(root_value);
    return c.emit(root_value, 0);
}

namespace {
// DFS over (child value, stack entries below the node); `kids` yields a node's
// children, `inner` tells which of them are nodes to descend into.
template <class KIDS>
int stack_bound(size_t n_nodes, int32_t root, int cap, KIDS kids) {
    std::vector<std::pair<int32_t, int>> todo;
    todo.push_back({root, 1});   // the bottom sentinel
    size_t visits = 0;
    int best = 1;
    while (!todo.empty()) {
        const auto [v, below] = todo.back();
        todo.pop_back();
        if (++visits > n_nodes) throw std::runtime_error("BVH: a node is reached twice (not a tree)");
        int32_t c[4];
        const int nk = kids(v, c);
        int used = 0;
        for (int i = 0; i < nk; i++) used += c[i] != kSentinel;
        const int here = below + (used > 0 ? used - 1 : 0);
        if (here > best) best = here;
        if (best > cap) return cap + 1;
        for (int i = 0; i < nk; i++)
            if (is_inner(c[i])) todo.push_back({c[i], here});
    }
    return best;
}
}  // namespace

int binary_stack_bound(const ctl_bvh_node* nodes, size_t n_nodes, int32_t root_value, int cap) {
    if (!is_inner(root_value)) return 1;
    return stack_bound(n_nodes, root_value, cap, [&](int32_t v, int32_t c[4]) {
        const size_t i = (size_t)v / 4;
        if ((v & 3) != 0 || i >= n_nodes) throw std::runtime_error("BVH: child offset out of range");
        std::memcpy(&c[0], &nodes[i].v[12], 4);
        std::memcpy(&c[1], &nodes[i].v[13], 4);
        return 2;
    });
}

int wide_stack_bound(const WideNode* nodes, size_t n_nodes, int32_t root, int cap) {
    if (!is_inner(root)) return 1;
    return stack_bound(n_nodes, root, cap, [&](int32_t v, int32_t c[4]) {
        if ((size_t)v >= n_nodes) throw std::runtime_error("wide BVH: child index out of range");
        for (int k = 0; k < 4; k++) c[k] = nodes[v].child[k];
        return 4;
    });
}

}  // namespace ctl

namespace ctl { void set_host_error(const std::string& s); }

extern "C" CTL_API ctl_status ctl_host_bvh_stack_bound(const ctl_bvh_node* nodes, uint64_t n_nodes,
                                                       int32_t root_value, int32_t out[2]) {
    if (!nodes || !out || n_nodes == 0) { ctl::set_host_error("bvh_stack_bound: no nodes"); return CTL_ERR_INVALID; }
    try {
        out[0] = ctl::binary_stack_bound(nodes, n_nodes, root_value, 1024);
        std::vector<ctl::WideNode> w;
        const int32_t root = ctl::collapse_wide(nodes, n_nodes, root_value, w);
        out[1] = ctl::wide_stack_bound(w.data(), w.size(), root, 1024);
    } catch (const std::exception& e) {
        ctl::set_host_error(std::string("bvh_stack_bound: ") + e.what());
        return CTL_ERR_INVALID;
    }
    return CTL_OK;
}


// The 4-wide trees ctl_scene_upload builds (device/scene_dev.hip commit): one
// counted-leaf tree per mesh, then the instance tree.
extern "C" CTL_API ctl_status ctl_host_wide_trees(const ctl_scene_desc* d, void* mesh_out, uint64_t mesh_capacity,
                                                  uint64_t* n_mesh_nodes, uint32_t* wbase_out, void* scene_out,
                                                  uint64_t scene_capacity, uint64_t* n_scene_nodes) {
    if (!d || !n_mesh_nodes || !n_scene_nodes) { ctl::set_host_error("host_wide_trees: null argument"); return CTL_ERR_INVALID; }
    try {
        std::vector<ctl::WideNode> wn, sw;
        std::vector<uint32_t> wb(d->n_meshes, 0);
        for (uint32_t m = 0; m < d->n_meshes && d->n_bvh_nodes > 0; m++) {
            const size_t first = d->meshes[m].bvh_node_offset / 4;
            if (first >= d->n_bvh_nodes) throw std::runtime_error("mesh BVH offset out of range");
            const uint64_t e0 = d->meshes[m].bvh_indices_offset;
            if (e0 > d->n_tri_indices) throw std::runtime_error("mesh entry offset out of range");
            wb[m] = (uint32_t)wn.size();
            ctl::collapse_wide(d->bvh_nodes + first, d->n_bvh_nodes - first, 0, wn, nullptr, d->tri_indices + e0,
                               (size_t)(d->n_tri_indices - e0));
        }
        if (d->n_bvh_nodes > 0 && d->n_nodes > 0 && d->scene_start_node >= 0)
            ctl::collapse_wide(d->scene_bvh_nodes, d->n_scene_bvh_nodes, d->scene_start_node, sw);
        // CTL_SCENE_WIDE_QUANT: the boxes the quantized nodes decode to (what the
        // device's slab test sees; empty slots NaN), when every node quantizes
        if ((d->flags & CTL_SCENE_WIDE_QUANT) && d->n_anim_meshes == 0) {
            std::vector<ctl::WideNode> dq[2] = {wn, sw};
            bool ok = true;
            for (auto& tree : dq)
                for (ctl::WideNode& w : tree) {
                    const float lo[3][4] = {{w.lo_x[0], w.lo_x[1], w.lo_x[2], w.lo_x[3]},
                                            {w.lo_y[0], w.lo_y[1], w.lo_y[2], w.lo_y[3]},
                                            {w.lo_z[0], w.lo_z[1], w.lo_z[2], w.lo_z[3]}};
                    const float hi[3][4] = {{w.hi_x[0], w.hi_x[1], w.hi_x[2], w.hi_x[3]},
                                            {w.hi_y[0], w.hi_y[1], w.hi_y[2], w.hi_y[3]},
                                            {w.hi_z[0], w.hi_z[1], w.hi_z[2], w.hi_z[3]}};
                    ctl::QWideNode q;
                    if (!ctl::quantize_wide(lo, hi, w.child, q)) { ok = false; break; }
                    const float nan = std::numeric_limits<float>::quiet_NaN();
                    for (int i = 0; i < 4; i++) {
                        const bool used = w.child[i] != 0x76543210;
                        auto b = [&](uint32_t word) { return (word >> (8 * i)) & 0xffu; };
                        w.lo_x[i] = used ? ctl::qdecode(q.px, b(q.lo_x), q.sx) : nan;
                        w.hi_x[i] = used ? ctl::qdecode(q.px, b(q.hi_x), q.sx) : nan;
                        w.lo_y[i] = used ? ctl::qdecode(q.py, b(q.lo_y), q.sy) : nan;
                        w.hi_y[i] = used ? ctl::qdecode(q.py, b(q.hi_y), q.sy) : nan;
                        w.lo_z[i] = used ? ctl::qdecode(q.pz, b(q.lo_z), q.sz) : nan;
                        w.hi_z[i] = used ? ctl::qdecode(q.pz, b(q.hi_z), q.sz) : nan;
                    }
                }
            if (ok) { wn = dq[0]; sw = dq[1]; }
        }
        *n_mesh_nodes = wn.size();
        *n_scene_nodes = sw.size();
        if ((mesh_out && mesh_capacity < wn.size()) || (scene_out && scene_capacity < sw.size()))
            throw std::runtime_error("output capacity too small");
        if (mesh_out && !wn.empty()) std::memcpy(mesh_out, wn.data(), wn.size() * sizeof(ctl::WideNode));
        if (scene_out && !sw.empty()) std::memcpy(scene_out, sw.data(), sw.size() * sizeof(ctl::WideNode));
        if (wbase_out && !wb.empty()) std::memcpy(wbase_out, wb.data(), wb.size() * sizeof(uint32_t));
    } catch (const std::exception& e) {
        ctl::set_host_error(std::string("host_wide_trees: ") + e.what());
        return CTL_ERR_INVALID;
    }
    return CTL_OK;
}

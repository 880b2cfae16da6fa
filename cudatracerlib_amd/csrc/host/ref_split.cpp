// ref_split.cpp — see ref_split.h.
#include "ref_split.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <thread>

namespace ctl {
namespace {

struct P3 { float v[3]; };

inline double box_area(const Box& b) {
    double x = (double)b.hi[0] - b.lo[0], y = (double)b.hi[1] - b.lo[1], z = (double)b.hi[2] - b.lo[2];
    return 2.0 * (x * y + x * z + y * z);
}

// Clip a convex polygon (at most 9 vertices after 6 planes on a triangle) to a box.
int clip_poly(P3* poly, int n, const Box& b) {
    P3 tmp[16];
    for (int ax = 0; ax < 3; ax++) {
        for (int side = 0; side < 2; side++) {
            const float lim = side == 0 ? b.lo[ax] : b.hi[ax];
            int m = 0;
            for (int i = 0; i < n; i++) {
                const P3& a = poly[i];
                const P3& c = poly[(i + 1) % n];
                const float av = a.v[ax], cv = c.v[ax];
                const bool ain = side == 0 ? av >= lim : av <= lim;
                const bool cin = side == 0 ? cv >= lim : cv <= lim;
                if (ain) tmp[m++] = a;
                if (ain != cin) {
                    const float t = (lim - av) / (cv - av);
                    P3 q;
                    for (int k = 0; k < 3; k++) q.v[k] = a.v[k] + t * (c.v[k] - a.v[k]);
                    q.v[ax] = lim;
                    tmp[m++] = q;
                }
            }
            n = m;
            for (int i = 0; i < n; i++) poly[i] = tmp[i];
            if (n == 0) return 0;
        }
    }
    return n;
}

struct Splitter {
    const float* V;
    double thr;
    uint32_t max_depth;
    std::vector<Box>* ob;
    std::vector<uint32_t>* oid;

    void piece(uint32_t t, const Box& cell, uint32_t depth) {
        P3 poly[16];
        for (int c = 0; c < 3; c++)
            for (int k = 0; k < 3; k++) poly[c].v[k] = V[9 * (size_t)t + 3 * c + k];
        const int n = clip_poly(poly, 3, cell);
        if (n == 0) return;
        Box tb;
        for (int k = 0; k < 3; k++) { tb.lo[k] = FLT_MAX; tb.hi[k] = -FLT_MAX; }
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) {
                tb.lo[k] = std::min(tb.lo[k], poly[i].v[k]);
                tb.hi[k] = std::max(tb.hi[k], poly[i].v[k]);
            }
        for (int k = 0; k < 3; k++) {   // one ulp of slack against clipping round-off, within the cell
            tb.lo[k] = std::max(cell.lo[k], std::nextafter(tb.lo[k], -FLT_MAX));
            tb.hi[k] = std::min(cell.hi[k], std::nextafter(tb.hi[k], FLT_MAX));
        }
        if (depth >= max_depth || box_area(tb) <= thr) {
            ob->push_back(tb);
            oid->push_back(t);
            return;
        }
        int ax = 0;
        float w = -1.0f;
        for (int k = 0; k < 3; k++)
            if (tb.hi[k] - tb.lo[k] > w) { w = tb.hi[k] - tb.lo[k]; ax = k; }
        const float mid = 0.5f * (tb.lo[ax] + tb.hi[ax]);
        Box l = tb, r = tb;
        l.hi[ax] = mid;
        r.lo[ax] = mid;
        piece(t, l, depth + 1);
        piece(t, r, depth + 1);
    }
};

}  // namespace

void split_refs(const float* V, const Box* boxes, uint64_t n, const RefSplitParams& p, std::vector<Box>& out_boxes,
                std::vector<uint32_t>& out_ids) {
    out_boxes.clear();
    out_ids.clear();
    double mean = 0.0;
    for (uint64_t t = 0; t < n; t++) mean += box_area(boxes[t]);
    mean = n ? mean / (double)n : 0.0;
    const double thr = (double)p.alpha * mean;
    uint32_t nt = p.threads ? p.threads : std::max(1u, std::thread::hardware_concurrency());
    if (n < 65536) nt = 1;
    std::vector<std::vector<Box>> pb(nt);
    std::vector<std::vector<uint32_t>> pid(nt);
    const uint64_t chunk = (n + nt - 1) / nt;
    auto work = [&](uint32_t w) {
        const uint64_t b = std::min(n, (uint64_t)w * chunk), e = std::min(n, b + chunk);
        Splitter S{V, thr, p.max_depth, &pb[w], &pid[w]};
        pb[w].reserve((e - b) + (e - b) / 4);
        pid[w].reserve((e - b) + (e - b) / 4);
        for (uint64_t t = b; t < e; t++) {
            if (p.alpha <= 0.0f || p.max_depth == 0 || box_area(boxes[t]) <= thr) {
                pb[w].push_back(boxes[t]);
                pid[w].push_back((uint32_t)t);
            } else {
                S.piece((uint32_t)t, boxes[t], 0);
            }
        }
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> ts;
        for (uint32_t w = 0; w < nt; w++) ts.emplace_back(work, w);
        for (auto& t : ts) t.join();
    }
    size_t total = 0;
    for (auto& v : pb) total += v.size();
    out_boxes.reserve(total);
    out_ids.reserve(total);
    for (uint32_t w = 0; w < nt; w++) {
        out_boxes.insert(out_boxes.end(), pb[w].begin(), pb[w].end());
        out_ids.insert(out_ids.end(), pid[w].begin(), pid[w].end());
    }
}

}  // namespace ctl

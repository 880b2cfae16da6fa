// scene_gen.cpp — deterministic synthetic workloads of BASELINE.json
// (SplitMix64, seed 0x5EED; SURVEY.md §8d "Synthetic inputs"):
//   C1  Cornell box, 32 triangles, one Node per shape, one quad DiffuseLight
//   C2  ~100k triangles in one mesh: height-field ground grid + boxes + icosahedra, 1 quad light
//   C3  ~10M triangles in one mesh "San-Miguel-scale": terrain 2M + clustered foliage 6M
//       + walls/columns 2M, 2 quad lights, camera inside the clusters
// No degenerate triangles are emitted (see SURVEY.md §7 on sentinel leaves).
#include <cmath>
#include <cstring>
#include <vector>
#include "scene.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double range(double a, double b) { return a + (b - a) * uni(); }
    double normal() {
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

struct V { double x, y, z; };
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V operator*(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dotv(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V norm(V a) { double l = std::sqrt(dotv(a, a)); return a * (1.0 / l); }

struct MeshB {
    std::vector<float> v;
    std::vector<uint32_t> idx;
    std::vector<uint8_t> mat;
    uint32_t vert(V p) {
        v.push_back((float)p.x); v.push_back((float)p.y); v.push_back((float)p.z);
        return (uint32_t)(v.size() / 3 - 1);
    }
    void tri(uint32_t a, uint32_t b, uint32_t c, uint8_t m) {
        idx.push_back(a); idx.push_back(b); idx.push_back(c); mat.push_back(m);
    }
    // quad p0 p1 p2 p3 (counter-clockwise seen from the side its normal points to)
    void quad(V p0, V p1, V p2, V p3, uint8_t m) {
        uint32_t a = vert(p0), b = vert(p1), c = vert(p2), d = vert(p3);
        tri(a, b, c, m); tri(a, c, d, m);
    }
    void box(V c, V h, double yaw, uint8_t m, bool bottom = true) {
        double cs = std::cos(yaw), sn = std::sin(yaw);
        auto P = [&](double sx, double sy, double sz) {
            double x = sx * h.x, z = sz * h.z;
            return V{c.x + cs * x - sn * z, c.y + sy * h.y, c.z + sn * x + cs * z};
        };
        V p000 = P(-1, -1, -1), p100 = P(1, -1, -1), p110 = P(1, 1, -1), p010 = P(-1, 1, -1);
        V p001 = P(-1, -1, 1), p101 = P(1, -1, 1), p111 = P(1, 1, 1), p011 = P(-1, 1, 1);
        quad(p000, p010, p110, p100, m);   // -z
        quad(p101, p111, p011, p001, m);   // +z
        quad(p001, p011, p010, p000, m);   // -x
        quad(p100, p110, p111, p101, m);   // +x
        quad(p010, p011, p111, p110, m);   // +y
        if (bottom) quad(p000, p100, p101, p001, m);   // -y
    }
    void icosa(V c, double r, uint8_t m) {
        const double t = (1.0 + std::sqrt(5.0)) / 2.0;
        V P[12] = {{-1, t, 0}, {1, t, 0}, {-1, -t, 0}, {1, -t, 0}, {0, -1, t}, {0, 1, t},
                   {0, -1, -t}, {0, 1, -t}, {t, 0, -1}, {t, 0, 1}, {-t, 0, -1}, {-t, 0, 1}};
        static const int F[20][3] = {{0, 11, 5}, {0, 5, 1}, {0, 1, 7}, {0, 7, 10}, {0, 10, 11}, {1, 5, 9}, {5, 11, 4},
                                     {11, 10, 2}, {10, 7, 6}, {7, 1, 8}, {3, 9, 4}, {3, 4, 2}, {3, 2, 6}, {3, 6, 8},
                                     {3, 8, 9}, {4, 9, 5}, {2, 4, 11}, {6, 2, 10}, {8, 6, 7}, {9, 8, 1}};
        uint32_t base = (uint32_t)(v.size() / 3);
        for (auto& p : P) vert(c + norm(p) * r);
        for (auto& f : F) tri(base + f[0], base + f[1], base + f[2], m);
    }
    void cylinder(V c, double r, double hgt, int seg, uint8_t m) {
        uint32_t base = (uint32_t)(v.size() / 3);
        for (int i = 0; i < seg; i++) {
            double a = 6.283185307179586 * i / seg;
            vert(V{c.x + r * std::cos(a), c.y, c.z + r * std::sin(a)});
            vert(V{c.x + r * std::cos(a), c.y + hgt, c.z + r * std::sin(a)});
        }
        for (int i = 0; i < seg; i++) {
            uint32_t a0 = base + 2 * i, a1 = a0 + 1, b0 = base + 2 * ((i + 1) % seg), b1 = b0 + 1;
            tri(a0, a1, b1, m); tri(a0, b1, b0, m);
        }
    }
    void grid(double x0, double z0, double size, int n, double (*hf)(double, double), uint8_t m, SplitMix64* rm,
              int nmat) {
        uint32_t base = (uint32_t)(v.size() / 3);
        for (int j = 0; j <= n; j++)
            for (int i = 0; i <= n; i++) {
                double x = x0 + size * i / n, z = z0 + size * j / n;
                vert(V{x, hf(x, z), z});
            }
        for (int j = 0; j < n; j++)
            for (int i = 0; i < n; i++) {
                uint32_t a = base + j * (n + 1) + i, b = a + 1, c = a + (n + 1), d = c + 1;
                uint8_t mm = rm ? (uint8_t)(rm->next() % nmat) : m;
                tri(a, c, d, mm); tri(a, d, b, mm);
            }
    }
};

ctl_material diffuse_mat(float r, float g, float b) {
    ctl_material m{};
    m.bsdf_type = CTL_BSDF_DIFFUSE;
    m.combined_type = CTL_EDIFFUSE_REFLECTION;
    m.two_sided = 1;
    m.node_light_index = 0xffffffffu;
    m.reflectance[0] = r; m.reflectance[1] = g; m.reflectance[2] = b;
    m.texture = 0xffffffffu;
    m.alpha_texture = 0xffffffffu;
    return m;
}

double hf_flat(double, double) { return 0.0; }
double hf_c2(double x, double z) { return 0.6 * std::sin(0.21 * x) * std::cos(0.17 * z) + 0.15 * std::sin(0.9 * x + 0.4 * z); }
double hf_c3(double x, double z) {
    return 2.5 * std::sin(0.031 * x) * std::cos(0.027 * z) + 0.6 * std::sin(0.11 * x + 0.07 * z) +
           0.15 * std::sin(0.53 * x - 0.41 * z);
}

int add_mesh(ctl_host_scene* s, MeshB& M, const std::vector<ctl_material>& mats, const float* uvs = nullptr) {
    return ctl_host_scene_add_mesh(s, M.v.data(), (uint32_t)(M.v.size() / 3), M.idx.data(),
                                   (uint32_t)(M.idx.size() / 3), nullptr, uvs, M.mat.data(), mats.data(),
                                   (uint32_t)mats.size());
}

// C5 textures: 1024^2 RGBA8 procedural images (row 0 = top).
std::vector<uint32_t> tex_checker(uint32_t n) {
    std::vector<uint32_t> img((size_t)n * n);
    for (uint32_t y = 0; y < n; y++)
        for (uint32_t x = 0; x < n; x++) {
            bool c = ((x / 32) + (y / 32)) & 1;
            uint32_t r = c ? 230 : 40, g = c ? 220 : 70, b = c ? 200 : 120;
            img[(size_t)y * n + x] = r | (g << 8) | (b << 16) | (255u << 24);
        }
    return img;
}
std::vector<uint32_t> tex_noise(uint32_t n, SplitMix64& R) {
    // value noise: 4 octaves of bilinearly interpolated lattice values
    std::vector<float> acc((size_t)n * n, 0.0f);
    float amp = 0.5f;
    for (uint32_t cell = 128; cell >= 16; cell /= 2, amp *= 0.5f) {
        uint32_t m = n / cell + 1;
        std::vector<float> lat((size_t)m * m);
        for (auto& v : lat) v = (float)R.range(0.0, 1.0);
        for (uint32_t y = 0; y < n; y++)
            for (uint32_t x = 0; x < n; x++) {
                float fx = (float)x / cell, fy = (float)y / cell;
                uint32_t ix = (uint32_t)fx, iy = (uint32_t)fy;
                float tx = fx - ix, ty = fy - iy;
                float a = lat[iy * m + ix], b = lat[iy * m + ix + 1], c = lat[(iy + 1) * m + ix], d = lat[(iy + 1) * m + ix + 1];
                acc[(size_t)y * n + x] += amp * ((a * (1 - tx) + b * tx) * (1 - ty) + (c * (1 - tx) + d * tx) * ty);
            }
    }
    std::vector<uint32_t> img((size_t)n * n);
    for (size_t i = 0; i < img.size(); i++) {
        float v = std::min(1.0f, std::max(0.0f, acc[i] * 1.1f));
        uint32_t r = (uint32_t)(60 + 150 * v), g = (uint32_t)(90 + 140 * v), b = (uint32_t)(30 + 60 * v);
        img[i] = r | (g << 8) | (b << 16) | (255u << 24);
    }
    return img;
}

ctl_material rough_mat(uint32_t dist, float eta, float alpha) {
    ctl_material m{};
    m.bsdf_type = CTL_BSDF_ROUGHDIELECTRIC;
    m.combined_type = CTL_EGLOSSY_REFLECTION | CTL_EGLOSSY_TRANSMISSION;
    m.two_sided = 0;
    m.node_light_index = 0xffffffffu;
    m.reflectance[0] = m.reflectance[1] = m.reflectance[2] = 1.0f;
    m.texture = 0xffffffffu;
    m.transmittance[0] = m.transmittance[1] = m.transmittance[2] = 1.0f;
    m.distribution = dist;
    m.eta = eta;
    m.inv_eta = 1.0f / eta;   // roughdielectric::Update
    m.alpha_u = m.alpha_v = alpha;
    m.sample_visible = 1;     // getSampleVisible(Beckmann/GGX, true)
    return m;
}

ctl_status gen_cornell(ctl_host_scene* s, uint32_t W, uint32_t H) {
    ctl_material white = diffuse_mat(0.725f, 0.71f, 0.68f), red = diffuse_mat(0.63f, 0.065f, 0.05f),
                 green = diffuse_mat(0.14f, 0.45f, 0.091f), lightm = diffuse_mat(0.78f, 0.78f, 0.78f);
    struct Shape { MeshB m; ctl_material mat; bool light; };
    std::vector<Shape> shapes;
    auto q = [&](V a, V b, V c, V d, ctl_material mt, bool light = false) {
        Shape sh; sh.m.quad(a, b, c, d, 0); sh.mat = mt; sh.light = light; shapes.push_back(sh);
    };
    q({0, 0, 0}, {0, 0, 559.2}, {556, 0, 559.2}, {552.8, 0, 0}, white);                      // floor (+y)
    q({0, 548.8, 0}, {556, 548.8, 0}, {556, 548.8, 559.2}, {0, 548.8, 559.2}, white);        // ceiling (-y)
    q({0, 0, 559.2}, {0, 548.8, 559.2}, {556, 548.8, 559.2}, {549.6, 0, 559.2}, white);      // back (-z)
    q({552.8, 0, 0}, {549.6, 0, 559.2}, {556, 548.8, 559.2}, {556, 548.8, 0}, red);          // left (-x)
    q({0, 0, 0}, {0, 548.8, 0}, {0, 548.8, 559.2}, {0, 0, 559.2}, green);                    // right (+x)
    q({343, 548.7, 227}, {343, 548.7, 332}, {213, 548.7, 332}, {213, 548.7, 227}, lightm, true);   // light (-y)
    {   // short box (no bottom face): 10 triangles
        Shape sh; sh.m.box({185.5, 82.5, 169}, {82.5, 82.5, 82.5}, -0.29, 0, false); sh.mat = white; sh.light = false;
        shapes.push_back(sh);
        Shape tb; tb.m.box({368.5, 165, 351}, {82.5, 165, 82.5}, 0.29, 0, false); tb.mat = white; tb.light = false;
        shapes.push_back(tb);
    }
    for (auto& sh : shapes) {
        std::vector<ctl_material> mats{sh.mat};
        int mi = add_mesh(s, sh.m, mats);
        if (mi < 0) return CTL_ERR_INVALID;
        int ni = ctl_host_scene_add_node(s, (uint32_t)mi, nullptr);
        if (ni < 0) return CTL_ERR_INVALID;
        if (sh.light) {
            float L[3] = {17.0f, 12.0f, 4.0f};
            if (ctl_host_scene_add_area_light(s, (uint32_t)ni, 0, L) < 0) return CTL_ERR_INVALID;
        }
    }
    float pos[3] = {278, 273, -250}, tar[3] = {278, 273, 0}, up[3] = {0, 1, 0};
    return ctl_host_scene_set_camera(s, pos, tar, up, 90.0f, 1.0f, 100000.0f, W, H);
}

ctl_status gen_c2(ctl_host_scene* s, double scale, uint32_t W, uint32_t H) {
    SplitMix64 R{0x5EED};
    std::vector<ctl_material> mats;
    for (int i = 0; i < 16; i++)
        mats.push_back(diffuse_mat((float)R.range(0.3, 0.8), (float)R.range(0.3, 0.8), (float)R.range(0.3, 0.8)));
    mats.push_back(diffuse_mat(0.8f, 0.8f, 0.8f));   // 16: light
    MeshB M;
    int n = std::max(2, (int)std::lround(180 * std::sqrt(scale)));
    M.grid(-50, -50, 100, n, hf_c2, 0, &R, 16);
    int nbox = std::max(1, (int)std::lround(1200 * scale)), nico = std::max(1, (int)std::lround(1000 * scale));
    for (int i = 0; i < nbox; i++) {
        double x = R.range(-45, 45), z = R.range(-40, 45);
        V h{R.range(0.2, 1.5), R.range(0.2, 2.5), R.range(0.2, 1.5)};
        M.box({x, hf_c2(x, z) + h.y - 0.05, z}, h, R.range(0, 3.14159), (uint8_t)(R.next() % 16));
    }
    for (int i = 0; i < nico; i++) {
        double x = R.range(-45, 45), z = R.range(-40, 45), r = R.range(0.2, 1.2);
        M.icosa({x, hf_c2(x, z) + r * 0.8, z}, r, (uint8_t)(R.next() % 16));
    }
    // one 10 x 10 m quad light at y = 25, facing down
    M.quad({5, 25, -5}, {5, 25, 5}, {-5, 25, 5}, {-5, 25, -5}, 16);
    int mi = add_mesh(s, M, mats);
    if (mi < 0) return CTL_ERR_INVALID;
    int ni = ctl_host_scene_add_node(s, (uint32_t)mi, nullptr);
    if (ni < 0) return CTL_ERR_INVALID;
    float L[3] = {40.0f, 38.0f, 34.0f};
    if (ctl_host_scene_add_area_light(s, (uint32_t)ni, 16, L) < 0) return CTL_ERR_INVALID;
    float pos[3] = {0, 1.6f + (float)hf_c2(0, -45), -45}, tar[3] = {0, 1.0f, 0}, up[3] = {0, 1, 0};
    return ctl_host_scene_set_camera(s, pos, tar, up, 60.0f, 1.0f, 100000.0f, W, H);
}

ctl_status gen_c3(ctl_host_scene* s, double scale, uint32_t W, uint32_t H, bool c5) {
    SplitMix64 R{0x5EED};
    std::vector<ctl_material> mats;
    for (int i = 0; i < 16; i++)
        mats.push_back(diffuse_mat((float)R.range(0.3, 0.8), (float)R.range(0.3, 0.8), (float)R.range(0.3, 0.8)));
    mats.push_back(diffuse_mat(0.8f, 0.8f, 0.8f));   // 16: lights
    if (c5) {
        // C5 materials (a separate stream, so the geometry stays C3's): 5 of the
        // 16 roughdielectric (Beckmann / GGX alternating, eta 1.5, alpha in
        // [0.05, 0.5]), 5 diffuse with an image texture (checker: trilinear,
        // noise: EWA), the rest constant diffuse.
        SplitMix64 Q{0x5EED ^ 0xC5C5ull};
        const float ident[6] = {1, 0, 0, 0, 1, 0}, one[3] = {1, 1, 1};
        std::vector<uint32_t> chk = tex_checker(1024), noi = tex_noise(1024, Q);
        int tc = ctl_host_scene_add_texture(s, chk.data(), 1024, 1024, CTL_TEX_TRILINEAR, CTL_WRAP_REPEAT, ident, one);
        int tn = ctl_host_scene_add_texture(s, noi.data(), 1024, 1024, CTL_TEX_EWA, CTL_WRAP_REPEAT, ident, one);
        if (tc < 0 || tn < 0) return CTL_ERR_INVALID;
        const int rough[5] = {0, 3, 6, 10, 13}, texd[5] = {1, 4, 7, 11, 14};
        for (int k = 0; k < 5; k++)
            mats[rough[k]] = rough_mat(k % 2 ? CTL_MICROFACET_GGX : CTL_MICROFACET_BECKMANN, 1.5f,
                                       (float)Q.range(0.05, 0.5));
        for (int k = 0; k < 5; k++) mats[texd[k]].texture = (uint32_t)(k % 2 ? tn : tc);
    }
    MeshB M;
    const double half = 100.0;
    // terrain: 2M triangles
    int n = std::max(4, (int)std::lround(1000 * std::sqrt(scale)));
    M.v.reserve((size_t)(10.5e6 * scale) * 3 * 2);
    M.idx.reserve((size_t)(10.5e6 * scale) * 3);
    M.mat.reserve((size_t)(10.5e6 * scale));
    M.grid(-half, -half, 2 * half, n, hf_c3, 0, &R, 4);
    // occluders: columns (128 tris) and walls (boxes), ~2M triangles
    int ncol = std::max(1, (int)std::lround(10000 * scale));
    for (int i = 0; i < ncol; i++) {
        double x = R.range(-half + 2, half - 2), z = R.range(-half + 2, half - 2);
        if (x * x + z * z < 9.0) continue;   // keep the camera position free
        M.cylinder({x, hf_c3(x, z) - 0.2, z}, R.range(0.25, 0.9), R.range(4, 12), 64, (uint8_t)(4 + R.next() % 4));
    }
    int nwall = std::max(1, (int)std::lround(60000 * scale));
    for (int i = 0; i < nwall; i++) {
        double x = R.range(-half + 2, half - 2), z = R.range(-half + 2, half - 2);
        if (x * x + z * z < 9.0) continue;
        V h{R.range(0.5, 4.0), R.range(0.5, 3.0), R.range(0.08, 0.3)};
        M.box({x, hf_c3(x, z) + h.y - 0.1, z}, h, R.range(0, 3.14159), (uint8_t)(8 + R.next() % 4));
    }
    // foliage: clustered, randomly oriented quads with log-normal edge length (sigma 1), ~6M triangles
    int nclus = std::max(1, (int)std::lround(2500 * scale));
    int perClus = 1200;
    for (int c = 0; c < nclus; c++) {
        double cx = R.range(-half + 3, half - 3), cz = R.range(-half + 3, half - 3);
        double top = R.range(4, 10);
        uint8_t m = (uint8_t)(12 + R.next() % 4);
        for (int k = 0; k < perClus; k++) {
            double x = cx + 1.6 * R.normal(), z = cz + 1.6 * R.normal();
            if (x * x + z * z < 1.0) continue;
            double y = hf_c3(cx, cz) + R.range(0.8, top);
            double e = 0.12 * std::exp(1.0 * R.normal());
            if (e < 0.02) e = 0.02;
            if (e > 1.0) e = 1.0;
            V a = norm(V{R.normal(), R.normal(), R.normal()});
            V t0 = std::fabs(a.x) > 0.5 ? V{0, 1, 0} : V{1, 0, 0};
            V u = norm(cross(a, t0)), w = norm(cross(a, u));
            V p{x, y, z};
            V hu = u * (0.5 * e), hw = w * (0.5 * e * R.range(0.4, 1.0));
            M.quad(p - hu - hw, p + hu - hw, p + hu + hw, p - hu + hw, m);
        }
    }
    // two 24 x 24 m quad lights at y = 60, facing down
    M.quad({-28, 60, -40}, {-28, 60, -16}, {-52, 60, -16}, {-52, 60, -40}, 16);
    M.quad({52, 60, 16}, {52, 60, 40}, {28, 60, 40}, {28, 60, 16}, 16);
    std::vector<float> uv;
    if (c5) {   // planar world-space UVs: the textures repeat every 50 m
        uv.resize(M.v.size() / 3 * 2);
        for (size_t i = 0; i < M.v.size() / 3; i++) {
            uv[2 * i] = (M.v[3 * i] + 100.0f) / 50.0f;
            uv[2 * i + 1] = (M.v[3 * i + 2] + 100.0f) / 50.0f;
        }
    }
    int mi = add_mesh(s, M, mats, c5 ? uv.data() : nullptr);
    if (mi < 0) return CTL_ERR_INVALID;
    int ni = ctl_host_scene_add_node(s, (uint32_t)mi, nullptr);
    if (ni < 0) return CTL_ERR_INVALID;
    float L[3] = {60.0f, 57.0f, 52.0f};
    if (ctl_host_scene_add_area_light(s, (uint32_t)ni, 16, L) < 0) return CTL_ERR_INVALID;
    float h0 = (float)hf_c3(0, 0);
    float pos[3] = {0, h0 + 1.7f, 0}, tar[3] = {30, h0 + 3.0f, 25}, up[3] = {0, 1, 0};
    return ctl_host_scene_set_camera(s, pos, tar, up, 70.0f, 1.0f, 100000.0f, W, H);
}

}  // namespace

extern "C" CTL_API ctl_status ctl_host_scene_generate(ctl_host_scene* s, int32_t config, double scale,
                                                      uint32_t width, uint32_t height) {
    if (!s || scale <= 0 || width == 0 || height == 0) return CTL_ERR_INVALID;
    switch (config) {
        case 1: return gen_cornell(s, width, height);
        case 2: return gen_c2(s, scale, width, height);
        case 3: return gen_c3(s, scale, width, height, false);
        case 5: return gen_c3(s, scale, width, height, true);
        default: ctl::set_host_error("generate: config must be 1, 2, 3 or 5"); return CTL_ERR_INVALID;
    }
}

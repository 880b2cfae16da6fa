#include <cstdlib>
// scene.cpp — host scene compiler (ctl_host_scene_* of include/ctl_trace.h).
// Produces exactly the arrays the reference's host code hands to the device:
//   Mesh::CompileMesh / ConstructBVH  (Engine/Mesh.cpp:199-290, BVHBuilderHelper.cpp:129-147)
//   TriangleData(P, mat, T, N)        (Engine/TriangleData.cu:10-68)
//   DynamicScene::CreateLight/Shape   (Engine/DynamicScene.cpp:689-766), ShapeSet (Engine/ShapeSet.cpp)
//   SceneBVH transforms               (Engine/SceneBVH.cpp:56-100)
//   LightStream::fillDeviceData       (Engine/DynamicScene.cpp:173-196)
//   getKernelSceneData eps            (Engine/DynamicScene.cpp:587)
#include "scene.h"
#include "../ctl_env.h"
#include "bvh_build.h"
#include "ref_split.h"
#include "../ctl_shade.h"
#include "../ctl_anim.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>

namespace ctl {

static thread_local std::string g_host_error;
void set_host_error(const std::string& s) { g_host_error = s; }

void woop_set(f3 a, f3 b, f3 c, ctl_woop_tri& out) { woop_set_hd(a, b, c, out.v); }

void woop_get(const ctl_woop_tri& in, f3& v0, f3& v1, f3& v2) { woop_get_hd(in.v, v0, v1, v2); }

void camera_setup(const float pos[3], const float tar[3], const float up[3], float fov_deg, float nearc, float farc,
                  uint32_t w, uint32_t h, ctl_camera& out) {
    f3 p = mk3(pos[0], pos[1], pos[2]), t = mk3(tar[0], tar[1], tar[2]), u = mk3(up[0], up[1], up[2]);
    f3 f = normalize(t - p);
    f3 r = normalize(cross(f, u));
    m44 view = m44_identity();
    view.set_col(0, mk4(r, 0)); view.set_col(1, mk4(u, 0)); view.set_col(2, mk4(f, 0));
    view.set_col(3, mk4(0, 0, 0, 1)); view.set_row(3, mk4(0, 0, 0, 1));
    m44 tr = m44_identity(); tr.at(0, 3) = p.x; tr.at(1, 3) = p.y; tr.at(2, 3) = p.z;
    m44 toWorld = matmul(tr, view);                                  // Translate(pos) % rot
    float resx = (float)w, resy = (float)h;
    float invx = 1.0f / resx, invy = 1.0f / resy;                    // Vec2f(1) / m_resolution
    float aspect = resx / resy;
    float fov = ((float)CTL_PI / 180.f) * fov_deg;                   // math::Radians
    m44 sc = m44_identity(); sc.at(0, 0) = -0.5f; sc.at(1, 1) = -0.5f * aspect; sc.at(2, 2) = 1.0f;
    m44 tl = m44_identity(); tl.at(0, 3) = -1.0f; tl.at(1, 3) = -1.0f / aspect; tl.at(2, 3) = 0.0f;
    float recip = 1.0f / (farc - nearc);                             // float4x4::Perspective
    float cot = 1.0f / cr_tan(fov / 2.0f);
    m44 pe = m44_zero();
    pe.at(0, 0) = cot; pe.at(1, 1) = cot; pe.at(2, 2) = farc * recip; pe.at(2, 3) = -nearc * farc * recip;
    pe.at(3, 2) = 1;
    m44 c2s = matmul(matmul(sc, tl), pe);
    m44 s2c = inverse(c2s);
    f3 dx = xform_point(s2c, mk3(invx, 0.0f, 0.0f)) - xform_point(s2c, mk3s(0.0f));
    f3 dy = xform_point(s2c, mk3(0.0f, invy, 0.0f)) - xform_point(s2c, mk3s(0.0f));
    memcpy(out.to_world.m, toWorld.d, 64);
    memcpy(out.sample_to_camera.m, s2c.d, 64);
    out.dx[0] = dx.x; out.dx[1] = dx.y; out.dx[2] = dx.z;
    out.dy[0] = dy.x; out.dy[1] = dy.y; out.dy[2] = dy.z;
    out.inv_resolution[0] = invx; out.inv_resolution[1] = invy;
    out.width = w; out.height = h;
}

namespace {

// TriangleData(P, matIndex, T, N) (TriangleData.cu:10-68); UVs decoded with the
// host half decode, as the reference's compile step always runs on the host.
void triangle_data(const f3 P[3], uint8_t mat, const f2 T[3], const f3 N[3], ctl_triangle_data& out) {
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    w[1] = (uint32_t)mat << 16;
    for (int i = 0; i < 3; i++)
        w[5 + i] = (uint32_t)float_to_half(T[i].x) | ((uint32_t)float_to_half(T[i].y) << 16);
    triangle_set_data(w, P[0], P[1], P[2], N[0], N[1], N[2], true);
    memcpy(out.w, w, 32);
}

template <class F>
void parallel_for(uint64_t n, uint32_t threads, F f) {
    if (threads <= 1 || n < 4096) { f(0, n); return; }
    std::vector<std::thread> ts;
    uint64_t chunk = (n + threads - 1) / threads;
    for (uint32_t t = 0; t < threads; t++) {
        uint64_t b = std::min(n, (uint64_t)t * chunk), e = std::min(n, b + chunk);
        if (b < e) ts.emplace_back([=] { f(b, e); });
    }
    for (auto& t : ts) t.join();
}

}  // namespace
bool scene_add_light(ctl_host_scene* s, uint32_t node, uint32_t local_mat, const float L[3]) {
    uint32_t perNode = 0;
    for (auto& l : s->lights) {
        if (l.node == node && l.local_mat == local_mat) {   // NodeLightIndex != -1: SetData on the old light
            l.L[0] = L[0]; l.L[1] = L[1]; l.L[2] = L[2];
            return true;
        }
        perNode += l.node == node;
    }
    if (perNode >= 2) { set_host_error("area light: MAX_AREALIGHT_NUM (2) lights per node"); return false; }
    if (s->lights.size() >= CTL_MAX_NUM_LIGHTS) { set_host_error("area light: MAX_NUM_LIGHTS (16)"); return false; }
    s->lights.push_back(ctl_host_scene::Light{node, local_mat, {L[0], L[1], L[2]}});
    return true;
}

}  // namespace ctl

using namespace ctl;

extern "C" {

CTL_API const char* ctl_host_last_error(void) { return g_host_error.c_str(); }

CTL_API void ctl_woop_set(const float v0[3], const float v1[3], const float v2[3], ctl_woop_tri* out) {
    woop_set(mk3(v0[0], v0[1], v0[2]), mk3(v1[0], v1[1], v1[2]), mk3(v2[0], v2[1], v2[2]), *out);
}

CTL_API ctl_host_scene* ctl_host_scene_create(void) { return new ctl_host_scene(); }
CTL_API void ctl_host_scene_destroy(ctl_host_scene* s) { delete s; }

CTL_API int32_t ctl_host_scene_add_mesh(ctl_host_scene* s, const float* vertices, uint32_t n_vertices,
                                        const uint32_t* indices, uint32_t n_triangles, const float* normals,
                                        const float* uvs, const uint8_t* mat_index, const ctl_material* materials,
                                        uint32_t n_materials) {
    if (!s || !vertices || !indices || n_materials == 0 || n_materials > 255) {
        set_host_error("add_mesh: invalid arguments (need vertices, indices, 1..255 materials)");
        return -1;
    }
    for (uint64_t i = 0; i < 3ull * n_triangles; i++)
        if (indices[i] >= n_vertices) { set_host_error("add_mesh: index out of range"); return -1; }
    if (mat_index)
        for (uint32_t i = 0; i < n_triangles; i++)
            if (mat_index[i] >= n_materials) { set_host_error("add_mesh: material index out of range"); return -1; }
    ctl_host_scene::Mesh m;
    m.v.assign(vertices, vertices + 3ull * n_vertices);
    m.idx.assign(indices, indices + 3ull * n_triangles);
    if (normals) m.n.assign(normals, normals + 3ull * n_vertices);
    if (uvs) m.uv.assign(uvs, uvs + 2ull * n_vertices);
    if (mat_index) m.mat.assign(mat_index, mat_index + n_triangles);
    m.materials.assign(materials, materials + n_materials);
    s->meshes.push_back(std::move(m));
    return (int32_t)s->meshes.size() - 1;
}

CTL_API int32_t ctl_host_scene_add_animated_mesh(ctl_host_scene* s, const ctl_anim_vertex* vertices,
                                                 uint32_t n_vertices, const uint32_t* indices, uint32_t n_triangles,
                                                 const float* uvs, const uint8_t* mat_index,
                                                 const ctl_material* materials, uint32_t n_materials) {
    if (!s || !vertices || n_vertices == 0) { set_host_error("add_animated_mesh: no vertices"); return -1; }
    std::vector<float> pos(3ull * n_vertices), nrm(3ull * n_vertices);
    uint32_t max_bone = 0;
    for (uint32_t i = 0; i < n_vertices; i++) {
        for (int k = 0; k < 3; k++) { pos[3ull * i + k] = vertices[i].pos[k]; nrm[3ull * i + k] = vertices[i].normal[k]; }
        uint64_t b = vertices[i].bone_indices;
        for (int k = 0; k < 8; k++, b >>= 8) max_bone = std::max(max_bone, (uint32_t)(b & 0xff));
    }
    int32_t r = ctl_host_scene_add_mesh(s, pos.data(), n_vertices, indices, n_triangles, nrm.data(), uvs, mat_index,
                                        materials, n_materials);
    if (r < 0) return r;
    auto& M = s->meshes[r];
    M.animated = true;
    M.anim_v.assign(vertices, vertices + n_vertices);
    M.max_bone = max_bone;
    return r;
}

CTL_API int32_t ctl_host_scene_add_node(ctl_host_scene* s, uint32_t mesh, const float* xf16) {
    if (!s || mesh >= s->meshes.size()) { set_host_error("add_node: bad mesh index"); return -1; }
    ctl_host_scene::Node n;
    n.mesh = mesh;
    n.has_xf = xf16 != nullptr;
    n.xf = m44_identity();
    if (xf16) memcpy(n.xf.d, xf16, 64);
    s->nodes.push_back(n);
    uint32_t ni = (uint32_t)s->nodes.size() - 1;
    // CreateNode: one light per MeshPartLight of the mesh (DynamicScene.cpp:340-341)
    for (const auto& al : s->meshes[mesh].auto_lights)
        if (!scene_add_light(s, ni, al.mat, al.L)) {
            s->lights.erase(std::remove_if(s->lights.begin(), s->lights.end(),
                                           [&](const ctl_host_scene::Light& l) { return l.node == ni; }),
                            s->lights.end());
            s->nodes.pop_back();
            return -1;
        }
    return (int32_t)ni;
}

CTL_API int32_t ctl_host_scene_add_area_light(ctl_host_scene* s, uint32_t node, uint32_t local_material,
                                              const float radiance[3]) {
    if (!s || node >= s->nodes.size()) { set_host_error("add_area_light: bad node"); return -1; }
    const auto& mesh = s->meshes[s->nodes[node].mesh];
    if (local_material >= mesh.materials.size()) { set_host_error("add_area_light: bad material"); return -1; }
    if (!scene_add_light(s, node, local_material, radiance)) return -1;
    for (size_t i = 0; i < s->lights.size(); i++)
        if (s->lights[i].node == node && s->lights[i].local_mat == local_material) return (int32_t)i;
    return -1;
}

CTL_API ctl_status ctl_host_scene_set_camera(ctl_host_scene* s, const float pos[3], const float target[3],
                                             const float up[3], float fov_deg, float near_clip, float far_clip,
                                             uint32_t width, uint32_t height) {
    if (!s || width == 0 || height == 0) return CTL_ERR_INVALID;
    memcpy(s->cam_pos, pos, 12); memcpy(s->cam_tar, target, 12); memcpy(s->cam_up, up, 12);
    s->cam_fov = fov_deg; s->cam_near = near_clip; s->cam_far = far_clip;
    s->cam_w = width; s->cam_h = height;
    s->has_camera = true;
    return CTL_OK;
}

CTL_API ctl_status ctl_host_scene_set_flags(ctl_host_scene* s, uint32_t flags) {
    if (!s) return CTL_ERR_INVALID;
    s->flags = flags;
    return CTL_OK;
}

// ImageTexture + KernelMIPMap of an RGBA8 image.  The pyramid is our own
// 2x2 box filter (the reference resamples with FreeImage, MIPMap.cpp:40-86,
// which this build does not have); the weight LUT is MIPMap.cpp:88-93.
CTL_API int32_t ctl_host_scene_add_texture(ctl_host_scene* s, const uint32_t* rgba, uint32_t w, uint32_t h,
                                           uint32_t filter, uint32_t wrap, const float mapping[6],
                                           const float scale[3]) {
    auto pow2 = [](uint32_t v) { return v && !(v & (v - 1)); };
    if (!s || !rgba || !mapping || !scale || !pow2(w) || !pow2(h) || filter > CTL_TEX_TRILINEAR || wrap > CTL_WRAP_BLACK) {
        set_host_error("add_texture: invalid argument (width and height must be powers of two)");
        return -1;
    }
    ctl_texture t{};
    t.m11 = mapping[0]; t.m12 = mapping[1]; t.m13 = mapping[2];
    t.m21 = mapping[3]; t.m22 = mapping[4]; t.m23 = mapping[5];
    t.set_id = 0;
    t.scale[0] = scale[0]; t.scale[1] = scale[1]; t.scale[2] = scale[2];
    t.width = w; t.height = h;
    t.filter = filter;
    t.wrap = wrap;
    uint32_t levels = 1;
    while (levels < 16 && (w >> levels) >= 1 && (h >> levels) >= 1) levels++;
    t.levels = levels;
    std::vector<uint32_t> cur(rgba, rgba + (size_t)w * h);
    uint64_t off = s->tex_data.size();
    for (uint32_t l = 0; l < levels; l++) {
        const uint32_t lw = w >> l, lh = h >> l;
        if (off + (uint64_t)lw * lh > 0xffffffffull) { set_host_error("add_texture: texel storage exceeds 2^32"); return -1; }
        t.offsets[l] = (uint32_t)off;
        s->tex_data.insert(s->tex_data.end(), cur.begin(), cur.end());
        off += (uint64_t)lw * lh;
        if (l + 1 == levels) break;
        std::vector<uint32_t> nxt((size_t)(lw / 2) * (lh / 2));
        for (uint32_t y = 0; y < lh / 2; y++)
            for (uint32_t x = 0; x < lw / 2; x++) {
                uint32_t px[4] = {cur[(2 * y) * lw + 2 * x], cur[(2 * y) * lw + 2 * x + 1], cur[(2 * y + 1) * lw + 2 * x],
                                  cur[(2 * y + 1) * lw + 2 * x + 1]};
                uint32_t o = 0;
                for (int c = 0; c < 4; c++) {
                    uint32_t sum = 2;
                    for (int k = 0; k < 4; k++) sum += (px[k] >> (8 * c)) & 0xffu;
                    o |= ((sum / 4) & 0xffu) << (8 * c);
                }
                nxt[(size_t)y * (lw / 2) + x] = o;
            }
        cur.swap(nxt);
    }
    for (int i = 0; i < 64; i++) {
        float r2 = (float)i / (float)(64 - 1);
        t.weight_lut[i] = cr_exp(-2.0f * r2) - cr_exp(-2.0f);
    }
    s->textures.push_back(t);
    return (int32_t)s->textures.size() - 1;
}

CTL_API ctl_status ctl_host_scene_set_bvh_params(ctl_host_scene* s, float split_alpha, uint32_t split_depth,
                                                 uint32_t bins, uint32_t max_leaf) {
    if (!s || !(split_alpha >= 0.0f) || split_depth > 16 || bins == 1 || bins > 1024 || max_leaf > 64) {
        set_host_error("set_bvh_params: invalid argument");
        return CTL_ERR_INVALID;
    }
    s->split_alpha = split_alpha;
    s->split_depth = split_depth;
    s->sah_bins = bins ? bins : CTL_DEFAULT_SAH_BINS;
    s->max_leaf = max_leaf ? max_leaf : CTL_DEFAULT_MAX_LEAF;
    return CTL_OK;
}

CTL_API ctl_status ctl_host_scene_set_environment(ctl_host_scene* s, uint32_t texture, const float scale[3]) {
    if (!s || (texture != 0xffffffffu && !scale)) { set_host_error("set_environment: invalid argument"); return CTL_ERR_INVALID; }
    s->env_texture = texture;
    if (scale)
        for (int k = 0; k < 3; k++) s->env_scale[k] = scale[k];
    return CTL_OK;
}

CTL_API ctl_status ctl_host_scene_set_environment_transform(ctl_host_scene* s, const float rot9[9]) {
    if (!s || !rot9) { set_host_error("set_environment_transform: invalid argument"); return CTL_ERR_INVALID; }
    for (int k = 0; k < 9; k++) s->env_rot[k] = rot9[k];
    return CTL_OK;
}

CTL_API ctl_status ctl_host_scene_set_bvh_builder(ctl_host_scene* s, uint32_t builder, float split_alpha) {
    if (!s || builder > CTL_BVH_SBVH || !(split_alpha >= 0.0f)) {
        set_host_error("set_bvh_builder: invalid argument");
        return CTL_ERR_INVALID;
    }
    s->builder = builder;
    s->sbvh_alpha = split_alpha;
    return CTL_OK;
}

CTL_API ctl_status ctl_host_scene_compile(ctl_host_scene* s, uint32_t threads, ctl_scene_desc* out) {
    if (!s || !out) return CTL_ERR_INVALID;
    if (!s->has_camera) { set_host_error("compile: no camera"); return CTL_ERR_INVALID; }
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    s->tri_data.clear(); s->woop.clear(); s->bvh_nodes.clear(); s->tri_indices.clear(); s->materials.clear();
    s->kmeshes.clear(); s->knodes.clear(); s->scene_bvh.clear(); s->xf.clear(); s->inv_xf.clear();
    s->klights.clear(); s->light_tris.clear(); s->light_tri_cdf.clear();
    s->max_mesh_depth = 0;
    s->compiled = false;

    std::vector<Box> meshBox(s->meshes.size());
    // --- per mesh: BVH, Woop entries, TriangleData, materials
    for (size_t mi = 0; mi < s->meshes.size(); mi++) {
        const auto& M = s->meshes[mi];
        uint32_t ntri = M.n_triangles();
        if (M.precompiled) {   // .xmsh mesh: arrays relocated as they are (Mesh::getKernelData)
            ctl_kernel_mesh km;
            km.triangle_offset = (uint32_t)s->tri_data.size();
            km.bvh_node_offset = (uint32_t)(s->bvh_nodes.size() * 4);
            km.bvh_triangle_offset = (uint32_t)(s->woop.size() * 3);
            km.bvh_indices_offset = (uint32_t)s->woop.size();
            km.std_material_offset = (uint32_t)s->materials.size();
            s->kmeshes.push_back(km);
            s->tri_data.insert(s->tri_data.end(), M.c_tri.begin(), M.c_tri.end());
            s->bvh_nodes.insert(s->bvh_nodes.end(), M.c_nodes.begin(), M.c_nodes.end());
            s->woop.insert(s->woop.end(), M.c_woop.begin(), M.c_woop.end());
            s->tri_indices.insert(s->tri_indices.end(), M.c_idx.begin(), M.c_idx.end());
            for (auto m : M.materials) {
                m.node_light_index = 0xffffffffu;
                s->materials.push_back(m);
            }
            memcpy(meshBox[mi].lo, M.c_box, 12);
            memcpy(meshBox[mi].hi, M.c_box + 3, 12);
            s->max_mesh_depth = std::max(s->max_mesh_depth, M.c_depth);
            continue;
        }
        auto V = [&](uint32_t vi) { return mk3(M.v[3 * vi], M.v[3 * vi + 1], M.v[3 * vi + 2]); };
        std::vector<Box> boxes(ntri);
        parallel_for(ntri, threads, [&](uint64_t b, uint64_t e) {
            for (uint64_t t = b; t < e; t++) {
                Box& bx = boxes[t];
                for (int k = 0; k < 3; k++) { bx.lo[k] = FLT_MAX; bx.hi[k] = -FLT_MAX; }
                for (int c = 0; c < 3; c++) {
                    f3 p = V(M.idx[3 * t + c]);
                    float q[3] = {p.x, p.y, p.z};
                    for (int k = 0; k < 3; k++) { bx.lo[k] = tmin(bx.lo[k], q[k]); bx.hi[k] = tmax(bx.hi[k], q[k]); }
                }
            }
        });
        BvhBuildParams bp;
        bp.threads = threads;
        bp.bins = s->sah_bins;
        bp.max_leaf = s->max_leaf;
        BvhOutput bo;
        if (s->builder == CTL_BVH_SBVH && !M.animated) {
            // the reference's SplitBVHBuilder (spatial splits inside the build)
            std::vector<float> tv((size_t)ntri * 9);
            parallel_for(ntri, threads, [&](uint64_t b, uint64_t e) {
                for (uint64_t t = b; t < e; t++)
                    for (int c = 0; c < 3; c++) {
                        f3 p = V(M.idx[3 * t + c]);
                        tv[9 * t + 3 * c] = p.x; tv[9 * t + 3 * c + 1] = p.y; tv[9 * t + 3 * c + 2] = p.z;
                    }
            });
            SbvhParams sp;
            sp.max_leaf = s->max_leaf;
            sp.split_alpha = s->sbvh_alpha;
            sp.threads = threads;
            build_sbvh(tv.data(), ntri, sp, bo);
        } else if (s->split_alpha > 0.0f && s->split_depth > 0 && !M.animated) {
            // references of large triangles split in space (ref_split.h)
            std::vector<float> tv((size_t)ntri * 9);
            parallel_for(ntri, threads, [&](uint64_t b, uint64_t e) {
                for (uint64_t t = b; t < e; t++)
                    for (int c = 0; c < 3; c++) {
                        f3 p = V(M.idx[3 * t + c]);
                        tv[9 * t + 3 * c] = p.x; tv[9 * t + 3 * c + 1] = p.y; tv[9 * t + 3 * c + 2] = p.z;
                    }
            });
            RefSplitParams rp;
            rp.alpha = s->split_alpha;
            rp.max_depth = s->split_depth;
            rp.threads = threads;
            std::vector<Box> rb;
            std::vector<uint32_t> rid;
            split_refs(tv.data(), boxes.data(), ntri, rp, rb, rid);
            if (rb.size() >= 0x7fffffffull) { set_host_error("compile: too many BVH references"); return CTL_ERR_INVALID; }
            build_bvh(rb.data(), (uint32_t)rb.size(), bp, bo, rid.data());
        } else {
            build_bvh(boxes.data(), ntri, bp, bo);
        }
        s->max_mesh_depth = std::max(s->max_mesh_depth, bo.max_depth);
        meshBox[mi] = bo.root_box;

        ctl_kernel_mesh km;
        km.triangle_offset = (uint32_t)s->tri_data.size();
        km.bvh_node_offset = (uint32_t)(s->bvh_nodes.size() * 4);
        km.bvh_triangle_offset = (uint32_t)(s->woop.size() * 3);
        km.bvh_indices_offset = (uint32_t)s->woop.size();
        km.std_material_offset = (uint32_t)s->materials.size();
        s->kmeshes.push_back(km);

        s->bvh_nodes.insert(s->bvh_nodes.end(), bo.nodes.begin(), bo.nodes.end());
        size_t e0 = s->woop.size(), ne = bo.leaf_objects.size();
        s->woop.resize(e0 + ne);
        s->tri_indices.resize(e0 + ne);
        parallel_for(ne, threads, [&](uint64_t b, uint64_t e) {
            for (uint64_t i = b; i < e; i++) {
                uint32_t t = bo.leaf_objects[i];
                woop_set(V(M.idx[3 * t]), V(M.idx[3 * t + 1]), V(M.idx[3 * t + 2]), s->woop[e0 + i]);
                s->tri_indices[e0 + i] = (t << 1) | (bo.leaf_last[i] ? 1u : 0u);
            }
        });
        size_t t0 = s->tri_data.size();
        s->tri_data.resize(t0 + ntri);
        parallel_for(ntri, threads, [&](uint64_t b, uint64_t e) {
            for (uint64_t t = b; t < e; t++) {
                f3 P[3]; f2 T[3]; f3 N[3];
                for (int c = 0; c < 3; c++) {
                    uint32_t vi = M.idx[3 * t + c];
                    P[c] = V(vi);
                    T[c] = M.uv.empty() ? mk2(0, 0) : mk2(M.uv[2 * vi], M.uv[2 * vi + 1]);
                }
                f3 fn = normalize(cross(P[1] - P[0], P[2] - P[0]));
                for (int c = 0; c < 3; c++) {
                    uint32_t vi = M.idx[3 * t + c];
                    N[c] = M.n.empty() ? fn : mk3(M.n[3 * vi], M.n[3 * vi + 1], M.n[3 * vi + 2]);
                }
                triangle_data(P, M.mat.empty() ? 0 : M.mat[t], T, N, s->tri_data[t0 + t]);
            }
        });
        for (auto m : M.materials) {
            m.node_light_index = 0xffffffffu;
            s->materials.push_back(m);
        }
    }
    s->kmesh_box.resize(6 * s->meshes.size());
    for (size_t mi = 0; mi < s->meshes.size(); mi++) {
        memcpy(&s->kmesh_box[6 * mi], meshBox[mi].lo, 12);
        memcpy(&s->kmesh_box[6 * mi + 3], meshBox[mi].hi, 12);
    }
    s->k_anim_vertices.clear(); s->k_anim_tris.clear(); s->k_anim_meshes.clear();
    for (size_t mi = 0; mi < s->meshes.size(); mi++) {
        const auto& M = s->meshes[mi];
        if (!M.animated) continue;
        ctl_anim_mesh am;
        am.mesh = (uint32_t)mi;
        am.vertex_first = (uint32_t)s->k_anim_vertices.size();
        am.vertex_count = (uint32_t)M.anim_v.size();
        am.tri_first = (uint32_t)(s->k_anim_tris.size() / 3);
        am.tri_count = M.n_triangles();
        am.max_bone = M.max_bone;
        s->k_anim_vertices.insert(s->k_anim_vertices.end(), M.anim_v.begin(), M.anim_v.end());
        s->k_anim_tris.insert(s->k_anim_tris.end(), M.idx.begin(), M.idx.end());
        s->k_anim_meshes.push_back(am);
    }

    // --- nodes (instances), transforms, top-level BVH
    Box sceneBox;
    for (int k = 0; k < 3; k++) { sceneBox.lo[k] = FLT_MAX; sceneBox.hi[k] = -FLT_MAX; }
    std::vector<Box> nodeBox(s->nodes.size());
    for (size_t ni = 0; ni < s->nodes.size(); ni++) {
        const auto& N = s->nodes[ni];
        ctl_node kn{};
        kn.mesh_index = N.mesh;
        kn.material_offset = s->kmeshes[N.mesh].std_material_offset;
        kn.instanced_material = 0;
        kn.lights[0] = kn.lights[1] = 0xffffffffu;
        kn.num_lights = 0;
        s->knodes.push_back(kn);
        ctl_float4x4 a, b;
        memcpy(a.m, N.xf.d, 64);
        m44 inv = N.has_xf ? inverse(N.xf) : m44_identity();   // SceneBVH::setTransform / ctor identity
        memcpy(b.m, inv.d, 64);
        s->xf.push_back(a);
        s->inv_xf.push_back(b);
        const Box& mb = meshBox[N.mesh];
        Box wb;
        instance_box(N.xf, mb.lo, mb.hi, wb.lo, wb.hi);
        nodeBox[ni] = wb;
        for (int k = 0; k < 3; k++) { sceneBox.lo[k] = tmin(sceneBox.lo[k], wb.lo[k]); sceneBox.hi[k] = tmax(sceneBox.hi[k], wb.hi[k]); }
    }
    int32_t startNode = 0x76543210;
    if (!s->nodes.empty()) {
        BvhBuildParams bp;
        bp.leaf_size_one = true;
        bp.threads = 1;
        BvhOutput bo;
        build_bvh(nodeBox.data(), (uint32_t)nodeBox.size(), bp, bo);
        s->scene_bvh = bo.nodes;
        startNode = bo.start_node;
    }

    // --- lights (CreateLight -> CreateShape -> ShapeSet)
    for (size_t li = 0; li < s->lights.size(); li++) {
        const auto& L = s->lights[li];
        if (s->meshes[s->nodes[L.node].mesh].animated) {
            set_host_error("compile: area lights on animated meshes are not supported");
            return CTL_ERR_INVALID;
        }
        ctl_node& kn = s->knodes[L.node];
        const ctl_kernel_mesh& km = s->kmeshes[kn.mesh_index];
        ctl_material& mat = s->materials[kn.material_offset + L.local_mat];
        if (mat.node_light_index == 0xffffffffu) {
            mat.node_light_index = kn.num_lights;
            kn.lights[kn.num_lights++] = (uint32_t)li;
        }
        ctl_light kl{};
        kl.radiance[0] = L.L[0]; kl.radiance[1] = L.L[1]; kl.radiance[2] = L.L[2];
        kl.orthogonal = 0;
        kl.tri_first = (uint32_t)s->light_tris.size();
        kl.cdf_first = (uint32_t)s->light_tri_cdf.size();
        kl.node_idx = L.node;
        const auto& M = s->meshes[kn.mesh_index];
        uint32_t ntri = M.n_triangles();
        // entries of this mesh: [bvh_indices_offset, next mesh)
        uint64_t e0 = km.bvh_indices_offset;
        uint64_t e1 = (kn.mesh_index + 1 < s->kmeshes.size()) ? s->kmeshes[kn.mesh_index + 1].bvh_indices_offset
                                                              : s->woop.size();
        std::vector<uint32_t> seen;
        std::vector<char> used(ntri, 0);
        m44 mxf = s->nodes[L.node].xf;
        for (uint64_t e = e0; e < e1; e++) {
            uint32_t i2 = s->tri_indices[e] >> 1;
            const ctl_triangle_data& td = s->tri_data[km.triangle_offset + i2];
            if (((td.w[1] >> 16) & 0xff) != L.local_mat || used[i2]) continue;
            used[i2] = 1;
            ctl_light_tri lt{};
            light_tri_recalc(s->woop[e].v, td, mxf, lt);   // ShapeSet::triData::Recalculate (host fillDG)
            lt.i_dat = (uint32_t)e;
            lt.t_dat = km.triangle_offset + i2;
            s->light_tris.push_back(lt);
        }
        kl.tri_count = (uint32_t)(s->light_tris.size() - kl.tri_first);
        if (kl.tri_count == 0) { set_host_error("compile: area light material has no triangles"); return CTL_ERR_INVALID; }
        std::vector<float> cdf(kl.tri_count + 1);
        kl.sum_area = shapeset_cdf(s->light_tris.data() + kl.tri_first, kl.tri_count, cdf.data());
        s->light_tri_cdf.insert(s->light_tri_cdf.end(), cdf.begin(), cdf.end());
        s->klights.push_back(kl);
    }
    // DynamicScene::setEnvironementMap: the InfiniteLight goes after the area lights
    // (m_uEnvMapIndex); its constructor's tables and Update()'s scene sphere
    uint32_t envIndex = 0xffffffffu;
    s->env_tables.clear();
    if (s->env_texture != 0xffffffffu) {
        if (s->env_texture >= s->textures.size()) { set_host_error("compile: environment texture index out of range"); return CTL_ERR_INVALID; }
        if (s->klights.size() >= CTL_MAX_NUM_LIGHTS) { set_host_error("compile: more than 16 lights"); return CTL_ERR_INVALID; }
        ctl_env_light& L = s->kenv;
        L = ctl_env_light{};
        L.texture = s->env_texture;
        for (int k = 0; k < 3; k++) L.scale[k] = s->env_scale[k];
        for (int k = 0; k < 9; k++) L.world[k / 3][k % 3] = s->env_rot[k];   // m_worldTransform
        const ctl_texture& t = s->textures[L.texture];
        s->env_tables.assign(env_table_floats(t.width, t.height), 0.0f);
        EnvView E{&L, nullptr, s->textures.data(), s->tex_data.data()};
        env_build_tables(E, L, s->env_tables.data());
        const f3 lo = mk3(sceneBox.lo[0], sceneBox.lo[1], sceneBox.lo[2]), hi = mk3(sceneBox.hi[0], sceneBox.hi[1], sceneBox.hi[2]);
        const f3 c = (lo + hi) * 0.5f;   // AABB::Center
        L.scene_center[0] = c.x; L.scene_center[1] = c.y; L.scene_center[2] = c.z;
        L.scene_radius = length(hi - lo) / 1.5f;
        ctl_light kl{};
        kl.kind = CTL_LIGHT_INFINITE;
        kl.node_idx = 0xffffffffu;
        envIndex = (uint32_t)s->klights.size();
        s->klights.push_back(kl);
    }

    ctl_scene_desc& d = s->desc;
    d = ctl_scene_desc{};
    d.tri_data = s->tri_data.data(); d.n_tri_data = s->tri_data.size();
    d.woop_tris = s->woop.data(); d.n_woop_tris = s->woop.size();
    d.bvh_nodes = s->bvh_nodes.data(); d.n_bvh_nodes = s->bvh_nodes.size();
    d.tri_indices = s->tri_indices.data(); d.n_tri_indices = s->tri_indices.size();
    d.materials = s->materials.data(); d.n_materials = (uint32_t)s->materials.size();
    d.meshes = s->kmeshes.data(); d.n_meshes = (uint32_t)s->kmeshes.size();
    d.nodes = s->knodes.data(); d.n_nodes = (uint32_t)s->knodes.size();
    d.scene_bvh_nodes = s->scene_bvh.data(); d.n_scene_bvh_nodes = (uint32_t)s->scene_bvh.size();
    d.scene_start_node = startNode;
    d.mesh_boxes = s->kmesh_box.data();
    d.anim_vertices = s->k_anim_vertices.data(); d.n_anim_vertices = (uint32_t)s->k_anim_vertices.size();
    d.anim_triangles = s->k_anim_tris.data(); d.n_anim_triangles = (uint32_t)(s->k_anim_tris.size() / 3);
    d.anim_meshes = s->k_anim_meshes.data(); d.n_anim_meshes = (uint32_t)s->k_anim_meshes.size();
    d.node_xf = s->xf.data(); d.node_inv_xf = s->inv_xf.data();
    d.lights = s->klights.data(); d.n_lights = (uint32_t)s->klights.size();
    d.light_tris = s->light_tris.data(); d.n_light_tris = (uint32_t)s->light_tris.size();
    d.light_tri_cdf = s->light_tri_cdf.data(); d.n_light_tri_cdf = (uint32_t)s->light_tri_cdf.size();
    {   // LightStream::fillDeviceData with unit weights
        uint32_t n = (uint32_t)s->klights.size();
        float accum = 0;
        for (uint32_t i = 0; i < n; i++) accum += 1.0f;
        for (uint32_t i = 0; i < n; i++) {
            float pdf = 1.0f / accum;
            d.light_cdf[i] = (i > 0 ? d.light_cdf[i - 1] : 0.0f) + pdf;
        }
    }
    d.env_map_index = envIndex;
    d.env = envIndex != 0xffffffffu ? &s->kenv : nullptr;
    d.env_data = s->env_tables.data();
    d.n_env_data = s->env_tables.size();
    d.textures = s->textures.data();
    d.n_textures = (uint32_t)s->textures.size();
    d.tex_data = s->tex_data.data();
    d.n_tex_data = s->tex_data.size();
    for (const ctl_material& m : s->materials)
        if (m.bsdf_type == CTL_BSDF_DIFFUSE && m.texture != 0xffffffffu && m.texture >= s->textures.size()) {
            set_host_error("compile: material texture index out of range");
            return CTL_ERR_INVALID;
        }
    for (int k = 0; k < 3; k++) { d.box_min[k] = sceneBox.lo[k]; d.box_max[k] = sceneBox.hi[k]; }
    f3 size = mk3(sceneBox.hi[0] - sceneBox.lo[0], sceneBox.hi[1] - sceneBox.lo[1], sceneBox.hi[2] - sceneBox.lo[2]);
    d.ray_eps = 1e-4f * length(size);   // MIN_RAYTRACE_DISTANCE_RELATIVE * |box|
    camera_setup(s->cam_pos, s->cam_tar, s->cam_up, s->cam_fov, s->cam_near, s->cam_far, s->cam_w, s->cam_h, d.camera);
    d.flags = s->flags;
    *out = d;
    s->compiled = true;
    return CTL_OK;
}

}  // extern "C"

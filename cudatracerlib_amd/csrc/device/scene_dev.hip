// scene_dev.hip — the device copy of the scene behind the C ABI:
//
//   ctl_scene_upload   replaces the scene (DynamicScene::UpdateScene after a load
//                      + UpdateKernel, Engine/DynamicScene.cpp:480-554,
//                      Kernel/TraceHelper.cu:182-217): every array copied once
//   ctl_scene_update   the per-pass UpdateKernel and the incremental
//                      UpdateScene: the scene constants (camera, ray epsilon,
//                      light CDF, box) always, and only the arrays the caller
//                      marks dirty (the reference's Stream<T>::Invalidate +
//                      UpdateInvalidated, Base/Buffer.h:257-291).  A clean
//                      scene costs no copy and no device synchronisation, so the
//                      reference's DoPass loop (UpdateKernel every pass,
//                      Kernel/Tracer.h:229) drops in at the cost of a kernel
//                      argument.
//
// One device allocation per KernelDynamicScene stream (SceneArr, common.h),
// reused while its contents fit.  The 4-wide trees are rebuilt from the binary
// ones only when a tree array is dirty; the instance tree's refit plan and the
// animation state follow the arrays they are built from.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/ctl_trace.h"
#include "../host/bvh_wide.h"
#include "../ctl_qnode.h"
#include "common.h"

using namespace ctl;

namespace {

#define SD_HIP(ctx, call)                                                                  \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string("scene: ") + #call + ": " + hipGetErrorString(e_);    \
            return CTL_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

constexpr uint32_t kDirtyTrees = CTL_DIRTY_BVH | CTL_DIRTY_NODES;

void free_arrays(ctl_ctx* c) {
    for (SceneArray& a : c->sarr) {
        if (a.p) (void)hipFree(a.p);
        a = SceneArray{};
    }
}

// Array slot `a` receives `bytes` from the host plus `pad` zero bytes.  The
// allocation is reused while it fits (stream-ordered copy: kernels queued
// before on the stream read the old contents); a larger array is reallocated
// after the device has drained (kernels on any stream may read the old one).
ctl_status put(ctl_ctx* c, int a, const void* src, size_t bytes, size_t pad, hipStream_t s) {
    SceneArray& A = c->sarr[a];
    const size_t need = std::max<size_t>(bytes + pad, 16);
    if (A.cap < need) {
        if (A.p) {
            SD_HIP(c, hipDeviceSynchronize());
            (void)hipFree(A.p);
            A = SceneArray{};
        }
        if (hipMalloc(&A.p, need) != hipSuccess) {
            A.p = nullptr;
            c->err = "scene: hipMalloc of " + std::to_string(need) + " bytes failed";
            return CTL_ERR_NOMEM;
        }
        A.cap = need;
    }
    if (pad) SD_HIP(c, hipMemsetAsync(static_cast<char*>(A.p) + bytes, 0, pad, s));
    if (bytes) SD_HIP(c, hipMemcpyAsync(A.p, src, bytes, hipMemcpyHostToDevice, s));
    A.bytes = bytes;
    return CTL_OK;
}

template <class T>
const T* dptr(ctl_ctx* c, int a) { return reinterpret_cast<const T*>(c->sarr[a].p); }

// What ctl_scene_upload refuses (include/ctl_trace.h), per group of arrays.
ctl_status validate(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty) {
    if (d->n_lights > CTL_MAX_NUM_LIGHTS) { c->err = "scene_upload: more than 16 lights"; return CTL_ERR_INVALID; }
    if (dirty & (CTL_DIRTY_LIGHTS | CTL_DIRTY_ENV)) {
        for (uint32_t i = 0; i < d->n_lights; i++) {
            if (d->lights[i].orthogonal) { c->err = "scene_upload: orthogonal DiffuseLight unsupported"; return CTL_ERR_INVALID; }
            if (d->lights[i].kind > CTL_LIGHT_INFINITE || (d->lights[i].kind == CTL_LIGHT_INFINITE) != (i == d->env_map_index)) {
                c->err = "scene_upload: the environment light must be the light env_map_index names";
                return CTL_ERR_INVALID;
            }
        }
    }
    if ((dirty & (CTL_DIRTY_ENV | CTL_DIRTY_TEXTURES | CTL_DIRTY_LIGHTS)) && d->env_map_index != 0xffffffffu) {
        const ctl_env_light* e = d->env;
        if (d->env_map_index >= d->n_lights || !e || e->texture >= d->n_textures || !d->env_data) {
            c->err = "scene_upload: environment light without its record, texture or tables";
            return CTL_ERR_INVALID;
        }
        const uint32_t w = (uint32_t)e->size[0], h = (uint32_t)e->size[1];
        if (w != d->textures[e->texture].width || h != d->textures[e->texture].height ||
            (uint64_t)e->cdf_cols + (uint64_t)(w + 1) * h > d->n_env_data || (uint64_t)e->cdf_rows + h + 1 > d->n_env_data ||
            (uint64_t)e->row_weights + h > d->n_env_data) {
            c->err = "scene_upload: environment tables do not match the radiance map";
            return CTL_ERR_INVALID;
        }
        bool ortho = true;   // the world transform: a rotation (orthonormal rows)
        for (int i = 0; i < 3 && ortho; i++)
            for (int j = 0; j < 3 && ortho; j++) {
                float s = 0.0f;
                for (int k = 0; k < 3; k++) s += e->world[i][k] * e->world[j][k];
                ortho = fabsf(s - (i == j ? 1.0f : 0.0f)) < 1e-4f;
            }
        if (!ortho) { c->err = "scene_upload: the environment's world transform is not a rotation"; return CTL_ERR_INVALID; }
    }
    if (dirty & (CTL_DIRTY_MATERIALS | CTL_DIRTY_TEXTURES)) {
        for (uint32_t i = 0; i < d->n_materials; i++) {
            const ctl_material& m = d->materials[i];
            if (m.bsdf_type != CTL_BSDF_DIFFUSE && m.bsdf_type != CTL_BSDF_ROUGHDIELECTRIC) {
                c->err = "scene_upload: only diffuse and roughdielectric BSDFs are supported";
                return CTL_ERR_INVALID;
            }
            if (m.bsdf_type == CTL_BSDF_ROUGHDIELECTRIC && (m.distribution > CTL_MICROFACET_GGX || !m.sample_visible)) {
                c->err = "scene_upload: roughdielectric needs a Beckmann/GGX distribution with visible-normal sampling";
                return CTL_ERR_INVALID;
            }
            if (m.bsdf_type == CTL_BSDF_DIFFUSE && m.texture != 0xffffffffu && m.texture >= d->n_textures) {
                c->err = "scene_upload: material texture index out of range";
                return CTL_ERR_INVALID;
            }
            if (m.alpha_state) {
                const uint32_t st = m.alpha_state;
                if (st != 1 && st != 2 && st != 5 && st != 6) {
                    c->err = "scene_upload: alpha state must be 0, 1, 2, 5 or 6 (color compare unsupported)";
                    return CTL_ERR_INVALID;
                }
                if (st < 4 && (m.alpha_texture == 0xffffffffu || m.alpha_texture >= d->n_textures)) {
                    c->err = "scene_upload: alpha map texture index out of range";
                    return CTL_ERR_INVALID;
                }
                if (m.bsdf_type != CTL_BSDF_DIFFUSE && st >= 4) {
                    c->err = "scene_upload: reflectance-map alpha needs a diffuse material";
                    return CTL_ERR_INVALID;
                }
            }
        }
    }
    if (dirty & CTL_DIRTY_TEXTURES) {
        for (uint32_t i = 0; i < d->n_textures; i++) {
            const ctl_texture& t = d->textures[i];
            if (t.levels == 0 || t.levels > 16 || t.width < 2 || t.height < 2 || t.set_id != 0 ||
                (uint64_t)t.offsets[t.levels - 1] + (uint64_t)(t.width >> (t.levels - 1)) * (t.height >> (t.levels - 1)) > d->n_tex_data) {
                c->err = "scene_upload: invalid texture record";
                return CTL_ERR_INVALID;
            }
        }
    }
    return CTL_OK;
}

// A clean array must still hold what the desc describes.
ctl_status check_clean(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty) {
    struct Row { uint32_t bit; int arr; uint64_t bytes; const char* name; };
    const Row rows[] = {
        {CTL_DIRTY_BVH, SA_BVH, d->n_bvh_nodes * sizeof(ctl_bvh_node), "bvh_nodes"},
        {CTL_DIRTY_WOOP, SA_WOOP, d->n_woop_tris * sizeof(ctl_woop_tri), "woop_tris"},
        {CTL_DIRTY_TRI_INDICES, SA_IDX, d->n_tri_indices * sizeof(ctl_tri_index), "tri_indices"},
        {CTL_DIRTY_TRI_DATA, SA_TRI, d->n_tri_data * sizeof(ctl_triangle_data), "tri_data"},
        {CTL_DIRTY_MATERIALS, SA_MATS, d->n_materials * sizeof(ctl_material), "materials"},
        {CTL_DIRTY_MESHES, SA_MESHES, d->n_meshes * sizeof(ctl_kernel_mesh), "meshes"},
        {CTL_DIRTY_NODES, SA_NODES, d->n_nodes * sizeof(ctl_node), "nodes"},
        {CTL_DIRTY_NODES, SA_SBVH, (uint64_t)d->n_scene_bvh_nodes * sizeof(ctl_bvh_node), "scene_bvh_nodes"},
        {CTL_DIRTY_LIGHTS, SA_LIGHTS, d->n_lights * sizeof(ctl_light), "lights"},
        {CTL_DIRTY_LIGHTS, SA_LTRIS, d->n_light_tris * sizeof(ctl_light_tri), "light_tris"},
        {CTL_DIRTY_LIGHTS, SA_LCDF, d->n_light_tri_cdf * sizeof(float), "light_tri_cdf"},
        {CTL_DIRTY_TEXTURES, SA_TEX, d->n_textures * sizeof(ctl_texture), "textures"},
        {CTL_DIRTY_TEXTURES, SA_TEXDATA, d->n_tex_data * sizeof(uint32_t), "tex_data"},
    };
    for (const Row& r : rows)
        if (!(dirty & r.bit) && c->sarr[r.arr].bytes != r.bytes) {
            c->err = std::string("scene_update: ") + r.name + " changed size but is not marked dirty";
            return CTL_ERR_INVALID;
        }
    if (!(dirty & CTL_DIRTY_ENV) && (d->env_map_index != 0xffffffffu) != (c->scene.env_index != 0xffffffffu)) {
        c->err = "scene_update: the environment light changed but CTL_DIRTY_ENV is not set";
        return CTL_ERR_INVALID;
    }
    if (!(dirty & CTL_DIRTY_NODES) && (d->scene_start_node != c->scene.start_node || d->n_nodes != c->scene.n_nodes)) {
        c->err = "scene_update: the instance tree changed but CTL_DIRTY_NODES is not set";
        return CTL_ERR_INVALID;
    }
    return CTL_OK;
}

// The scene constants every UpdateKernel refreshes (KernelDynamicScene's
// non-array members: m_Camera, m_rayTraceEps, m_sBox, the light CDF), plus the
// shading level from the materials and the environment light.
void set_constants(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty) {
    DevScene& S = c->scene;
    S.n_lights = d->n_lights;
    S.flags = d->flags;
    // After ctl_scene_set_transform / ctl_scene_animate the device holds the
    // scene box the reference's getSceneBox would return (DynamicScene.cpp:583-587),
    // and its epsilon wins over the desc's until the instances are uploaded again.
    if (!c->device_eps || (dirty & CTL_DIRTY_NODES)) {
        S.ray_eps = d->ray_eps;
        cull_bound(d->box_min, d->box_max, d->mesh_boxes, d->n_meshes, S.cull_m);
        // the desc's boxes bound the device's trees here: after set_transform /
        // animate (device_edited) an instance update re-uploads every edited array
        // with the trees (commit), so no moved box outlives this bound
        c->device_eps = false;
    }
    for (int i = 0; i < CTL_MAX_NUM_LIGHTS; i++) S.light_cdf[i] = d->light_cdf[i];
    S.camera = d->camera;
    c->half_quirk = (d->flags & CTL_SCENE_HALF_HOST_QUIRK) != 0;
}

ctl_status commit_arrays(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty, hipStream_t s);

// Every commit that changes the device scene (an array, or a constant such as
// the camera) moves the scene epoch: render-ahead passes (ctl_render_pass)
// belong to the epoch they were rendered in.
ctl_status commit(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty, hipStream_t s) {
    DevScene before = c->scene;
    const ctl_status r = commit_arrays(c, d, dirty, s);
    if (r != CTL_OK || dirty != 0 || std::memcmp(&before, &c->scene, sizeof(DevScene)) != 0) c->scene_epoch++;
    return r;
}

ctl_status commit_arrays(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty, hipStream_t s) {
    // a change of the device tree format rebuilds the trees
    const uint32_t tree_bits = CTL_SCENE_BINARY_BVH | CTL_SCENE_WIDE_QUANT;
    if ((d->flags & tree_bits) != c->tree_flags) dirty |= kDirtyTrees;
    // quantized trees are encoded together
    if ((d->flags & CTL_SCENE_WIDE_QUANT) && (dirty & kDirtyTrees)) dirty |= kDirtyTrees;
    // animated meshes: their rebuild plans describe the trees on the device (shape,
    // leaf holders, 4-wide links), so a tree update re-uploads every tree with them
    if (d->n_anim_meshes > 0 && (dirty & (kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES)))
        dirty |= kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES;
    // the rebuild plans (anim_setup) keep host copies of the instance trees
    if (dirty & (kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES)) dirty |= CTL_DIRTY_NODES;
    // after set_transform / animate, re-uploading any tree group returns every
    // device-edited array to the desc (geometry, instances, their area lights,
    // the environment's scene sphere), never a mix of moved and unmoved state
    if (c->device_edited && (dirty & (kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES)))
        dirty |= kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES | CTL_DIRTY_TRI_DATA | CTL_DIRTY_WOOP |
                 CTL_DIRTY_LIGHTS | CTL_DIRTY_ENV;
    ctl_status r;
    if ((r = validate(c, d, dirty)) != CTL_OK) return r;
    if ((r = check_clean(c, d, dirty)) != CTL_OK) return r;
    DevScene& S = c->scene;
#define PUT(bit, arr, src, cnt, T, pad)                                                             \
    if (dirty & (bit)) {                                                                            \
        if ((r = put(c, arr, src, (size_t)(cnt) * sizeof(T), (size_t)(pad) * sizeof(T), s)) != CTL_OK) return r; \
    }
    PUT(CTL_DIRTY_BVH, SA_BVH, d->bvh_nodes, d->n_bvh_nodes, ctl_bvh_node, 0);
    // one zeroed entry past the end: the leaf loop loads entry i+1 while it tests entry i
    PUT(CTL_DIRTY_WOOP, SA_WOOP, d->woop_tris, d->n_woop_tris, ctl_woop_tri, 1);
    PUT(CTL_DIRTY_TRI_INDICES, SA_IDX, d->tri_indices, d->n_tri_indices, ctl_tri_index, 1);
    PUT(CTL_DIRTY_TRI_DATA, SA_TRI, d->tri_data, d->n_tri_data, ctl_triangle_data, 0);
    PUT(CTL_DIRTY_MATERIALS, SA_MATS, d->materials, d->n_materials, ctl_material, 0);
    PUT(CTL_DIRTY_MESHES, SA_MESHES, d->meshes, d->n_meshes, ctl_kernel_mesh, 0);
    PUT(CTL_DIRTY_NODES, SA_NODES, d->nodes, d->n_nodes, ctl_node, 0);
    PUT(CTL_DIRTY_NODES, SA_SBVH, d->scene_bvh_nodes, d->n_scene_bvh_nodes, ctl_bvh_node, 0);
    PUT(CTL_DIRTY_NODES, SA_XF, d->node_xf, d->n_nodes, ctl_float4x4, 0);
    PUT(CTL_DIRTY_NODES, SA_IXF, d->node_inv_xf, d->n_nodes, ctl_float4x4, 0);
    PUT(CTL_DIRTY_LIGHTS, SA_LIGHTS, d->lights, d->n_lights, ctl_light, 0);
    PUT(CTL_DIRTY_LIGHTS, SA_LTRIS, d->light_tris, d->n_light_tris, ctl_light_tri, 0);
    PUT(CTL_DIRTY_LIGHTS, SA_LCDF, d->light_tri_cdf, d->n_light_tri_cdf, float, 0);
    PUT(CTL_DIRTY_TEXTURES, SA_TEX, d->textures, d->n_textures, ctl_texture, 0);
    PUT(CTL_DIRTY_TEXTURES, SA_TEXDATA, d->tex_data, d->n_tex_data, uint32_t, 0);
    if ((dirty & CTL_DIRTY_ENV) && d->env_map_index != 0xffffffffu) {
        PUT(CTL_DIRTY_ENV, SA_ENV, d->env, 1, ctl_env_light, 0);
        PUT(CTL_DIRTY_ENV, SA_ENVDATA, d->env_data, d->n_env_data, float, 0);
    }
    if (!c->sarr[SA_LUT].bytes) {
        // decoded spherical-normal table (Uchar2ToNormalizedFloat3, Compression.h:20-31)
        std::vector<float4> lut(65536);
        for (uint32_t code = 0; code < 65536; code++) {
            f3 v = normal_decode16(code);
            lut[code] = make_float4(v.x, v.y, v.z, 0.0f);
        }
        if ((r = put(c, SA_LUT, lut.data(), lut.size() * sizeof(float4), 0, s)) != CTL_OK) return r;
        SD_HIP(c, hipStreamSynchronize(s));   // the table is a local
    }
#undef PUT
    // 4-wide trees (host/bvh_wide.h) for the device traversal, unless the caller
    // asks for the reference's binary visit order
    const bool wide = (d->flags & CTL_SCENE_BINARY_BVH) == 0 && d->n_bvh_nodes > 0;
    const bool animated = d->n_anim_meshes > 0;
    std::vector<WideNode> wn, sw;
    // the 4-wide mesh trees read the binary nodes, the leaf entries' last-in-leaf
    // flags (counted leaves) and the per-mesh offsets
    const bool mesh_trees = (dirty & (CTL_DIRTY_BVH | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES)) != 0;
    const bool top_tree = (dirty & CTL_DIRTY_NODES) != 0;
    try {
        if (mesh_trees) {
            c->h_wbase.assign(d->n_meshes, 0);
            int mesh_bin = 0, mesh_wide = 0;
            for (uint32_t m = 0; m < d->n_meshes && d->n_bvh_nodes > 0; m++) {
                const size_t first = d->meshes[m].bvh_node_offset / 4;
                if (first >= d->n_bvh_nodes) throw std::runtime_error("mesh BVH offset out of range");
                mesh_bin = std::max(mesh_bin, binary_stack_bound(d->bvh_nodes + first, d->n_bvh_nodes - first, 0, kStackMax));
                if (!wide) continue;
                c->h_wbase[m] = (uint32_t)wn.size();
                // the mesh's entries start at bvh_indices_offset (meshes may be stored in any
                // order); leaf children carry counts, each leaf bounded by its last-in-leaf flag
                const uint64_t e0 = d->meshes[m].bvh_indices_offset;
                if (e0 > d->n_tri_indices) throw std::runtime_error("mesh entry offset out of range");
                collapse_wide(d->bvh_nodes + first, d->n_bvh_nodes - first, 0, wn, nullptr, d->tri_indices + e0,
                              (size_t)(d->n_tri_indices - e0));
                mesh_wide = std::max(mesh_wide, wide_stack_bound(wn.data() + c->h_wbase[m], wn.size() - c->h_wbase[m], 0, kStackMax));
            }
            c->stack_mesh_bin = mesh_bin;
            c->stack_mesh_wide = mesh_wide;
        }
        if (top_tree) {
            c->stack_top_bin = c->stack_top_wide = -1;
            if (d->n_nodes > 0 && d->scene_start_node >= 0) {
                c->stack_top_bin = binary_stack_bound(d->scene_bvh_nodes, d->n_scene_bvh_nodes, d->scene_start_node, kStackMax);
                if (wide) {
                    collapse_wide(d->scene_bvh_nodes, d->n_scene_bvh_nodes, d->scene_start_node, sw);
                    c->stack_top_wide = wide_stack_bound(sw.data(), sw.size(), 0, kStackMax);
                }
            }
        }
    } catch (const std::exception& e) {
        c->err = std::string("scene_upload: ") + e.what();
        return CTL_ERR_INVALID;
    }
    // Worst-case traversal stack for every traversal the scene can take (the
    // 4-wide trees, and the binary trees of stats launches and
    // CTL_SCENE_BINARY_BVH): a scene that could overflow the kStackMax entries
    // of a lane is refused, so no ray can end early on a full stack.  Two
    // levels: top-level stack + the pending top-level entry + the mesh stack.
    {
        int bound = std::max(c->stack_mesh_bin, c->stack_mesh_wide);
        if (c->stack_top_bin >= 0)
            bound = std::max(c->stack_top_bin + 1 + c->stack_mesh_bin,
                             c->stack_top_wide >= 0 ? c->stack_top_wide + 1 + c->stack_mesh_wide : 0);
        if (bound > kStackMax) {
            c->err = "scene_upload: the BVH needs a deeper traversal stack than " + std::to_string(kStackMax) + " entries";
            return CTL_ERR_INVALID;
        }
        c->stack_bound = bound;
    }
    if (wide && (mesh_trees || top_tree)) {
        // 64-B quantized nodes on request (not when the refit will rewrite float nodes)
        const bool quant = (d->flags & CTL_SCENE_WIDE_QUANT) != 0 && !animated;
        auto encode = [](const std::vector<WideNode>& in, std::vector<QWideNode>& out) {
            out.resize(in.size());
            for (size_t i = 0; i < in.size(); i++) {
                const WideNode& w = in[i];
                const float lo[3][4] = {{w.lo_x[0], w.lo_x[1], w.lo_x[2], w.lo_x[3]},
                                        {w.lo_y[0], w.lo_y[1], w.lo_y[2], w.lo_y[3]},
                                        {w.lo_z[0], w.lo_z[1], w.lo_z[2], w.lo_z[3]}};
                const float hi[3][4] = {{w.hi_x[0], w.hi_x[1], w.hi_x[2], w.hi_x[3]},
                                        {w.hi_y[0], w.hi_y[1], w.hi_y[2], w.hi_y[3]},
                                        {w.hi_z[0], w.hi_z[1], w.hi_z[2], w.hi_z[3]}};
                if (!quantize_wide(lo, hi, w.child, out[i])) return false;
            }
            return true;
        };
        std::vector<QWideNode> qn, qs;
        bool q = quant && encode(wn, qn) && encode(sw, qs);
        // host arrays handed to async copies must outlive them
        if (mesh_trees) {
            r = q ? put(c, SA_WBVH, qn.data(), qn.size() * sizeof(QWideNode), 0, s)
                  : put(c, SA_WBVH, wn.data(), wn.size() * sizeof(WideNode), 0, s);
            if (r != CTL_OK) return r;
            if ((r = put(c, SA_WBASE, c->h_wbase.data(), c->h_wbase.size() * 4, 0, s)) != CTL_OK) return r;
            c->wide_nodes = wn.size();
        }
        if (top_tree) {
            r = q ? put(c, SA_SWBVH, qs.data(), qs.size() * sizeof(QWideNode), 0, s)
                  : put(c, SA_SWBVH, sw.data(), sw.size() * sizeof(WideNode), 0, s);
            if (r != CTL_OK) return r;
        }
        S.quant = q ? 1 : 0;
        SD_HIP(c, hipStreamSynchronize(s));   // wn / sw / qn / qs are locals
    }
    if (mesh_trees || top_tree) {
        S.wide = wide ? 1 : 0;
        c->tree_flags = d->flags & tree_bits;
    }
    S.bvh = dptr<float4>(c, SA_BVH);
    S.woop = dptr<float4>(c, SA_WOOP);
    S.tri_idx = dptr<uint32_t>(c, SA_IDX);
    S.tri_data = dptr<ctl_triangle_data>(c, SA_TRI);
    S.mats = dptr<ctl_material>(c, SA_MATS);
    S.meshes = dptr<ctl_kernel_mesh>(c, SA_MESHES);
    S.nodes = dptr<ctl_node>(c, SA_NODES);
    S.scene_bvh = dptr<float4>(c, SA_SBVH);
    S.xf = dptr<float4>(c, SA_XF);
    S.inv_xf = dptr<float4>(c, SA_IXF);
    S.lights = dptr<ctl_light>(c, SA_LIGHTS);
    S.light_tris = dptr<ctl_light_tri>(c, SA_LTRIS);
    S.light_tri_cdf = dptr<float>(c, SA_LCDF);
    S.normal_lut = dptr<float4>(c, SA_LUT);
    S.textures = dptr<ctl_texture>(c, SA_TEX);
    S.tex_data = dptr<uint32_t>(c, SA_TEXDATA);
    S.wbvh = wide ? dptr<float4>(c, SA_WBVH) : nullptr;
    S.scene_wbvh = wide ? dptr<float4>(c, SA_SWBVH) : nullptr;
    S.mesh_wbase = wide ? dptr<uint32_t>(c, SA_WBASE) : nullptr;
    if (dirty & CTL_DIRTY_ENV) {
        S.env_index = d->env_map_index;
        S.env = d->env_map_index != 0xffffffffu ? dptr<ctl_env_light>(c, SA_ENV) : nullptr;
        S.env_data = d->env_map_index != 0xffffffffu ? dptr<float>(c, SA_ENVDATA) : nullptr;
    }
    set_constants(c, d, dirty);
    if (dirty & (CTL_DIRTY_MATERIALS | CTL_DIRTY_ENV)) {
        S.full_shading = kShadeLean;
        S.alpha = 0;
        for (uint32_t i = 0; i < d->n_materials; i++) {
            const ctl_material& m = d->materials[i];
            if (m.bsdf_type != CTL_BSDF_DIFFUSE || m.texture != 0xffffffffu || m.alpha_state) S.full_shading = kShadeFull;
            if (m.alpha_state) S.alpha = 1;   // DynamicScene.cpp:586 doAlphaMapping
        }
        if (S.alpha) S.full_shading = kShadeAlpha;
        if (S.env_index != 0xffffffffu) S.full_shading = kShadeEnv;
    }
    if (dirty & (CTL_DIRTY_NODES | CTL_DIRTY_MESHES | CTL_DIRTY_BVH)) {
        S.n_nodes = d->n_nodes;
        S.start_node = d->scene_start_node;
        S.single = 0;
        if (d->n_nodes > 0 && d->scene_start_node < 0) {
            const uint32_t node = ~(uint32_t)d->scene_start_node;
            if (node >= d->n_nodes) { c->err = "scene_upload: start node out of range"; return CTL_ERR_INVALID; }
            const uint32_t mi = d->nodes[node].mesh_index;
            if (mi >= d->n_meshes) { c->err = "scene_upload: node mesh index out of range"; return CTL_ERR_INVALID; }
            const ctl_kernel_mesh& M = d->meshes[mi];
            S.single = 1;
            S.s_node_base = M.bvh_node_offset;
            S.s_tri_base = M.bvh_triangle_offset;
            S.s_idx_base = M.bvh_indices_offset;
            S.s_tri_offset = M.triangle_offset;
            S.s_wnode_base = S.wide ? c->h_wbase[mi] : 0;
        }
    }
    c->n_tri_data = d->n_tri_data;
    c->n_woop = d->n_woop_tris;
    c->n_bvh_nodes = d->n_bvh_nodes;
    c->n_scene_bvh = d->n_scene_bvh_nodes;
    if (dirty & (kDirtyTrees | CTL_DIRTY_TRI_INDICES | CTL_DIRTY_MESHES)) {
        // instance-tree refit plan (moved nodes) and animated meshes' plans
        int ar = anim_setup(c, d, wn, c->h_wbase, sw);
        if (ar != CTL_OK) return (ctl_status)ar;
        SD_HIP(c, hipStreamSynchronize(s));
    }
    c->n_anim_meshes = d->n_anim_meshes;
    if (dirty & CTL_DIRTY_NODES) c->device_edited = false;
    return CTL_OK;
}

}  // namespace

namespace ctl {
void free_scene(ctl_ctx* c) {
    c->scene_epoch++;
    c->spec.pending = false;
    free_arrays(c);
    anim_free(c);
    c->has_scene = false;
    c->h_wbase.clear();
    c->tree_flags = 0xffffffffu;
    c->device_eps = false;
    c->device_edited = false;
    c->scene = DevScene{};
    c->scene.env_index = 0xffffffffu;
}
}  // namespace ctl

extern "C" {

CTL_API ctl_status ctl_scene_upload(ctl_ctx* c, const ctl_scene_desc* d) {
    if (!c || !d) return CTL_ERR_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "scene_upload: hipSetDevice failed"; return CTL_ERR_HIP; }
    ctl_status r = validate(c, d, CTL_DIRTY_ALL);
    if (r != CTL_OK) return r;
    if (hipDeviceSynchronize() != hipSuccess) { c->err = "scene_upload: device synchronisation failed"; return CTL_ERR_HIP; }
    free_scene(c);
    r = commit(c, d, CTL_DIRTY_ALL, nullptr);
    if (r == CTL_OK && hipStreamSynchronize(nullptr) != hipSuccess) { c->err = "scene_upload: copy failed"; r = CTL_ERR_HIP; }
    if (r != CTL_OK) { std::string e = c->err; free_scene(c); c->err = e; return r; }
    c->has_scene = true;
    return CTL_OK;
}

CTL_API ctl_status ctl_scene_update(ctl_ctx* c, const ctl_scene_desc* d, uint32_t dirty, void* stream) {
    if (!c || !d || (dirty & ~(uint32_t)CTL_DIRTY_ALL)) return CTL_ERR_INVALID;
    if (!c->has_scene) return ctl_scene_upload(c, d);
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "scene_update: hipSetDevice failed"; return CTL_ERR_HIP; }
    if (c->n_anim_meshes != d->n_anim_meshes) dirty = CTL_DIRTY_ALL;
    // refusals that leave the uploaded scene as it was
    ctl_status r = validate(c, d, dirty);
    if (r == CTL_OK) r = check_clean(c, d, dirty);
    if (r != CTL_OK) return r;
    r = commit(c, d, dirty, reinterpret_cast<hipStream_t>(stream));
    if (r != CTL_OK) {   // the device scene may be half updated: drop it
        std::string e = c->err;
        (void)hipDeviceSynchronize();
        free_scene(c);
        c->err = e;
    }
    return r;
}

}  // extern "C"

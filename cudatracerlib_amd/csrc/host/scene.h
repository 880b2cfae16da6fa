// scene.h — host scene compiler: the product-side equivalent of the
// reference's DynamicScene / Mesh::CompileMesh / SceneBVH host code that
// produces the KernelDynamicScene arrays (Engine/DynamicScene.cpp:567-589,
// Engine/Mesh.cpp:199-290, Engine/SceneBVH.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include "../../../include/ctl_trace.h"
#include "../ctl_math.h"

struct ctl_host_scene {
    struct Mesh {
        std::vector<float> v;         // xyz
        std::vector<uint32_t> idx;    // 3 per triangle
        std::vector<float> n;         // per-vertex normals (may be empty)
        std::vector<float> uv;        // per-vertex uv (may be empty)
        std::vector<uint8_t> mat;     // per triangle (may be empty)
        std::vector<ctl_material> materials;
        // compiled mesh loaded from an .xmsh file (xmsh.cpp): the arrays are
        // taken as they are, compile() only relocates them
        bool precompiled = false;
        std::vector<ctl_triangle_data> c_tri;
        std::vector<ctl_bvh_node> c_nodes;
        std::vector<ctl_woop_tri> c_woop;
        std::vector<ctl_tri_index> c_idx;
        float c_box[6] = {0, 0, 0, 0, 0, 0};   // m_sLocalBox minV, maxV
        uint32_t c_depth = 0;
        // MeshPartLight entries resolved to material indices: every node
        // created on the mesh gets these lights (DynamicScene.cpp:340-341)
        struct AutoLight { uint32_t mat; float L[3]; };
        std::vector<AutoLight> auto_lights;
        // skinned mesh (ctl_host_scene_add_animated_mesh): v/n hold the rest pose
        bool animated = false;
        std::vector<ctl_anim_vertex> anim_v;
        uint32_t max_bone = 0;
        uint32_t n_triangles() const { return precompiled ? (uint32_t)c_tri.size() : (uint32_t)(idx.size() / 3); }
    };
    struct Node { uint32_t mesh; bool has_xf; ctl::m44 xf; };
    struct Light { uint32_t node; uint32_t local_mat; float L[3]; };
    std::vector<Mesh> meshes;
    std::vector<Node> nodes;
    std::vector<Light> lights;
    bool has_camera = false;
    float cam_pos[3], cam_tar[3], cam_up[3], cam_fov, cam_near, cam_far;
    uint32_t cam_w = 0, cam_h = 0;
    uint32_t flags = 0;
    // reference splitting of large triangles before the BVH build (ref_split.h)
    float split_alpha = CTL_DEFAULT_SPLIT_ALPHA;
    uint32_t split_depth = CTL_DEFAULT_SPLIT_DEPTH;
    uint32_t sah_bins = CTL_DEFAULT_SAH_BINS;
    uint32_t max_leaf = CTL_DEFAULT_MAX_LEAF;
    uint32_t builder = CTL_BVH_SBVH;   // ctl_host_scene_set_bvh_builder (default: the reference's SBVH)
    float sbvh_alpha = 1.0e-5f;

    // compiled arrays (owned)
    std::vector<ctl_triangle_data> tri_data;
    std::vector<ctl_woop_tri> woop;
    std::vector<ctl_bvh_node> bvh_nodes;
    std::vector<ctl_tri_index> tri_indices;
    std::vector<ctl_material> materials;
    std::vector<ctl_kernel_mesh> kmeshes;
    std::vector<ctl_node> knodes;
    std::vector<ctl_bvh_node> scene_bvh;
    std::vector<ctl_float4x4> xf, inv_xf;
    std::vector<ctl_light> klights;
    // environment (ctl_host_scene_set_environment): InfiniteLight record + its tables
    uint32_t env_texture = 0xffffffffu;
    float env_scale[3] = {1.0f, 1.0f, 1.0f};
    float env_rot[9] = {1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f, 1.0f};   // InfiniteLight::m_worldTransform
    ctl_env_light kenv{};
    std::vector<float> env_tables;
    std::vector<ctl_light_tri> light_tris;
    std::vector<float> light_tri_cdf;
    std::vector<ctl_texture> textures;   // added by ctl_host_scene_add_texture (kept across compiles)
    std::vector<uint32_t> tex_data;
    std::vector<float> kmesh_box;        // 6 floats per mesh: local box of the last compile
    std::vector<ctl_anim_vertex> k_anim_vertices;
    std::vector<uint32_t> k_anim_tris;
    std::vector<ctl_anim_mesh> k_anim_meshes;
    ctl_scene_desc desc{};
    uint32_t max_mesh_depth = 0;
    bool compiled = false;
};

namespace ctl {
// TriIntersectorData::setData (Engine/TriIntersectorData.cu:5-18)
void woop_set(f3 a, f3 b, f3 c, ctl_woop_tri& out);
// TriIntersectorData::getData (Engine/TriIntersectorData.cu:20-32)
void woop_get(const ctl_woop_tri& in, f3& v0, f3& v1, f3& v2);
// PerspectiveSensor::Update + Sensor::SetToWorld(pos, tar, up)
void camera_setup(const float pos[3], const float tar[3], const float up[3], float fov_deg, float nearc, float farc,
                  uint32_t w, uint32_t h, ctl_camera& out);
void set_host_error(const std::string& s);
// adds lights to node `node` (area light of material `local_mat`); replaces
// the radiance when the node already has a light on that material
// (DynamicScene::CreateLight, DynamicScene.cpp:689-711); false + error set
// when a per-node / per-scene limit is hit
bool scene_add_light(ctl_host_scene* s, uint32_t node, uint32_t local_mat, const float L[3]);
}  // namespace ctl

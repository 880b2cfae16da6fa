// xmsh.cpp — the reference's compiled-mesh file (.xmsh), host side.
//   reader: Mesh::Mesh(path, IInStream&, ...) (Engine/Mesh.cpp:46-98) and the
//           area-light step of DynamicScene::CreateNode (DynamicScene.cpp:340-341,
//           CreateLight -> CreateShape name lookup, DynamicScene.cpp:689-734);
//   writer: the byte stream of Mesh::CompileMesh (Mesh.cpp:279-288) followed by
//           ConstructBVH(..., FileOutputStream&) (MeshLoader/BVHBuilderHelper.cpp:129-147).
// The file is packed little-endian:
//   u32 MeshCompileType                    4 B  (0 Static, 1 Animated; MeshCompiler.cpp:94,
//                                               read back in DynamicScene.cpp:313-318)
//   AABB m_sLocalBox                      24 B  (Vec3f minV, Vec3f maxV)
//   u32 n, MeshPartLight[n]               48 B  (FixedString<32> MatName, Spectrum L)
//   u32 n, TriangleData[n]                32 B
//   u32 n, Material[n]                    sizeof(Material): FixedString<64> Name first
//   u64 n, BVHNodeData[n]                 64 B
//   u64 n, TriIntersectorData[n]          48 B
//   u64 n, TriIntersectorData2[n]          4 B
// FixedString<L> = FixedSizeArray<char, L> = {u32 length; char buffer[L]}
// (Base/FixedSizeArray.h:108-109), read back as a C string (FixedString.h:36-39).
//
// A reference Material record is the BSDFALL/Texture variant aggregate of the
// build that wrote the file (vtable slots included), so the reader does not
// decode it: it reads the Name of each record (to resolve the MeshPartLight
// names) and takes the flattened kernel materials from the caller.  Files
// written by ctl_host_scene_write_xmsh carry CTL_XMSH_MATERIAL_RECORD_SIZE-byte
// records (Name + ctl_material) that the reader decodes itself.
#include "scene.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace ctl {
namespace {

constexpr uint32_t kNameLen = 64;          // Material::Name, FixedString<64>
constexpr uint32_t kLightNameLen = 32;     // MeshPartLight::MatName, FixedString<32>
constexpr uint32_t kLightRecord = 4 + kLightNameLen + 12;
constexpr uint32_t kNameRecord = 4 + kNameLen;
constexpr int kMaxDepth = 64;              // traversal stacks of the reference: STACK_SIZE 64
static_assert(CTL_XMSH_MATERIAL_RECORD_SIZE == kNameRecord + sizeof(ctl_material), "record layout");

struct Reader {
    const uint8_t* p;
    uint64_t left;
    bool ok = true;
    bool take(void* dst, uint64_t n) {
        if (!ok || n > left) { ok = false; return false; }
        if (n) memcpy(dst, p, n);
        p += n; left -= n;
        return true;
    }
    template <class T> bool get(T& v) { return take(&v, sizeof(T)); }
    template <class T> bool array(std::vector<T>& v, uint64_t n) {
        if (!ok || n > left / sizeof(T)) { ok = false; return false; }
        v.resize(n);
        return take(v.data(), n * sizeof(T));
    }
};

std::string fixed_string(const uint8_t* rec, uint32_t cap) {
    const char* b = (const char*)rec + 4;
    size_t n = 0;
    while (n < cap && b[n]) n++;
    return std::string(b, n);
}

void put_fixed_string(std::vector<uint8_t>& o, const std::string& str, uint32_t cap) {
    uint32_t n = (uint32_t)std::min<size_t>(str.size(), cap - 1);
    uint32_t len = n + 1;   // FixedString(std::string): chars + the pushed NUL
    const uint8_t* lp = (const uint8_t*)&len;
    o.insert(o.end(), lp, lp + 4);
    size_t at = o.size();
    o.resize(at + cap, 0);
    memcpy(&o[at], str.data(), n);
}

template <class T> void put(std::vector<uint8_t>& o, const T& v) {
    const uint8_t* b = (const uint8_t*)&v;
    o.insert(o.end(), b, b + sizeof(T));
}
template <class T> void put_array(std::vector<uint8_t>& o, const T* v, size_t n) {
    const uint8_t* b = (const uint8_t*)v;
    o.insert(o.end(), b, b + n * sizeof(T));
}

// The arrays index each other with 32-bit values the GPU follows without bound
// checks, so a file is accepted only as a well-formed tree: inner children
// 4*k in range, every inner node reached exactly once from node 0, leaf runs
// ending on a last-in-leaf flag inside the array, triangle indices and
// material bytes in range, depth <= the reference's 64-entry stack.
bool validate(const ctl_host_scene::Mesh& M, uint32_t n_materials, uint32_t& depth_out, std::string& err) {
    const uint64_t nn = M.c_nodes.size(), ne = M.c_idx.size(), nt = M.c_tri.size();
    if (nn == 0) { err = "no BVH nodes"; return false; }
    if (ne != M.c_woop.size()) { err = "TriIntersectorData / TriIntersectorData2 counts differ"; return false; }
    if (nn > 0x1fffffffull || ne > 0x7fffffffull || nt > 0x7fffffffull) { err = "array too large"; return false; }
    for (uint64_t e = 0; e < ne; e++)
        if ((M.c_idx[e] >> 1) >= nt) { err = "triangle index out of range"; return false; }
    for (uint64_t t = 0; t < nt; t++)
        if (((M.c_tri[t].w[1] >> 16) & 0xff) >= n_materials) { err = "material index out of range"; return false; }
    std::vector<uint8_t> seen(nn, 0);
    std::vector<std::pair<uint32_t, int>> stack{{0u, 0}};
    seen[0] = 1;
    uint64_t reached = 1;
    int depth = 0;
    while (!stack.empty()) {
        auto [k, d] = stack.back();
        stack.pop_back();
        depth = std::max(depth, d);
        if (depth > kMaxDepth) { err = "BVH deeper than 64"; return false; }
        const int32_t* ch = (const int32_t*)&M.c_nodes[k] + 12;   // children .x/.y of the 4th float4
        for (int c = 0; c < 2; c++) {
            int32_t v = ch[c];
            if (v == 0x76543210) continue;   // empty child
            if (v >= 0) {
                uint32_t j = (uint32_t)v >> 2;
                if ((v & 3) || j >= nn || seen[j]) { err = "inner child out of range or shared"; return false; }
                seen[j] = 1;
                reached++;
                stack.push_back({j, d + 1});
            } else {
                uint64_t e = (uint32_t)~v;
                while (e < ne && !(M.c_idx[e] & 1)) e++;
                if (e >= ne) { err = "leaf runs past the entry array"; return false; }
            }
        }
    }
    if (reached != nn) { err = "unreachable BVH nodes"; return false; }
    depth_out = (uint32_t)depth;
    return true;
}

}  // namespace
}  // namespace ctl

using namespace ctl;

extern "C" {

CTL_API int32_t ctl_host_scene_add_xmsh(ctl_host_scene* s, const void* data, uint64_t size,
                                        uint32_t material_record_size, const ctl_material* materials,
                                        uint32_t n_materials) {
    auto fail = [](const std::string& m) { set_host_error("add_xmsh: " + m); return -1; };
    if (!s || !data) return fail("invalid arguments");
    if (material_record_size < kNameRecord) return fail("material record smaller than Material::Name");
    if (!materials && material_record_size != CTL_XMSH_MATERIAL_RECORD_SIZE)
        return fail("reference Material records need caller-provided kernel materials");
    Reader r{(const uint8_t*)data, size};
    ctl_host_scene::Mesh M;
    M.precompiled = true;
    uint32_t type = 0xffffffffu;
    r.get(type);
    if (r.ok && type == 1) return fail("animated meshes (MeshCompileType::Animated) are not supported");
    if (r.ok && type != 0) return fail("not an .xmsh stream (unknown MeshCompileType)");
    r.take(M.c_box, 24);
    uint32_t n_lights = 0;
    r.get(n_lights);
    std::vector<uint8_t> lights;
    if (!r.ok || n_lights > r.left / kLightRecord) return fail("truncated (area lights)");
    r.array(lights, (uint64_t)n_lights * kLightRecord);
    uint32_t n_tri = 0;
    r.get(n_tri);
    r.array(M.c_tri, n_tri);
    uint32_t n_mat = 0;
    r.get(n_mat);
    std::vector<uint8_t> recs;
    if (!r.ok || n_mat > r.left / material_record_size) return fail("truncated (materials)");
    r.array(recs, (uint64_t)n_mat * material_record_size);
    uint64_t n_nodes = 0, n_ent = 0, n_ent2 = 0;
    r.get(n_nodes);
    r.array(M.c_nodes, n_nodes);
    r.get(n_ent);
    r.array(M.c_woop, n_ent);
    r.get(n_ent2);
    r.array(M.c_idx, n_ent2);
    if (!r.ok) return fail("truncated stream");
    if (r.left) return fail("trailing bytes after TriIntersectorData2");
    if (n_mat == 0 || n_mat > 255) return fail("need 1..255 materials");
    if (materials && n_materials != n_mat) return fail("material count differs from the file");
    std::vector<std::string> names(n_mat);
    for (uint32_t i = 0; i < n_mat; i++) {
        const uint8_t* rec = &recs[(size_t)i * material_record_size];
        names[i] = fixed_string(rec, kNameLen);
        if (materials) {
            M.materials.push_back(materials[i]);
        } else {
            ctl_material m;
            memcpy(&m, rec + kNameRecord, sizeof(m));
            M.materials.push_back(m);
        }
    }
    std::string err;
    if (!validate(M, n_mat, M.c_depth, err)) return fail(err);
    for (uint32_t i = 0; i < n_lights; i++) {
        const uint8_t* rec = &lights[(size_t)i * kLightRecord];
        std::string name = fixed_string(rec, kLightNameLen);
        auto it = std::find(names.begin(), names.end(), name);
        if (it == names.end()) return fail("Could not find material name in mesh! (" + name + ")");
        ctl_host_scene::Mesh::AutoLight al;
        al.mat = (uint32_t)(it - names.begin());
        memcpy(al.L, rec + 4 + kLightNameLen, 12);
        M.auto_lights.push_back(al);
    }
    if (M.auto_lights.size() > 2) return fail("more than MAX_AREALIGHT_NUM (2) area lights");
    s->meshes.push_back(std::move(M));
    return (int32_t)s->meshes.size() - 1;
}

CTL_API ctl_status ctl_host_scene_write_xmsh(ctl_host_scene* s, uint32_t mesh, void* out, uint64_t capacity,
                                             uint64_t* size) {
    if (!s || !size) return CTL_ERR_INVALID;
    if (!s->compiled || mesh >= s->kmeshes.size()) {
        set_host_error("write_xmsh: compile the scene first (mesh index of the compiled scene)");
        return CTL_ERR_INVALID;
    }
    const ctl_kernel_mesh& km = s->kmeshes[mesh];
    const bool last = mesh + 1 == s->kmeshes.size();
    const uint64_t t0 = km.triangle_offset, t1 = last ? s->tri_data.size() : s->kmeshes[mesh + 1].triangle_offset;
    const uint64_t n0 = km.bvh_node_offset / 4, n1 = last ? s->bvh_nodes.size() : s->kmeshes[mesh + 1].bvh_node_offset / 4;
    const uint64_t e0 = km.bvh_indices_offset, e1 = last ? s->woop.size() : s->kmeshes[mesh + 1].bvh_indices_offset;
    const auto& M = s->meshes[mesh];
    std::vector<uint8_t> o;
    put(o, (uint32_t)0);   // MeshCompileType::Static
    put_array(o, &s->kmesh_box[6 * mesh], 6);
    // MeshPartLight per lit material: the mesh's own entries, then the area
    // lights added on its nodes (CompileMesh's Les, Mesh.cpp:201-206)
    std::vector<std::pair<uint32_t, const float*>> lit;
    for (const auto& al : M.auto_lights) lit.push_back({al.mat, al.L});
    for (const auto& l : s->lights)
        if (s->nodes[l.node].mesh == mesh &&
            std::none_of(lit.begin(), lit.end(), [&](const auto& x) { return x.first == l.local_mat; }))
            lit.push_back({l.local_mat, l.L});
    auto mat_name = [](uint32_t i) { return "material" + std::to_string(i); };
    put(o, (uint32_t)lit.size());
    for (const auto& x : lit) {
        put_fixed_string(o, mat_name(x.first), kLightNameLen);
        put_array(o, x.second, 3);
    }
    put(o, (uint32_t)(t1 - t0));
    put_array(o, s->tri_data.data() + t0, t1 - t0);
    put(o, (uint32_t)M.materials.size());
    for (uint32_t i = 0; i < M.materials.size(); i++) {
        put_fixed_string(o, mat_name(i), kNameLen);
        ctl_material m = M.materials[i];
        m.node_light_index = 0xffffffffu;
        put(o, m);
    }
    put(o, (uint64_t)(n1 - n0));
    put_array(o, s->bvh_nodes.data() + n0, n1 - n0);
    put(o, (uint64_t)(e1 - e0));
    put_array(o, s->woop.data() + e0, e1 - e0);
    put(o, (uint64_t)(e1 - e0));
    put_array(o, s->tri_indices.data() + e0, e1 - e0);
    *size = o.size();
    if (!out) return CTL_OK;   // size query
    if (capacity < o.size()) {
        set_host_error("write_xmsh: buffer too small");
        return CTL_ERR_INVALID;
    }
    memcpy(out, o.data(), o.size());
    return CTL_OK;
}

}  // extern "C"

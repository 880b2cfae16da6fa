/*
 * ctl_trace.h — C-ABI drop-in boundary of the MI355X-native traversal backend.
 *
 * This header is the ONLY contract between a host renderer (the reference's
 * Tracer / KernelDynamicScene / BSDF plugin surface, or our own Python/C++ host
 * code) and the hand-written gfx950 HIP kernels in libctl_trace.so.
 * Plain C, plain pointers and sizes; no torch, no HIP types in the signatures
 * (streams are passed as `void*` = hipStream_t).
 *
 * Citations are `file:line` in the reference (Ilinite/CudaTracerLib).
 *
 *   reference entry point                               replaced by
 *   --------------------------------------------------- --------------------------------
 *   InitializeKernel / DeinitializeKernel               ctl_create / ctl_destroy
 *     Kernel/TraceHelper.h:41-42, TraceHelper.cu:253-272
 *   UpdateKernel(DynamicScene*, ISamplingSeq...&)       ctl_scene_update + ctl_sampler_generate
 *     Kernel/TraceHelper.h:44, TraceHelper.cu:182-217     (first call / full replace: ctl_scene_upload)
 *   DynamicScene::UpdateScene (DynamicScene.cpp:480-554) ctl_scene_update's dirty groups
 *   DynamicScene::SetNodeTransform (:433-443)           ctl_scene_set_transform
 *   __internal__IntersectBuffers(N, rays, res, skip, any_hit)
 *     Kernel/TraceHelper.h:71, TraceHelper.cu:736-746  ctl_intersect
 *   PathTracer::RenderBlock / pathKernel2 per pass      ctl_render_pass
 *     Integrators/PathTracer.cu:182-217, Kernel/Tracer.h:209-248
 *   k_getNumRaysTraced / k_setNumRaysTraced             ctl_rays_traced / ctl_reset_rays
 *     Kernel/TraceHelper.h:52-53, TraceHelper.cu:309-320
 *   ThrowCudaErrors (Defines.cpp:15-29)                 ctl_status + ctl_last_error (never throws)
 *
 * Ownership: the caller owns every host array passed in a ctl_scene_desc (the
 * backend copies and may re-layout them) and every device buffer passed to
 * ctl_intersect / ctl_render_pass (rays, hits, framebuffer).  The context owns
 * its device copy of the scene and sampler tables.  All state is per context
 * (no process globals), so one context per GPU / rank is re-entrant.
 */
#ifndef CTL_TRACE_H
#define CTL_TRACE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CTL_ABI_VERSION 4   /* 2: round 4 (ctl_env_light 112 B, ctl_fb_reduce d_out, wide-tree reads);
                               3: round 5 (ctl_occluded; CTL_SCENE_WIDE8 / CTL_ARRAY_W8_* / ctl_host_w8_tree
                               removed);
                               4: round 6 (CTL_PT_RENDER_AHEAD, CTL_ARRAY_CULL_BOUND; ctl_scene_animate /
                               ctl_scene_set_transform rebuild trees with BVHRebuilder's rotations) */

#if defined(_WIN32)
#define CTL_API __declspec(dllexport)
#else
#define CTL_API __attribute__((visibility("default")))
#endif

typedef int32_t ctl_status;
enum {
    CTL_OK = 0,
    CTL_ERR_INVALID = 1,   /* bad argument / inconsistent scene description  */
    CTL_ERR_HIP = 2,       /* a HIP runtime call failed (see ctl_last_error)  */
    CTL_ERR_NOMEM = 3,     /* device or host allocation failed                */
    CTL_ERR_STATE = 4,     /* call order violated (e.g. render before upload) */
    CTL_ERR_NODEVICE = 5   /* no usable gfx950 device / HIP code object       */
};

/* ------------------------------------------------------------------------ */
/* Byte-identical reference data layouts (static_assert'ed in the sources).  */
/* ------------------------------------------------------------------------ */

/* BVHNodeData, 64 B (Engine/TriIntersectorData.h:42-117):
 *   v[0..3]  = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
 *   v[4..7]  = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
 *   v[8..11] = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
 *   v[12..13]= int child0, child1 : >=0 inner node as float4 offset (=index*4),
 *              <0 leaf (= ~first leaf entry), 0x76543210 = empty/sentinel
 *   v[14]    = parent (uint), v[15] unused                                   */
typedef struct { float v[16]; } ctl_bvh_node;

/* TriIntersectorData, 48 B Woop unit-triangle transform
 * (Engine/TriIntersectorData.h:30-40, setData TriIntersectorData.cu:5-18).   */
typedef struct { float v[12]; } ctl_woop_tri;

/* TriIntersectorData2, 4 B: (local triangle index << 1) | last-in-leaf flag
 * (Engine/TriIntersectorData.h:8-28).                                        */
typedef uint32_t ctl_tri_index;

/* TriangleData (EXT_TRI), 32 B (Engine/TriangleData.h:10-36):
 *   w[0..1] NorMatExtra: 3 x 16-bit spherical normals, u8 material, u8 extra
 *   w[2..4] DpduDpdv   : dpdu, dpdv as 6 x half
 *   w[5..7] UVSets[0]  : 3 x half2 texture coordinates                        */
typedef struct { uint32_t w[8]; } ctl_triangle_data;

/* KernelMesh, 20 B (Engine/Mesh.h:12-19).  bvh_node_offset is in float4 units
 * (Mesh.cpp:104), bvh_triangle_offset in float4 units (= entry*3, Mesh.cpp:105). */
typedef struct {
    uint32_t triangle_offset;
    uint32_t bvh_node_offset;
    uint32_t bvh_triangle_offset;
    uint32_t bvh_indices_offset;
    uint32_t std_material_offset;
} ctl_kernel_mesh;

/* Node, 24 B (SceneTypes/Node.h:13-24; m_uLights is a FixedSizeArray<uint,2>). */
typedef struct {
    uint32_t mesh_index;
    uint32_t material_offset;
    uint32_t instanced_material;
    uint32_t lights[2];
    uint32_t num_lights;
} ctl_node;

/* float4x4, row-major, 64 B (Math/float4x4.h:12-17, idx(i,j) = i*4+j). */
typedef struct { float m[16]; } ctl_float4x4;

/* traversalRay, 32 B (Kernel/TraceHelper.h:55-59): {o.xyz, tmin ; d.xyz, tmax} */
typedef struct { float o[3]; float tmin; float d[3]; float tmax; } ctl_ray;

/* traversalResult, 16 B (Kernel/TraceHelper.h:61-69, written TraceHelper.cu:722-731):
 *   hit : {t, node, tri(global), (v16 << 16) | u16}   miss : {tmax, -1, -1, 0} */
typedef struct { float dist; int32_t node_idx; int32_t tri_idx; int32_t bary; } ctl_hit;

/* PixelData, 28 B (Engine/Image.h:10-29). */
typedef struct { float rgb[3]; float rgb_splat[3]; float weight_sum; } ctl_pixel;

/* ------------------------------------------------------------------------ */
/* Flattened plugin data (the fields of Material / DiffuseLight / Sensor the */
/* path reads; the reference keeps them in CudaVirtualAggregate unions).     */
/* ------------------------------------------------------------------------ */

enum {                        /* BSDF TYPE_FUNC ids (SceneTypes/BSDF_Simple.h) */
    CTL_BSDF_DIFFUSE = 1,         /* diffuse, BSDF_Simple.cu:7-75                  */
    CTL_BSDF_ROUGHDIELECTRIC = 5  /* roughdielectric, BSDF_Simple.cu:373-615        */
};

/* EBSDFType bits used by the path (SceneTypes/Samples.h:32-60). */
enum {
    CTL_EDIFFUSE_REFLECTION = 0x00002,
    CTL_EDIFFUSE_TRANSMISSION = 0x00004,
    CTL_EGLOSSY_REFLECTION = 0x00008,
    CTL_EGLOSSY_TRANSMISSION = 0x00010
};

/* MicrofacetDistribution::EType (Engine/MicrofacetDistribution.h:14-21). */
enum { CTL_MICROFACET_BECKMANN = 0, CTL_MICROFACET_GGX = 1 };

/* Material + the parameters of its BSDF (the reference keeps them in the
 * BSDFALL CudaVirtualAggregate, SceneTypes/BSDF.h:140), 80 B.  Textures other
 * than ConstantTexture are supported for diffuse::m_reflectance only. */
typedef struct {
    uint32_t bsdf_type;          /* CTL_BSDF_*                                   */
    uint32_t combined_type;      /* BSDF::m_combinedType (EBSDFType bits)        */
    uint32_t two_sided;          /* BSDF::m_enableTwoSided                       */
    uint32_t node_light_index;   /* Material::NodeLightIndex, 0xFFFFFFFF = none  */
    float reflectance[3];        /* diffuse: ConstantTexture value of m_reflectance;
                                    roughdielectric: m_specularReflectance       */
    uint32_t texture;            /* diffuse: ImageTexture index of m_reflectance
                                    (0xFFFFFFFF: the constant above)             */
    float transmittance[3];      /* roughdielectric: m_specularTransmittance     */
    uint32_t distribution;       /* roughdielectric: CTL_MICROFACET_*            */
    float eta, inv_eta;          /* roughdielectric: m_eta, m_invEta = 1/m_eta   */
    float alpha_u, alpha_v;      /* ConstantTexture values of m_alphaU / m_alphaV */
    uint32_t sample_visible;     /* m_sampleVisible                              */
    uint32_t alpha_state;        /* Material::AlphaMap.state (AlphaBlendState,
                                    Engine/Material.h:14-22): 0 disabled, 1/2 =
                                    alpha texture luminance/alpha, 5/6 = the
                                    reflectance texture's luminance/alpha    */
    uint32_t alpha_texture;      /* ImageTexture of AlphaMap.tex (states 1, 2)    */
    float alpha_threshold;       /* AlphaMap.test_val_scalar                     */
} ctl_material;

/* ImageTexture (SceneTypes/Texture.h:159-183) with its TextureMapping2D and
 * the KernelMIPMap it samples (Engine/MIPMap_device.h:59-80).  Texels are
 * RGBCOL (r, g, b, a bytes, little-endian uint32) in the scene's tex_data
 * array; level l starts at tex_data[offsets[l]] and is (width >> l) x
 * (height >> l). */
enum { CTL_TEX_POINT = 0, CTL_TEX_BILINEAR = 1, CTL_TEX_EWA = 2, CTL_TEX_TRILINEAR = 3 };   /* ImageFilter */
enum { CTL_WRAP_REPEAT = 0, CTL_WRAP_CLAMP = 1, CTL_WRAP_MIRROR = 2, CTL_WRAP_BLACK = 3 };  /* ImageWrap */
typedef struct {
    float m11, m12, m13, m21, m22, m23;   /* TextureMapping2D                     */
    uint32_t set_id;                      /* must be 0 (one UV set in TriangleData) */
    float scale[3];                       /* ImageTexture::m_scale                */
    uint32_t width, height, levels;       /* KernelMIPMap m_uWidth/m_uHeight/m_uLevels */
    uint32_t filter;                      /* CTL_TEX_*                            */
    uint32_t wrap;                        /* CTL_WRAP_*                           */
    uint32_t offsets[16];                 /* m_sOffsets (MAX_MIPS 16)             */
    float weight_lut[64];                 /* m_weightLut (MTS_MIPMAP_LUT_SIZE 64) */
} ctl_texture;

/* ShapeSet::triData, 64 B (Engine/ShapeSet.h:17-27), world space. */
typedef struct {
    float p[3][3];
    float n[3];
    float area;
    uint32_t i_dat;
    uint32_t t_dat;
    uint32_t pad;
} ctl_light_tri;

/* DiffuseLight (SceneTypes/Light.h:96-143) with a ConstantTexture radiance and
 * its ShapeSet: triangles [tri_first, tri_first+tri_count) of the light_tris
 * array and area CDF entries [cdf_first, cdf_first+tri_count+1).             */
typedef struct {
    float radiance[3];
    uint32_t orthogonal;         /* m_bOrthogonal (must be 0; reserved)          */
    uint32_t tri_first;
    uint32_t tri_count;
    uint32_t cdf_first;
    float sum_area;              /* ShapeSet::sumArea                            */
    uint32_t node_idx;           /* m_uNodeIdx                                   */
    uint32_t kind;               /* CTL_LIGHT_DIFFUSE, or CTL_LIGHT_INFINITE: the
                                    environment (desc.env; other fields unused) */
    uint32_t pad[2];
} ctl_light;
enum { CTL_LIGHT_DIFFUSE = 0, CTL_LIGHT_INFINITE = 1 };

/* InfiniteLight (SceneTypes/Light.h:294-367, Light.cpp:10-58): a latitude-
 * longitude radiance map around the scene.  The radiance map is an image
 * texture (textures[texture], level 0 read; its wrap mode applies to the
 * bilinear lookups); env_data holds the sampling tables the constructor builds:
 * cdf_cols ((width + 1) x height), cdf_rows (height + 1) and row_weights
 * (height) at the given float offsets.  world = the rotation part of
 * m_worldTransform (NormalizedT<OrthogonalAffineMap>, Light.h:307), row-major:
 * directions are mapped world = world * local (TransformDirection) and back
 * with its transpose (TransformDirectionTranspose, Light.cu:342-510); the
 * reference's constructor sets the identity, which ctl_host_scene compiles
 * unless ctl_host_scene_set_environment_transform says otherwise.  Upload
 * refuses a matrix whose rows are not orthonormal. */
typedef struct {
    uint32_t texture;
    float scale[3];              /* m_scale                                      */
    float size[2];               /* m_size = (width, height)                     */
    float pixel_size[2];         /* m_pixelSize = (2 pi / width, pi / height)    */
    float normalization;         /* m_normalization                              */
    float scene_center[3];       /* Update(): scene box centre                   */
    float scene_radius;          /*           |scene box size| / 1.5             */
    uint32_t cdf_cols, cdf_rows, row_weights;
    float world[3][3];           /* m_worldTransform rotation, row-major          */
    uint32_t pad[3];
} ctl_env_light;

/* PerspectiveSensor device state after Update() (SceneTypes/Sensor.cu:76-96). */
typedef struct {
    ctl_float4x4 to_world;          /* SensorBase::toWorld                      */
    ctl_float4x4 sample_to_camera;  /* m_sampleToCamera                         */
    float dx[3];                    /* m_dx                                     */
    float dy[3];                    /* m_dy                                     */
    float inv_resolution[2];        /* m_invResolution                          */
    uint32_t width, height;
} ctl_camera;

#define CTL_MAX_NUM_LIGHTS 16   /* KernelDynamicScene.h:26 */

/* scene flags */
enum {
    /* decode half floats like the reference's HOST path (Math/half.h:72-84,
     * ((h & 0x7fff) << 13) + 0x38000000, i.e. +0 -> 2^-15); off = IEEE decode
     * like its CUDA path (__half2float).  The oracle supports both.          */
    CTL_SCENE_HALF_HOST_QUIRK = 1u << 0,
    /* traverse the uploaded binary BVH in the reference's own (host) visit
     * order: every hit, ties included, is the reference CPU traversal's
     * (BVHTraversal.h:122-232, TraceHelper.cu:88-172).
     * Off (default): the backend collapses each tree into 4-wide 128-B nodes
     * on upload and traverses them in its own per-ray order:
     * deterministic (a function of the ray alone), first-found ties; it can
     * differ from the reference where two triangles tie exactly or a box's
     * rounded entry lies past the hit inside it (counted in DESIGN.md §5).    */
    CTL_SCENE_BINARY_BVH = 1u << 1,
    /* re-encode the 4-wide trees as 64-B nodes with 8-bit child bounds on a
     * per-node power-of-two grid, rounded outward (csrc/ctl_qnode.h): half the
     * node bytes; changes which nodes are visited, never which triangle is hit.
     * Off (default): 128-B float nodes, measured faster on MI355X.
     * Ignored for scenes with animated meshes (the refit writes float nodes). */
    CTL_SCENE_WIDE_QUANT = 1u << 2
    /* 1u << 3 is reserved: ABI v2's 8-wide compressed tree (CTL_SCENE_WIDE8),
     * measured 18 % slower on C3 and kept as probes/round4_variants.patch; v3 ignores
     * the bit. */
};

/* AnimatedVertex (Engine/AnimatedMesh.h:10-22), 40 B: rest position and
 * normal, 8 bone indices (u8 each, low byte first) and 8 weights (u8, w/255). */
typedef struct {
    float pos[3];
    float normal[3];
    uint64_t bone_indices;
    uint64_t bone_weights;
} ctl_anim_vertex;

/* One animated (skinned) mesh of a compiled scene (e_KernelAnimatedMesh,
 * AnimatedMesh.h:57-67): its vertices are anim_vertices[vertex_first ..
 * +vertex_count), its triangles' vertex indices (local to the mesh)
 * anim_triangles[3*tri_first .. 3*(tri_first+tri_count)). */
typedef struct {
    uint32_t mesh;           /* index into meshes[]                  */
    uint32_t vertex_first, vertex_count;
    uint32_t tri_first, tri_count;
    uint32_t max_bone;       /* largest bone index any vertex uses   */
} ctl_anim_mesh;

/* Everything KernelDynamicScene (Engine/KernelDynamicScene.h:28-57) holds that
 * the traversal + PathTracer path reads. */
typedef struct {
    const ctl_triangle_data* tri_data;  uint64_t n_tri_data;    /* m_sTriData    */
    const ctl_woop_tri* woop_tris;      uint64_t n_woop_tris;   /* m_sBVHIntData */
    const ctl_bvh_node* bvh_nodes;      uint64_t n_bvh_nodes;   /* m_sBVHNodeData */
    const ctl_tri_index* tri_indices;   uint64_t n_tri_indices; /* m_sBVHIndexData */
    const ctl_material* materials;      uint32_t n_materials;   /* m_sMatData    */
    const ctl_kernel_mesh* meshes;      uint32_t n_meshes;      /* m_sMeshData   */
    const ctl_node* nodes;              uint32_t n_nodes;       /* m_sNodeData   */
    /* KernelSceneBVH (Engine/SceneBVH_device.h:8-15) */
    const ctl_bvh_node* scene_bvh_nodes; uint32_t n_scene_bvh_nodes;
    int32_t scene_start_node;           /* m_sStartNode (<0: single leaf ~node) */
    const ctl_float4x4* node_xf;        /* m_pNodeTransforms[n_nodes]           */
    const ctl_float4x4* node_inv_xf;    /* m_pInvNodeTransforms[n_nodes]        */
    /* lights (m_sLightBuf + ShapeSet data held in m_sAnimData) */
    const ctl_light* lights;            uint32_t n_lights;
    const ctl_light_tri* light_tris;    uint32_t n_light_tris;
    const float* light_tri_cdf;         uint32_t n_light_tri_cdf;
    float light_cdf[CTL_MAX_NUM_LIGHTS];/* m_pLightCDF (lights are active, identity index map) */
    /* m_sTexData: image textures and their texel data */
    const ctl_texture* textures;        uint32_t n_textures;
    const uint32_t* tex_data;           uint64_t n_tex_data;
    uint32_t env_map_index;             /* m_uEnvMapIndex: the CTL_LIGHT_INFINITE light, 0xFFFFFFFF: none */
    const ctl_env_light* env;           /* that light's record (NULL without one) */
    const float* env_data;              uint64_t n_env_data;   /* its sampling tables */
    float box_min[3], box_max[3];       /* m_sBox                               */
    float ray_eps;                      /* m_rayTraceEps, DynamicScene.cpp:587  */
    ctl_camera camera;                  /* m_Camera                             */
    uint32_t flags;                     /* CTL_SCENE_*                          */
    /* Mesh::m_sLocalBox per mesh (6 floats: min xyz, max xyz): the instance
     * boxes of the scene BVH are these boxes transformed (SceneBVH.cpp:77-100) */
    const float* mesh_boxes;
    /* animated meshes (AnimatedMesh::k_ComputeState input, AnimatedMesh.cpp:163-184) */
    const ctl_anim_vertex* anim_vertices; uint32_t n_anim_vertices;
    const uint32_t* anim_triangles;     uint32_t n_anim_triangles;   /* 3 indices each */
    const ctl_anim_mesh* anim_meshes;   uint32_t n_anim_meshes;
} ctl_scene_desc;

/* PathTracer parameters (Integrators/PathTracer.h:10-19) + multi-GPU tiling. */
typedef struct {
    int32_t direct;            /* KEY_Direct, default 1                       */
    int32_t max_path_length;   /* KEY_MaxPathLength, default 50               */
    int32_t rr_start_depth;    /* KEY_RRStartDepth, default 5                 */
    int32_t shadow_any_hit;    /* 1: Occluded() as any-hit over (eps,tmax-eps)
                                  (identical boolean, KernelDynamicScene.cu:70-80);
                                  0: closest-hit like the reference           */
    uint32_t tile_size;        /* image tile edge (64 = BLOCK_SAMPLER_BlockSize) */
    uint32_t num_ranks;        /* tiles with (tile_id % num_ranks) == rank are */
    uint32_t rank;             /*   rendered by this call                      */
    uint32_t flags;            /* CTL_PT_*                                     */
} ctl_pt_params;

enum {
    /* Pass schedules; all three give bit-identical framebuffers.
     * default (0): persistent path kernel with path regeneration
     * CTL_PT_MEGAKERNEL: one thread per pixel path (pathKernel2's launch shape)
     * CTL_PT_WAVEFRONT: wavefront pipeline (gen / trace / shade / shadow /
     *                   resolve kernels per bounce over compacted queues)   */
    CTL_PT_MEGAKERNEL = 1u << 0,
    CTL_PT_WAVEFRONT = 1u << 1,
    /* ctl_render_pass may render ahead (persistent schedule only): once the
     * calls follow each other with consecutive ctl_sampler_generate passes and
     * nothing changing (scene, tables, parameters, framebuffer, stream), a call
     * renders a window of the next 2, 4, then 8 passes in one launch and folds
     * its own; the next calls of the window only fold theirs.  The
     * framebuffer after each call is bit-identical to one pass per call; a
     * change drops the pending passes.  ctl_rays_traced counts a window's
     * rays when it is launched (rays of dropped passes included).            */
    CTL_PT_RENDER_AHEAD = 1u << 2
};

/* ------------------------------------------------------------------------ */
/* Device API (needs a gfx950 GPU)                                           */
/* ------------------------------------------------------------------------ */

typedef struct ctl_ctx ctl_ctx;

CTL_API int32_t ctl_abi_version(void);
/* Creates a context bound to HIP device `device`.  Returns NULL on failure;
 * the reason is then available from ctl_last_error(NULL). */
CTL_API ctl_ctx* ctl_create(int32_t device);
CTL_API void ctl_destroy(ctl_ctx* ctx);
/* Last error message of ctx (or of the last failed ctl_create when ctx==NULL). */
CTL_API const char* ctl_last_error(const ctl_ctx* ctx);

/* Copies the scene to the device (synchronous).  Replaces any previous scene. */
CTL_API ctl_status ctl_scene_upload(ctl_ctx* ctx, const ctl_scene_desc* desc);

/* The arrays of a ctl_scene_desc grouped as the reference's DynamicScene
 * streams that UpdateScene re-uploads when invalidated
 * (Engine/DynamicScene.cpp:480-554, Base/Buffer.h:257-291). */
enum {
    CTL_DIRTY_TRI_DATA = 1u << 0,     /* tri_data        (m_pTriDataStream)          */
    CTL_DIRTY_WOOP = 1u << 1,         /* woop_tris       (m_pTriIntStream)           */
    CTL_DIRTY_BVH = 1u << 2,          /* bvh_nodes       (m_pBVHStream); the 4-wide  */
                                      /*   mesh trees are rebuilt from them           */
    CTL_DIRTY_TRI_INDICES = 1u << 3,  /* tri_indices     (m_pBVHIndicesStream)       */
    CTL_DIRTY_MATERIALS = 1u << 4,    /* materials       (m_pMaterialBuffer)         */
    CTL_DIRTY_MESHES = 1u << 5,       /* meshes + mesh_boxes (m_pMeshBuffer)         */
    CTL_DIRTY_NODES = 1u << 6,        /* nodes, node_xf / node_inv_xf, scene_bvh_nodes,
                                         scene_start_node (m_pNodeStream + SceneBVH) */
    CTL_DIRTY_LIGHTS = 1u << 7,       /* lights, light_tris, light_tri_cdf
                                         (m_pLightStream + the ShapeSet data)        */
    CTL_DIRTY_TEXTURES = 1u << 8,     /* textures, tex_data (m_pTextureBuffer)       */
    CTL_DIRTY_ENV = 1u << 9,          /* env_map_index, env, env_data                */
    CTL_DIRTY_ALL = (1u << 10) - 1u
};

/* UpdateKernel(DynamicScene*) (Kernel/TraceHelper.cu:182-217), called by the
 * reference at the start of every Tracer::DoPass (Kernel/Tracer.h:229), plus
 * the incremental DynamicScene::UpdateScene.  Refreshes the scene constants
 * every time (camera, ray_eps, box, light_cdf, flags: KernelDynamicScene's
 * non-array members) and copies only the array groups in `dirty` (CTL_DIRTY_*),
 * stream-ordered on `stream`; clean arrays must keep their counts (else
 * CTL_ERR_INVALID, the uploaded scene unchanged).  With dirty = 0 it costs no
 * copy and no device synchronisation.  An array whose size grows is
 * reallocated after the device drains; a dirty tree array rebuilds the 4-wide
 * copies on the host.  ray_eps: after ctl_scene_set_transform or
 * ctl_scene_animate the device's own epsilon (from the moved scene box) stays
 * until the instances are uploaded again (CTL_DIRTY_NODES).  Those two calls
 * edit device arrays only: marking such an array dirty uploads the desc's
 * version again, and after them any tree group (BVH, TRI_INDICES, MESHES,
 * NODES) re-uploads every array they edit (TRI_DATA, WOOP, BVH, NODES,
 * LIGHTS, ENV), so geometry, instances, lights and the environment's scene
 * sphere all return to the desc together.  Without an uploaded scene this is ctl_scene_upload. */
CTL_API ctl_status ctl_scene_update(ctl_ctx* ctx, const ctl_scene_desc* desc, uint32_t dirty, void* stream);

/* DynamicScene::SetNodeTransform (Engine/DynamicScene.cpp:433-443) +
 * SceneBVH::setTransform (Engine/SceneBVH.cpp:77-89) on the device: writes the
 * node's object->world transform (row-major 4x4) and its inverse
 * (float4x4::inverse, computed on the host as the reference does), recomputes
 * the ShapeSet of every area light on the node (RecomputeShape,
 * ShapeSet.cpp:39-57: world triangles, normals, areas, CDF, sumArea), refits
 * the instance boxes and the scene BVH (binary and 4-wide; the reference's
 * BVHRebuilder also rotates the tree, which traversal does not observe), and
 * derives the scene box, ray epsilon (DynamicScene.cpp:583-587) and the
 * environment light's scene sphere (InfiniteLight::Update) from it.
 * Synchronises `stream` once (the epsilon is a kernel argument).  The caller's
 * desc is not changed. */
CTL_API ctl_status ctl_scene_set_transform(ctl_ctx* ctx, uint32_t node, const ctl_float4x4* xf, void* stream);

/* Generates the SequenceSamplerData tables of render pass `pass_index` (the
 * pass-th UpdateKernel call, Kernel/Sampler.h:36-55 + 63-85) on the device,
 * asynchronously on `stream` (double-buffered; safe to call while the
 * previous pass still renders).  num_sequences=4096, length=30 as
 * InitializeKernel (TraceHelper.cu:253-257).  Replaces the host generation in
 * UpdateKernel (TraceHelper.cu:182-217). */
CTL_API ctl_status ctl_sampler_generate(ctl_ctx* ctx, uint64_t pass_index, void* stream);
/* Uploads caller-provided tables instead (element-major: [k*num_seq + s]). */
CTL_API ctl_status ctl_sampler_upload(ctl_ctx* ctx, const float* seq1d, const float* seq2d,
                                      uint32_t num_sequences, uint32_t sequence_length, void* stream);

/* Batched closest/any-hit over device buffers; asynchronous on `stream`.
 * Semantics of intersectKernel<ANY_HIT> (TraceHelper.cu:326-734): triangle
 * accepted when tmin < t < current tmax, result layout as ctl_hit. */
CTL_API ctl_status ctl_intersect(ctl_ctx* ctx, int64_t n, const ctl_ray* d_rays, ctl_hit* d_hits,
                                 int32_t any_hit, void* stream);

/* Batched KernelDynamicScene::Occluded(Ray(o, d), 0, tmax)
 * (Engine/KernelDynamicScene.cu:70-80), the shadow test EstimateDirect makes
 * (Kernel/TraceAlgorithms.cu:55), over device buffers; asynchronous on `stream`.
 * Per ray: tmax = d_rays[i].tmax (the light distance), tmin (o.w) ignored;
 * d_out[i] = 1 when occluded.  any_hit = 0: the reference's form, a closest-hit
 * traceRay and eps < t < tmax - eps (a miss with tmax = inf is not occluded);
 * any_hit = 1: the query ctl_pt_params.shadow_any_hit = 1 runs in the path
 * kernels, any hit with eps < t < tmax - eps, boxes culled at tmax +
 * slab_slack(ray) (traverse.h: a per-ray bound on the slab rounding).  traceRay's
 * traversal (span tmin 0, the alpha test in scenes with alpha maps) in the
 * scene's tree order (CTL_SCENE_BINARY_BVH: the reference's).  Counts n rays
 * (each Occluded is one traceRay).  How often the two forms disagree is
 * measured in tests/test_shadow_query.py and DESIGN.md §5. */
CTL_API ctl_status ctl_occluded(ctl_ctx* ctx, int64_t n, const ctl_ray* d_rays, uint32_t* d_out, int32_t any_hit,
                                void* stream);

/* One progressive PathTracer pass (one sample per owned pixel) accumulated
 * into the caller's device framebuffer d_fb[width*height] (PixelData,
 * Engine/Image.cu:22-44).  Uses the tables from the last ctl_sampler_generate /
 * ctl_sampler_upload on the same stream.  Asynchronous on `stream`.  The
 * samples go through per-context slots and are added to d_fb in image order
 * (see DESIGN.md §5), so the passes of one context belong on one stream. */
CTL_API ctl_status ctl_render_pass(ctl_ctx* ctx, const ctl_pt_params* params, ctl_pixel* d_fb,
                                   void* stream);

/* n_passes consecutive passes first_pass .. first_pass + n_passes - 1 in one
 * launch: the same framebuffer as n_passes rounds of ctl_sampler_generate +
 * ctl_render_pass (Tracer::DoPass called n times, Kernel/Tracer.h:209-248),
 * with the sampler tables generated inside.  Each pass's samples land in a
 * per-pass slice of the owned tiles that is folded into d_fb in pass order, so
 * a rank owning 1/N of the image keeps the resident grid as busy as a
 * full-image pass.  Asynchronous on `stream`; ctl_last_pass_ms covers the call. */
CTL_API ctl_status ctl_render_passes(ctl_ctx* ctx, const ctl_pt_params* params, uint64_t first_pass,
                                     uint32_t n_passes, ctl_pixel* d_fb, void* stream);

/* Device time of the last ctl_render_pass on its stream, in milliseconds
 * (Tracer::getLastTimeSpentRenderingSec, Kernel/Tracer.h:133-140, which times
 * DoPass with cudaEvents, Tracer.h:213,239-244).  Waits for that pass. */
CTL_API ctl_status ctl_last_pass_ms(ctl_ctx* ctx, float* ms);

/* The primary rays of a pass (what ctl_render_pass traces first: pixel jitter,
 * aperture draw, PerspectiveSensor::sampleRayDifferential, Sensor.cu:130-144)
 * as a traversalRay batch in work order, for ctl_intersect - the camera stage
 * of the reference's batch tracers (DoubleRayBuffer callers).  Work items
 * outside the image get tmax = 0.  *n_out = number of rays (owned tiles x
 * tile_size^2); d_rays must hold that many (query with capacity 0). */
CTL_API ctl_status ctl_camera_rays(ctl_ctx* ctx, const ctl_pt_params* params, ctl_ray* d_rays, int64_t capacity,
                                   int64_t* n_out, void* stream);

/* ---- multi-GPU: tile shards + one PixelData reduce over RCCL --
 * The reference renders on one GPU (Tracer<true>::DoPass accumulating into
 * PixelData, Kernel/Tracer.h:209-248, Engine/Image.h:10-29).  Rank r of N
 * renders the tiles with tile_id % N == r (ctl_pt_params.num_ranks / rank);
 * its framebuffer holds exactly the owned pixels' sums, in the 1-GPU order
 * (samples that round over a tile border are traced by the target's owner),
 * so one sum-reduce of the N framebuffers is the 1-GPU framebuffer bit for
 * bit.  A communicator is an RCCL ncclComm_t passed as void*: the caller's own
 * or one made by these helpers. */
#define CTL_COMM_ID_BYTES 128u   /* sizeof(ncclUniqueId) */
/* ncclGetUniqueId: one rank calls it and hands the bytes to the others. */
CTL_API ctl_status ctl_comm_unique_id(void* id_out);
/* ncclCommInitRank on `device` (one process per GPU). */
CTL_API ctl_status ctl_comm_init_rank(void** comm_out, int32_t nranks, const void* id, int32_t rank,
                                      int32_t device);
/* ncclCommInitAll: one process driving ndev GPUs; comms_out[i] is rank i on devices[i]. */
CTL_API ctl_status ctl_comm_init_all(void** comms_out, int32_t ndev, const int32_t* devices);
CTL_API ctl_status ctl_comm_destroy(void* comm);
/* Sum the n_pixels PixelData records of every rank's d_fb into d_out on the
 * root (ncclReduce, fp32 sum).  d_fb is only read: each rank keeps
 * accumulating its own pixels into it, so the reduce may run after any step and
 * any number of times (d_out then holds the image of all passes so far; it must
 * not alias d_fb; it is required on the root and ignored on the other ranks: a
 * NULL d_out is CTL_ERR_INVALID where the rank reads as the root through
 * ncclCommUserRank, and passed to RCCL otherwise, so a rank whose number cannot
 * be read never drops out of the collective).  Every rank calls it with
 * its own ctx and stream; asynchronous on `stream`.  RCCL is loaded on first
 * use (CTL_ERR_NODEVICE when it cannot be). */
CTL_API ctl_status ctl_fb_reduce(ctl_ctx* ctx, void* comm, const ctl_pixel* d_fb, ctl_pixel* d_out,
                                 uint64_t n_pixels, int32_t root, void* stream);
/* The same for n contexts of one process (one per GPU, communicators from
 * ctl_comm_init_all), as one grouped RCCL call; d_out lives on ctxs[root]'s GPU. */
CTL_API ctl_status ctl_fb_reduce_all(ctl_ctx* const* ctxs, void* const* comms, const ctl_pixel* const* d_fbs,
                                     ctl_pixel* d_out, int32_t n, uint64_t n_pixels, int32_t root,
                                     void* const* streams);

/* ---- animated meshes: skinning + BVH refit ------------ */

/* AnimatedMesh::k_ComputeState (Engine/AnimatedMesh.cpp:163-184) for animated
 * mesh `anim` (index into desc->anim_meshes) of the uploaded scene, on the
 * device: skins every vertex between bone matrices frame0 and frame1
 * (g_ComputeVertices, AnimatedMesh.cu:29-43; n_bones row-major float4x4 each,
 * host memory), rewrites its TriangleData (g_ComputeTriangles ->
 * TriangleData::setData) and TriIntersectorData (AnimProvider::setObject,
 * AnimatedMesh.cpp:113-117), refits its BVH boxes bottom-up, then the
 * instance boxes and the scene BVH, and recomputes the ray epsilon from the
 * new scene box (DynamicScene.cpp:587).  The refit keeps the compiled tree
 * (the reference's BVHRebuilder also rotates subtrees, BVHRebuilder.cpp:281-340;
 * traversal results do not depend on the tree).  Synchronises `stream` once
 * (the epsilon is a host-side kernel argument). */
CTL_API ctl_status ctl_scene_animate(ctl_ctx* ctx, uint32_t anim, const ctl_float4x4* frame0,
                                     const ctl_float4x4* frame1, uint32_t n_bones, float lerp, void* stream);

/* Copies `count` elements from element `first` of a device scene array to
 * host memory (Stream<T>::CopyFromDevice, e.g. AnimatedMesh.cpp:178), for
 * inspecting what ctl_scene_animate wrote.  Synchronous. */
enum {
    CTL_ARRAY_TRI_DATA = 0,    /* ctl_triangle_data   */
    CTL_ARRAY_WOOP = 1,        /* ctl_woop_tri        */
    CTL_ARRAY_BVH_NODES = 2,   /* ctl_bvh_node        */
    CTL_ARRAY_SCENE_BVH = 3,   /* ctl_bvh_node        */
    CTL_ARRAY_MESH_BOXES = 4,  /* 6 floats per mesh   */
    CTL_ARRAY_RAY_EPS = 5,     /* 1 float             */
    CTL_ARRAY_SAMPLES_1D = 6,  /* float, element-major [len][num_sequences]: the tables of the last
                                  ctl_sampler_generate / ctl_sampler_upload */
    CTL_ARRAY_SAMPLES_2D = 7,  /* float2, same layout */
    CTL_ARRAY_NODE_XF = 8,     /* ctl_float4x4 per node */
    CTL_ARRAY_NODE_INV_XF = 9, /* ctl_float4x4 per node */
    CTL_ARRAY_LIGHTS = 10,     /* ctl_light           */
    CTL_ARRAY_LIGHT_TRIS = 11, /* ctl_light_tri       */
    CTL_ARRAY_LIGHT_CDF = 12,  /* float               */
    CTL_ARRAY_SCENE_BOX = 13,  /* 6 floats: min xyz, max xyz (after set_transform / animate) */
    CTL_ARRAY_ENV = 14,        /* ctl_env_light       */
    /* the 4-wide trees the default traversal walks (CTL_ERR_STATE under
     * CTL_SCENE_BINARY_BVH): 128-B nodes {lo_x, hi_x, lo_y, hi_y, lo_z, hi_z}
     * float[4] each + int32 child[4] + pad[4] (64-B quantized nodes under
     * CTL_SCENE_WIDE_QUANT, csrc/ctl_qnode.h); child >= 0 a node of the same
     * tree, < 0 a leaf (mesh trees: ~((first entry << 3) | count 1..7, 0 = 8 or
     * more); instance tree: ~node), 0x76543210 an empty slot.                */
    CTL_ARRAY_WIDE_BVH = 15,       /* all mesh trees                          */
    CTL_ARRAY_SCENE_WIDE_BVH = 16, /* the instance tree (root at node 0)      */
    CTL_ARRAY_MESH_WIDE_BASE = 17, /* uint32 per mesh: its tree's first node  */
    /* 3 floats: per axis, the bound on every box coordinate the any-hit shadow
     * query's cull slack uses (DevScene::cull_m, traverse.h slab_slack): the
     * scene box and mesh boxes of the desc, and of the device after
     * set_transform / animate (an animated mesh's boxes are kept in it until
     * its tree is uploaded again).                                           */
    CTL_ARRAY_CULL_BOUND = 18
};
CTL_API ctl_status ctl_scene_read(ctl_ctx* ctx, uint32_t array, uint64_t first, uint64_t count, void* host_dst);

/* ---- PrimTracer (BASELINE config C1) ------------------------------------- */

/* PathTrace_DrawMode (Integrators/PrimTracer.h:7-9), in the reference's order. */
enum {
    CTL_PRIM_LINEAR_DEPTH = 0, CTL_PRIM_D3D_DEPTH = 1, CTL_PRIM_V_ABSDOT_N_GEO = 2, CTL_PRIM_V_DOT_N_GEO = 3,
    CTL_PRIM_V_DOT_N_SHADE = 4, CTL_PRIM_N_GEO_COLORED = 5, CTL_PRIM_N_SHADE_COLORED = 6, CTL_PRIM_UV = 7,
    CTL_PRIM_BARY_COORDS = 8, CTL_PRIM_FIRST_LE = 9, CTL_PRIM_FIRST_F = 10, CTL_PRIM_FIRST_F_DIRECT = 11,
    CTL_PRIM_FIRST_NON_DELTA_LE = 12, CTL_PRIM_FIRST_NON_DELTA_F = 13, CTL_PRIM_FIRST_NON_DELTA_F_DIRECT = 14
};

/* PrimTracer parameters (PrimTracer.h:15-16, defaults PrimTracer.cu:246-247). */
typedef struct {
    int32_t draw_mode;         /* KEY_DrawingMode, default CTL_PRIM_FIRST_F        */
    int32_t max_path_length;   /* KEY_MaxPathLength, default 7 (the first_non_delta_* */
                               /* walk through delta BSDFs; the supported BSDFs     */
                               /* have none, so it is never taken)                 */
    float near_depth;          /* the sensor's m_fNearFarDepths (Sensor.h:46), for  */
    float far_depth;           /* the depth modes and the depth image              */
    uint32_t flags;            /* reserved, 0                                      */
} ctl_prim_params;

/* PrimTracer::DoRender (Integrators/PrimTracer.cu:214-233) as Tracer<false>::DoPass
 * runs it: clears d_fb (Image::Clear), then one primary ray per pixel through
 * the pixel corner (PrimTracer.cu:22) and the draw mode's first-hit value
 * (computePixel, :19-106) into the pixel's PixelData.  d_depth (optional,
 * width*height floats) receives DeviceDepthImage::NormalizeDepthD3D of the
 * hit distance (g_DepthImage2.Store, :104-105).  Uses the sampler tables of the
 * last ctl_sampler_generate.  Asynchronous; ctl_last_pass_ms times it. */
CTL_API ctl_status ctl_prim_pass(ctl_ctx* ctx, const ctl_prim_params* params, ctl_pixel* d_fb, float* d_depth,
                                 void* stream);

/* ---- WavefrontPathTracer over a DoubleRayBuffer -------- */

/* WavefrontPathTracer parameters (Integrators/PseudoRealtime/WavefrontPathTracer.h:27-38). */
typedef struct {
    int32_t direct;            /* KEY_Direct, default 1                          */
    int32_t max_path_length;   /* KEY_MaxPathLength, default 50                  */
    int32_t rr_start_depth;    /* KEY_RRStartDepth, default 5                    */
    uint32_t passes_done;      /* Tracer::m_uPassesDone inside this DoRender: 1  */
                               /* for the first pass of a trace (Tracer.h:231)   */
    uint32_t flags;            /* CTL_WPT_* below, else 0                        */
} ctl_wpt_params;

/* ctl_wpt_params.flags.  CTL_WPT_SHADOW_ANY_HIT: trace the secondary (shadow)
 * rays as the any-hit query over (eps, dist (1 - eps)), boxes culled at that
 * bound + slab_slack(ray) (the path tracer's shadow_any_hit query),
 * instead of the reference's closest hit and distance compare
 * (WavefrontPathTracer.cu:58-63).  The visibility is the same wherever the
 * slab slack bounds the rounding (measured: tests/test_gpu_parity.py); the
 * default (0) is the reference's query. */
enum { CTL_WPT_SHADOW_ANY_HIT = 1u << 0 };

/* One WavefrontPathTracer::DoRender (WavefrontPathTracer.cu:152-189) into
 * d_fb[width*height]: pathCreateKernelWPT (one camera ray per pixel, the
 * uniform block sampler's single sample), then per bounce the
 * DoubleRayBuffer::FinishIteration batch traversals (payload rays closest-hit,
 * the previous bounce's shadow rays closest-hit, DoubleRayBuffer.h:84-112) and
 * pathIterateKernel<Direct> (WavefrontPathTracer.cu:51-150), until the buffer
 * is empty or MaxPathLength bounces.  Payload and shadow-ray slots are assigned
 * in fetch order (a stable compaction), so the image is the reference's under
 * the sequential schedule of its insertion atomics, and deterministic.  Uses
 * the sampler tables of the last ctl_sampler_generate.  Synchronises `stream`
 * once per bounce (the host reads the queue lengths, as the reference's
 * CopyFromSymbol does).  Rays counted by ctl_rays_traced: every traversal of
 * the batch (the reference's counter only counts traceRay, so it reports 0). */
CTL_API ctl_status ctl_wpt_render_pass(ctl_ctx* ctx, const ctl_wpt_params* params, ctl_pixel* d_fb, void* stream);

/* ---- final-image stage -------------------------------------- */

/* PixelVarianceInfo (Kernel/PixelVarianceBuffer.h:10-63), 44 B. */
typedef struct {
    float prev_I[3];          /* Spectrum prev_I                                */
    float half_buffer[3];     /* Spectrum half_buffer                           */
    int32_t iterations_done;
    float weight;
    float sum_x, sum_x2;      /* VarAccumulator<float> I                        */
    int32_t num_samples_var;
} ctl_pixel_variance;

/* applyImagePipeline without filter or post-process (ImagePipeline.cu:57-65):
 * copySamplesToOutput, d_rgba[y*w+x] = gammaCorrecture(PixelData::toSpectrum(
 * splat_scale)) as RGBCOL (r in the low byte, a = 255).  Asynchronous. */
CTL_API ctl_status ctl_image_resolve(ctl_ctx* ctx, const ctl_pixel* d_fb, uint32_t width, uint32_t height,
                                     float splat_scale, uint32_t* d_rgba, void* stream);

/* PixelVarianceBuffer::AddPass (PixelVarianceBuffer.cu:10-37): updates the
 * moments of every pixel of the tiles sampled in this pass.  tile_samples
 * (host, one byte per tile_size^2 block, row-major over ceil(w/tile_size) x
 * ceil(h/tile_size); the reference's BLOCK_SAMPLER_BlockSize is 64 or 128,
 * IBlockSampler_device.h:6-19) is the block-flag array: how many samples the
 * pass put into each block (0 = not rendered, its pixels untouched).  d_var
 * holds width*height records, zero-initialised by the caller before the first
 * pass.  Asynchronous. */
CTL_API ctl_status ctl_variance_add_pass(ctl_ctx* ctx, const ctl_pixel* d_fb, uint32_t width, uint32_t height,
                                         float splat_scale, uint32_t tile_size, const uint8_t* tile_samples,
                                         ctl_pixel_variance* d_var, void* stream);

/* PixelVarianceInfo::computeError / computeVariance / computeAverage
 * (PixelVarianceBuffer.h:43-62) for n records; any output may be NULL. */
CTL_API ctl_status ctl_variance_stats(ctl_ctx* ctx, const ctl_pixel_variance* d_var, uint64_t n, float* d_error,
                                      float* d_variance, float* d_average, void* stream);

/* Number of traceRay-equivalent queries (camera + bounce + shadow rays +
 * batched rays) since the last reset; 64-bit (the reference's counter is a
 * 32-bit atomicInc, Base/Platform.cu:12-21).  Synchronises the device. */
CTL_API uint64_t ctl_rays_traced(ctl_ctx* ctx);
/* Zeroes the ray counter and clears a recorded traversal stack overflow. */
CTL_API ctl_status ctl_reset_rays(ctl_ctx* ctx, void* stream);
/* The ABI's sync point (the reference's cudaDeviceSynchronize after a pass,
 * Tracer.h:240, TraceHelper.cu:744): waits for the stream, then returns
 * CTL_ERR_STATE if any traversal since the last ctl_reset_rays overflowed its
 * stack (the ray's result is then invalid; the reference would have written
 * past its int[64] local stack, BVHTraversal.h:14).  The overflow is sticky:
 * render / intersect calls return CTL_ERR_STATE until ctl_reset_rays.  Scene
 * upload already refuses a BVH whose worst-case stack could overflow, so this
 * is a second line of defence. */
CTL_API ctl_status ctl_sync(ctl_ctx* ctx, void* stream);

/* Worst-case traversal stack (entries per lane) of the uploaded scene over
 * every traversal it can take; ctl_scene_upload refuses scenes above the
 * device stack depth (128).  0 without a scene. */
CTL_API int32_t ctl_scene_stack_bound(const ctl_ctx* ctx);

/* Traversal statistics for the roofline's algorithmic byte count (same kernel
 * compiled with counters; off in the timed path).  out[0]=rays,
 * out[1]=inner-node visits, out[2]=triangle tests, out[3]=instance entries. */
CTL_API ctl_status ctl_intersect_stats(ctl_ctx* ctx, int64_t n, const ctl_ray* d_rays, ctl_hit* d_hits,
                                       int32_t any_hit, uint64_t out[4], void* stream);
CTL_API ctl_status ctl_render_pass_stats(ctl_ctx* ctx, const ctl_pt_params* params, ctl_pixel* d_fb,
                                         uint64_t out[4], void* stream);

/* ------------------------------------------------------------------------ */
/* Host helpers (no GPU needed): the reference's host-side compile step      */
/* ------------------------------------------------------------------------ */

/* Worst-case traversal stack of one reference BVH (BVHNodeData tree rooted at
 * the child value root_value, SplitBVHBuilder.cpp:163-203): out[0] for the
 * reference's binary order, out[1] for the 4-wide tree the upload collapses it
 * into.  CTL_ERR_INVALID on a malformed tree (ctl_host_last_error).  Caps at
 * 1024 (a bound above the cap reads 1025). */
/* The 4-wide trees ctl_scene_upload builds from desc (bvh_nodes, tri_indices,
 * meshes, scene_bvh_nodes / scene_start_node), in the CTL_ARRAY_WIDE_BVH /
 * _SCENE_WIDE_BVH / _MESH_WIDE_BASE layouts (float nodes).  Query the sizes
 * with NULL outputs; *n_mesh_nodes / *n_scene_nodes are always set.
 * wbase_out holds desc->n_meshes entries.  CTL_ERR_INVALID on a malformed
 * tree or too small a capacity. */
CTL_API ctl_status ctl_host_wide_trees(const ctl_scene_desc* desc, void* mesh_out, uint64_t mesh_capacity,
                                       uint64_t* n_mesh_nodes, uint32_t* wbase_out, void* scene_out,
                                       uint64_t scene_capacity, uint64_t* n_scene_nodes);

CTL_API ctl_status ctl_host_bvh_stack_bound(const ctl_bvh_node* nodes, uint64_t n_nodes, int32_t root_value,
                                            int32_t out[2]);

/* TriIntersectorData::setData (Engine/TriIntersectorData.cu:5-18). */
CTL_API void ctl_woop_set(const float v0[3], const float v1[3], const float v2[3], ctl_woop_tri* out);

/* The SequenceSamplerData tables of pass `pass_index`
 * (seq1d/seq2d: num_sequences*length floats / float2, element-major). */
CTL_API ctl_status ctl_host_sampler_tables(uint64_t pass_index, uint32_t num_sequences,
                                           uint32_t sequence_length, float* seq1d, float* seq2d);

/* Host scene compiler: triangle soups -> the arrays of ctl_scene_desc
 * (BVH build = parallel binned SAH emitting the reference BVHNodeData layout,
 * leaf <= 8 tris as ConstructBVH, BVHBuilderHelper.cpp:129-147). */
typedef struct ctl_host_scene ctl_host_scene;
CTL_API ctl_host_scene* ctl_host_scene_create(void);
CTL_API void ctl_host_scene_destroy(ctl_host_scene* s);
/* Adds a mesh; returns its index (or -1).  normals/uvs may be NULL (flat /
 * zero), mat_index per triangle may be NULL (all 0).  Materials are local to
 * the mesh (Mesh::m_sMatInfo). */
CTL_API int32_t ctl_host_scene_add_mesh(ctl_host_scene* s, const float* vertices, uint32_t n_vertices,
                                        const uint32_t* indices, uint32_t n_triangles,
                                        const float* normals, const float* uvs,
                                        const uint8_t* mat_index,
                                        const ctl_material* materials, uint32_t n_materials);
/* Adds a node (instance) of a mesh with an object->world transform (row-major
 * 4x4, NULL = identity); returns the node index or -1. */
/* Adds an ImageTexture over the RGBA8 image `rgba` (width x height, both
 * powers of two, row 0 = top as loaded images are): builds the MIP pyramid
 * (2x2 box filter) and the EWA weight table (MIPMap.cpp:88-93).  mapping =
 * TextureMapping2D {m11, m12, m13, m21, m22, m23}, scale = m_scale.  Returns
 * the texture index for ctl_material.texture, or -1. */
CTL_API int32_t ctl_host_scene_add_texture(ctl_host_scene* s, const uint32_t* rgba, uint32_t width, uint32_t height,
                                           uint32_t filter, uint32_t wrap, const float mapping[6],
                                           const float scale[3]);
CTL_API int32_t ctl_host_scene_add_node(ctl_host_scene* s, uint32_t mesh, const float* xf16);
/* Marks material `local_material` of `node` as a DiffuseLight with constant
 * radiance (DynamicScene::CreateLight on a mesh part). Returns the light index. */
CTL_API int32_t ctl_host_scene_add_area_light(ctl_host_scene* s, uint32_t node, uint32_t local_material,
                                              const float radiance[3]);
/* PerspectiveSensor: position, target, up, fov (degrees), near/far, resolution. */
CTL_API ctl_status ctl_host_scene_set_camera(ctl_host_scene* s, const float pos[3], const float target[3],
                                             const float up[3], float fov_deg, float near_clip,
                                             float far_clip, uint32_t width, uint32_t height);
CTL_API ctl_status ctl_host_scene_set_flags(ctl_host_scene* s, uint32_t flags);
/* DynamicScene::setEnvironementMap: an InfiniteLight over image texture
 * `texture` (ctl_host_scene_add_texture) with radiance scale `scale`; the
 * compile builds its sampling tables (InfiniteLight::InfiniteLight) and adds it
 * after the area lights (env_map_index).  texture = 0xFFFFFFFF removes it. */
CTL_API ctl_status ctl_host_scene_set_environment(ctl_host_scene* s, uint32_t texture, const float scale[3]);
/* The environment light's m_worldTransform rotation (row-major 3x3, world =
 * R * local); the reference's constructor sets the identity (Light.cpp:58). */
CTL_API ctl_status ctl_host_scene_set_environment_transform(ctl_host_scene* s, const float rot9[9]);
/* Builds BVHs (threads=0: all hardware threads) and fills *out; the arrays
 * stay owned by `s` until it is destroyed or compiled again. */
/* BVH build quality knobs of the compile (SplitBVHBuilder's splitAlpha /
 * MaxSpatialDepth play this role in the reference, SplitBVHBuilder.hpp:62-67):
 * triangles whose box area exceeds split_alpha x the mesh mean get up to
 * 2^split_depth references with clipped boxes (split_alpha = 0 disables);
 * `bins` SAH bins per axis and leaves of at most `max_leaf` references
 * (Platform::m_maxLeafSize = 8, BVHBuilderHelper.cpp:119).  0 = default.
 * Defaults measured on C3 (10M triangles, 1080p PathTracer, 4-wide device
 * traversal): alpha 0.5 / 32 bins / leaf 8: 1673 Mrays/s; alpha 0.1875 /
 * 64 bins / leaf 2: 1984 Mrays/s (4.2 references per triangle). */
#define CTL_DEFAULT_SPLIT_ALPHA 0.1875f
#define CTL_DEFAULT_SPLIT_DEPTH 8u
#define CTL_DEFAULT_SAH_BINS 64u
#define CTL_DEFAULT_MAX_LEAF 2u
CTL_API ctl_status ctl_host_scene_set_bvh_params(ctl_host_scene* s, float split_alpha, uint32_t split_depth,
                                                 uint32_t bins, uint32_t max_leaf);
/* BVH builder of the compile (mesh trees; the instance tree is always binned):
 * CTL_BVH_BINNED: early split clipping + binned SAH (set_bvh_params' knobs);
 * CTL_BVH_SBVH (default): the reference's SplitBVHBuilder algorithm (SplitBVHBuilder.cpp:232-597,
 *   Stich et al. 2009): object splits by a SAH sweep over sorted references
 *   (binned above 16k references), spatial splits over 128 planes per axis with
 *   the triangle clipped at each plane (BVHBuilderHelper.cpp:78-113), reference
 *   unsplitting, spatial splits only where the object split's children overlap
 *   by >= split_alpha x the root area (reference 1e-5) and above depth 48; leaves
 *   of 1 .. max_leaf references (set_bvh_params; the reference's is 8).  Parallel
 *   over subtrees.  split_alpha is the SBVH's; the binned builder's stays in
 *   set_bvh_params.  C3 (10M triangles, 1080p PathTracer, 4-wide device
 *   traversal): binned + splitting (alpha 0.1875, 64 bins, leaf 2, 41.7M
 *   references) 2250 Mrays/s; SBVH leaf 2: 2618 (26.6M references), leaf 1 / 3
 *   / 4 / 8: 2566 / 2560 / 2504 / 2345; split_alpha 1e-6 / 1e-4: 2642 / 2456.
 *   Skinned meshes always take the binned builder without splitting (refit). */
#define CTL_BVH_BINNED 0u
#define CTL_BVH_SBVH 1u
CTL_API ctl_status ctl_host_scene_set_bvh_builder(ctl_host_scene* s, uint32_t builder, float split_alpha);
CTL_API ctl_status ctl_host_scene_compile(ctl_host_scene* s, uint32_t threads, ctl_scene_desc* out);

/* Skinned mesh (AnimatedMesh, Engine/AnimatedMesh.h:71-110): compiled in its
 * rest pose (vertex positions as given; no reference splitting, so every
 * triangle has one BVH reference) and re-posed on the device by
 * ctl_scene_animate.  uvs: 2 floats per vertex or NULL; mat_index as
 * ctl_host_scene_add_mesh.  Area lights on animated meshes are refused at
 * compile (their ShapeSet would go stale).  Returns the mesh index or -1. */
CTL_API int32_t ctl_host_scene_add_animated_mesh(ctl_host_scene* s, const ctl_anim_vertex* vertices,
                                                 uint32_t n_vertices, const uint32_t* indices, uint32_t n_triangles,
                                                 const float* uvs, const uint8_t* mat_index,
                                                 const ctl_material* materials, uint32_t n_materials);

/* Compiled meshes (.xmsh).  Replaces Mesh::Mesh(path, IInStream&, ...)
 * (Engine/Mesh.cpp:46-98) as called by DynamicScene::CreateNode(path)
 * (DynamicScene.cpp:270-345) on a static mesh file (leading u32
 * MeshCompileType 0; Animated files are refused): loads the box, MeshPartLights, TriangleData,
 * BVHNodeData, TriIntersectorData and TriIntersectorData2 arrays of the file
 * as they are (no rebuild).  Every node later created on the mesh gets one
 * area light per MeshPartLight, matched to a material by name
 * (DynamicScene.cpp:340-341, 689-734).  A reference Material record is a
 * build-specific variant blob: pass its size (sizeof(Material) of the writing
 * build) and the flattened kernel materials in file order; only each record's
 * leading FixedString<64> Name is read.  With materials == NULL the records
 * must be the CTL_XMSH_MATERIAL_RECORD_SIZE-byte records written by
 * ctl_host_scene_write_xmsh (Name + ctl_material).  The arrays are checked to
 * form one tree (children and entries in range, depth <= 64) before they are
 * accepted.  Returns the mesh index, or -1 (ctl_host_last_error). */
#define CTL_XMSH_MATERIAL_RECORD_SIZE 148u
CTL_API int32_t ctl_host_scene_add_xmsh(ctl_host_scene* s, const void* data, uint64_t size,
                                        uint32_t material_record_size, const ctl_material* materials,
                                        uint32_t n_materials);
/* Writes mesh `mesh` of the last compile as an .xmsh stream: the byte layout
 * of Mesh::CompileMesh + ConstructBVH (Mesh.cpp:279-288,
 * MeshLoader/BVHBuilderHelper.cpp:129-147), materials as
 * CTL_XMSH_MATERIAL_RECORD_SIZE-byte records named "material<i>", one
 * MeshPartLight per lit material.  out == NULL: only *size is set. */
CTL_API ctl_status ctl_host_scene_write_xmsh(ctl_host_scene* s, uint32_t mesh, void* out, uint64_t capacity,
                                             uint64_t* size);
CTL_API const char* ctl_host_last_error(void);

/* Synthetic workloads of BASELINE.json (seed 0x5EED): 1 = C1 Cornell box
 * (32 tris), 2 = C2 100k-tri field, 3 = C3 ~10M-tri "San-Miguel-scale",
 * 5 = C5: C3 geometry with 30 % roughdielectric (Beckmann / GGX, eta 1.5,
 * alpha 0.05-0.5) and 30 % image-textured diffuse materials (procedural
 * 1024^2 checker/noise MIP maps, trilinear and EWA filtering).
 * `scale` multiplies the triangle budget (1.0 = the named size).  The camera
 * resolution is width x height. */
CTL_API ctl_status ctl_host_scene_generate(ctl_host_scene* s, int32_t config, double scale,
                                           uint32_t width, uint32_t height);

#ifdef __cplusplus
}
#endif
#endif /* CTL_TRACE_H */

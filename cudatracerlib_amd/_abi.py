"""ctypes mirror of include/ctl_trace.h (the C-ABI drop-in boundary).

Layouts are byte-identical to the reference structures named in the header;
``tests/test_abi.py`` checks every size against the C side.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CTL_LIB overrides the library path (the sanitizer build, tools/san_tests.sh).
LIB_PATH = os.environ.get("CTL_LIB") or os.path.join(_HERE, "_lib", "libctl_trace.so")

# CTL_ABI_VERSION of the include/ctl_trace.h these bindings mirror; load()
# refuses a library that reports another (mismatched struct layouts).
ABI_VERSION = 4
CTL_OK = 0
CTL_SCENE_HALF_HOST_QUIRK = 1
CTL_SCENE_BINARY_BVH = 2
CTL_SCENE_WIDE_QUANT = 4
CTL_DEFAULT_SPLIT_ALPHA = 0.1875   # include/ctl_trace.h
CTL_XMSH_MATERIAL_RECORD_SIZE = 148
CTL_COMM_ID_BYTES = 128
CTL_BVH_BINNED, CTL_BVH_SBVH = 0, 1
(CTL_ARRAY_TRI_DATA, CTL_ARRAY_WOOP, CTL_ARRAY_BVH_NODES, CTL_ARRAY_SCENE_BVH, CTL_ARRAY_MESH_BOXES, CTL_ARRAY_RAY_EPS,
 CTL_ARRAY_SAMPLES_1D, CTL_ARRAY_SAMPLES_2D) = range(8)
CTL_BSDF_DIFFUSE = 1
CTL_EDIFFUSE_REFLECTION = 0x2
CTL_EGLOSSY_REFLECTION = 0x8
CTL_EGLOSSY_TRANSMISSION = 0x10
CTL_BSDF_ROUGHDIELECTRIC = 5
CTL_MICROFACET_BECKMANN = 0
CTL_MICROFACET_GGX = 1
CTL_TEX_POINT, CTL_TEX_BILINEAR, CTL_TEX_EWA, CTL_TEX_TRILINEAR = 0, 1, 2, 3
CTL_WRAP_REPEAT, CTL_WRAP_CLAMP, CTL_WRAP_MIRROR, CTL_WRAP_BLACK = 0, 1, 2, 3
CTL_MAX_NUM_LIGHTS = 16
CTL_PT_MEGAKERNEL = 1
CTL_PT_WAVEFRONT = 2
CTL_PT_RENDER_AHEAD = 4
# ctl_scene_update dirty groups (DynamicScene streams)
CTL_DIRTY_TRI_DATA, CTL_DIRTY_WOOP, CTL_DIRTY_BVH, CTL_DIRTY_TRI_INDICES = 1, 2, 4, 8
CTL_DIRTY_MATERIALS, CTL_DIRTY_MESHES, CTL_DIRTY_NODES, CTL_DIRTY_LIGHTS = 16, 32, 64, 128
CTL_DIRTY_TEXTURES, CTL_DIRTY_ENV, CTL_DIRTY_ALL = 256, 512, 1023
# ctl_scene_read arrays
(CTL_ARRAY_TRI_DATA, CTL_ARRAY_WOOP, CTL_ARRAY_BVH_NODES, CTL_ARRAY_SCENE_BVH, CTL_ARRAY_MESH_BOXES, CTL_ARRAY_RAY_EPS,
 CTL_ARRAY_SAMPLES_1D, CTL_ARRAY_SAMPLES_2D, CTL_ARRAY_NODE_XF, CTL_ARRAY_NODE_INV_XF, CTL_ARRAY_LIGHTS,
 CTL_ARRAY_LIGHT_TRIS, CTL_ARRAY_LIGHT_CDF, CTL_ARRAY_SCENE_BOX, CTL_ARRAY_ENV, CTL_ARRAY_WIDE_BVH,
 CTL_ARRAY_SCENE_WIDE_BVH, CTL_ARRAY_MESH_WIDE_BASE, CTL_ARRAY_CULL_BOUND) = range(19)


class BVHNode(C.Structure):          # BVHNodeData, 64 B
    _fields_ = [("v", C.c_float * 16)]


class WoopTri(C.Structure):          # TriIntersectorData, 48 B
    _fields_ = [("v", C.c_float * 12)]


class TriangleData(C.Structure):     # TriangleData (EXT_TRI), 32 B
    _fields_ = [("w", C.c_uint32 * 8)]


class KernelMesh(C.Structure):       # KernelMesh, 20 B
    _fields_ = [("triangle_offset", C.c_uint32), ("bvh_node_offset", C.c_uint32),
                ("bvh_triangle_offset", C.c_uint32), ("bvh_indices_offset", C.c_uint32),
                ("std_material_offset", C.c_uint32)]


class Node(C.Structure):             # Node, 24 B
    _fields_ = [("mesh_index", C.c_uint32), ("material_offset", C.c_uint32),
                ("instanced_material", C.c_uint32), ("lights", C.c_uint32 * 2), ("num_lights", C.c_uint32)]


class Float4x4(C.Structure):
    _fields_ = [("m", C.c_float * 16)]


class Ray(C.Structure):              # traversalRay, 32 B
    _fields_ = [("o", C.c_float * 3), ("tmin", C.c_float), ("d", C.c_float * 3), ("tmax", C.c_float)]


class Hit(C.Structure):              # traversalResult, 16 B
    _fields_ = [("dist", C.c_float), ("node_idx", C.c_int32), ("tri_idx", C.c_int32), ("bary", C.c_int32)]


class Pixel(C.Structure):            # PixelData, 28 B
    _fields_ = [("rgb", C.c_float * 3), ("rgb_splat", C.c_float * 3), ("weight_sum", C.c_float)]


class Material(C.Structure):        # 80 B
    _fields_ = [("bsdf_type", C.c_uint32), ("combined_type", C.c_uint32), ("two_sided", C.c_uint32),
                ("node_light_index", C.c_uint32), ("reflectance", C.c_float * 3), ("texture", C.c_uint32),
                ("transmittance", C.c_float * 3), ("distribution", C.c_uint32), ("eta", C.c_float),
                ("inv_eta", C.c_float), ("alpha_u", C.c_float), ("alpha_v", C.c_float),
                ("sample_visible", C.c_uint32), ("alpha_state", C.c_uint32), ("alpha_texture", C.c_uint32),
                ("alpha_threshold", C.c_float)]


class Texture(C.Structure):
    _fields_ = [("mapping", C.c_float * 6), ("set_id", C.c_uint32), ("scale", C.c_float * 3),
                ("width", C.c_uint32), ("height", C.c_uint32), ("levels", C.c_uint32), ("filter", C.c_uint32),
                ("wrap", C.c_uint32), ("offsets", C.c_uint32 * 16), ("weight_lut", C.c_float * 64)]


class LightTri(C.Structure):         # ShapeSet::triData, 64 B
    _fields_ = [("p", (C.c_float * 3) * 3), ("n", C.c_float * 3), ("area", C.c_float),
                ("i_dat", C.c_uint32), ("t_dat", C.c_uint32), ("pad", C.c_uint32)]


class Light(C.Structure):
    _fields_ = [("radiance", C.c_float * 3), ("orthogonal", C.c_uint32), ("tri_first", C.c_uint32),
                ("tri_count", C.c_uint32), ("cdf_first", C.c_uint32), ("sum_area", C.c_float),
                ("node_idx", C.c_uint32), ("kind", C.c_uint32), ("pad", C.c_uint32 * 2)]


CTL_LIGHT_DIFFUSE = 0
CTL_LIGHT_INFINITE = 1


class EnvLight(C.Structure):          # ctl_env_light (InfiniteLight), 112 B
    _fields_ = [("texture", C.c_uint32), ("scale", C.c_float * 3), ("size", C.c_float * 2),
                ("pixel_size", C.c_float * 2), ("normalization", C.c_float), ("scene_center", C.c_float * 3),
                ("scene_radius", C.c_float), ("cdf_cols", C.c_uint32), ("cdf_rows", C.c_uint32),
                ("row_weights", C.c_uint32), ("world", (C.c_float * 3) * 3), ("pad", C.c_uint32 * 3)]


class Camera(C.Structure):
    _fields_ = [("to_world", Float4x4), ("sample_to_camera", Float4x4), ("dx", C.c_float * 3),
                ("dy", C.c_float * 3), ("inv_resolution", C.c_float * 2), ("width", C.c_uint32),
                ("height", C.c_uint32)]


class AnimVertex(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("normal", C.c_float * 3), ("bone_indices", C.c_uint64),
                ("bone_weights", C.c_uint64)]


class AnimMesh(C.Structure):
    _fields_ = [("mesh", C.c_uint32), ("vertex_first", C.c_uint32), ("vertex_count", C.c_uint32),
                ("tri_first", C.c_uint32), ("tri_count", C.c_uint32), ("max_bone", C.c_uint32)]


class SceneDesc(C.Structure):
    _fields_ = [
        ("tri_data", C.POINTER(TriangleData)), ("n_tri_data", C.c_uint64),
        ("woop_tris", C.POINTER(WoopTri)), ("n_woop_tris", C.c_uint64),
        ("bvh_nodes", C.POINTER(BVHNode)), ("n_bvh_nodes", C.c_uint64),
        ("tri_indices", C.POINTER(C.c_uint32)), ("n_tri_indices", C.c_uint64),
        ("materials", C.POINTER(Material)), ("n_materials", C.c_uint32),
        ("meshes", C.POINTER(KernelMesh)), ("n_meshes", C.c_uint32),
        ("nodes", C.POINTER(Node)), ("n_nodes", C.c_uint32),
        ("scene_bvh_nodes", C.POINTER(BVHNode)), ("n_scene_bvh_nodes", C.c_uint32),
        ("scene_start_node", C.c_int32),
        ("node_xf", C.POINTER(Float4x4)), ("node_inv_xf", C.POINTER(Float4x4)),
        ("lights", C.POINTER(Light)), ("n_lights", C.c_uint32),
        ("light_tris", C.POINTER(LightTri)), ("n_light_tris", C.c_uint32),
        ("light_tri_cdf", C.POINTER(C.c_float)), ("n_light_tri_cdf", C.c_uint32),
        ("light_cdf", C.c_float * CTL_MAX_NUM_LIGHTS),
        ("textures", C.POINTER(Texture)), ("n_textures", C.c_uint32),
        ("tex_data", C.POINTER(C.c_uint32)), ("n_tex_data", C.c_uint64),
        ("env_map_index", C.c_uint32),
        ("env", C.POINTER(EnvLight)),
        ("env_data", C.POINTER(C.c_float)), ("n_env_data", C.c_uint64),
        ("box_min", C.c_float * 3), ("box_max", C.c_float * 3),
        ("ray_eps", C.c_float),
        ("camera", Camera),
        ("flags", C.c_uint32),
        ("mesh_boxes", C.POINTER(C.c_float)),
        ("anim_vertices", C.POINTER(AnimVertex)), ("n_anim_vertices", C.c_uint32),
        ("anim_triangles", C.POINTER(C.c_uint32)), ("n_anim_triangles", C.c_uint32),
        ("anim_meshes", C.POINTER(AnimMesh)), ("n_anim_meshes", C.c_uint32),
    ]


class PixelVariance(C.Structure):    # PixelVarianceInfo, 44 B
    _fields_ = [("prev_I", C.c_float * 3), ("half_buffer", C.c_float * 3), ("iterations_done", C.c_int32),
                ("weight", C.c_float), ("sum_x", C.c_float), ("sum_x2", C.c_float), ("num_samples_var", C.c_int32)]


class PTParams(C.Structure):
    _fields_ = [("direct", C.c_int32), ("max_path_length", C.c_int32), ("rr_start_depth", C.c_int32),
                ("shadow_any_hit", C.c_int32), ("tile_size", C.c_uint32), ("num_ranks", C.c_uint32),
                ("rank", C.c_uint32), ("flags", C.c_uint32)]


class PrimParams(C.Structure):
    _fields_ = [("draw_mode", C.c_int32), ("max_path_length", C.c_int32), ("near_depth", C.c_float),
                ("far_depth", C.c_float), ("flags", C.c_uint32)]


# PathTrace_DrawMode (PrimTracer.h:7-9)
PRIM_DRAW_MODES = ["linear_depth", "D3D_depth", "v_absdot_n_geo", "v_dot_n_geo", "v_dot_n_shade", "n_geo_colored",
                   "n_shade_colored", "uv", "bary_coords", "first_Le", "first_f", "first_f_direct",
                   "first_non_delta_Le", "first_non_delta_f", "first_non_delta_f_direct"]


CTL_WPT_SHADOW_ANY_HIT = 1 << 0   # ctl_wpt_params.flags


class WptParams(C.Structure):
    _fields_ = [("direct", C.c_int32), ("max_path_length", C.c_int32), ("rr_start_depth", C.c_int32),
                ("passes_done", C.c_uint32), ("flags", C.c_uint32)]


# Every symbol include/ctl_trace.h declares: (name, restype, argtypes)
_vp = C.c_void_p
SYMBOLS = [
    ("ctl_abi_version", C.c_int32, []),
    ("ctl_create", _vp, [C.c_int32]),
    ("ctl_destroy", None, [_vp]),
    ("ctl_last_error", C.c_char_p, [_vp]),
    ("ctl_scene_upload", C.c_int32, [_vp, C.POINTER(SceneDesc)]),
    ("ctl_scene_update", C.c_int32, [_vp, C.POINTER(SceneDesc), C.c_uint32, _vp]),
    ("ctl_scene_set_transform", C.c_int32, [_vp, C.c_uint32, _vp, _vp]),
    ("ctl_sampler_generate", C.c_int32, [_vp, C.c_uint64, _vp]),
    ("ctl_sampler_upload", C.c_int32, [_vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
    ("ctl_intersect", C.c_int32, [_vp, C.c_int64, _vp, _vp, C.c_int32, _vp]),
    ("ctl_occluded", C.c_int32, [_vp, C.c_int64, _vp, _vp, C.c_int32, _vp]),
    ("ctl_render_pass", C.c_int32, [_vp, C.POINTER(PTParams), _vp, _vp]),
    ("ctl_render_passes", C.c_int32, [_vp, C.POINTER(PTParams), C.c_uint64, C.c_uint32, _vp, _vp]),
    ("ctl_wpt_render_pass", C.c_int32, [_vp, C.POINTER(WptParams), _vp, _vp]),
    ("ctl_prim_pass", C.c_int32, [_vp, C.POINTER(PrimParams), _vp, _vp, _vp]),
    ("ctl_rays_traced", C.c_uint64, [_vp]),
    ("ctl_reset_rays", C.c_int32, [_vp, _vp]),
    ("ctl_sync", C.c_int32, [_vp, _vp]),
    ("ctl_scene_stack_bound", C.c_int32, [_vp]),
    ("ctl_host_bvh_stack_bound", C.c_int32, [_vp, C.c_uint64, C.c_int32, _vp]),
    ("ctl_host_wide_trees", C.c_int32, [C.POINTER(SceneDesc), _vp, C.c_uint64, C.POINTER(C.c_uint64), _vp, _vp,
                                        C.c_uint64, C.POINTER(C.c_uint64)]),
    ("ctl_intersect_stats", C.c_int32, [_vp, C.c_int64, _vp, _vp, C.c_int32, C.POINTER(C.c_uint64), _vp]),
    ("ctl_render_pass_stats", C.c_int32, [_vp, C.POINTER(PTParams), _vp, C.POINTER(C.c_uint64), _vp]),
    ("ctl_last_pass_ms", C.c_int32, [_vp, C.POINTER(C.c_float)]),
    ("ctl_camera_rays", C.c_int32, [_vp, C.POINTER(PTParams), _vp, C.c_int64, C.POINTER(C.c_int64), _vp]),
    ("ctl_comm_unique_id", C.c_int32, [_vp]),
    ("ctl_comm_init_rank", C.c_int32, [C.POINTER(_vp), C.c_int32, _vp, C.c_int32, C.c_int32]),
    ("ctl_comm_init_all", C.c_int32, [C.POINTER(_vp), C.c_int32, _vp]),
    ("ctl_comm_destroy", C.c_int32, [_vp]),
    ("ctl_fb_reduce", C.c_int32, [_vp, _vp, _vp, _vp, C.c_uint64, C.c_int32, _vp]),
    ("ctl_fb_reduce_all", C.c_int32, [_vp, _vp, _vp, _vp, C.c_int32, C.c_uint64, C.c_int32, _vp]),
    ("ctl_image_resolve", C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, C.c_float, _vp, _vp]),
    ("ctl_variance_add_pass", C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, C.c_float, C.c_uint32, _vp, _vp, _vp]),
    ("ctl_variance_stats", C.c_int32, [_vp, _vp, C.c_uint64, _vp, _vp, _vp, _vp]),
    ("ctl_woop_set", None, [_vp, _vp, _vp, C.POINTER(WoopTri)]),
    ("ctl_host_sampler_tables", C.c_int32, [C.c_uint64, C.c_uint32, C.c_uint32, _vp, _vp]),
    ("ctl_host_scene_create", _vp, []),
    ("ctl_host_scene_destroy", None, [_vp]),
    ("ctl_host_scene_add_mesh", C.c_int32, [_vp, _vp, C.c_uint32, _vp, C.c_uint32, _vp, _vp, _vp,
                                            C.POINTER(Material), C.c_uint32]),
    ("ctl_host_scene_add_texture", C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _vp, _vp]),
    ("ctl_host_scene_add_node", C.c_int32, [_vp, C.c_uint32, _vp]),
    ("ctl_host_scene_add_area_light", C.c_int32, [_vp, C.c_uint32, C.c_uint32, _vp]),
    ("ctl_host_scene_set_camera", C.c_int32, [_vp, _vp, _vp, _vp, C.c_float, C.c_float, C.c_float,
                                              C.c_uint32, C.c_uint32]),
    ("ctl_host_scene_set_flags", C.c_int32, [_vp, C.c_uint32]),
    ("ctl_host_scene_set_environment", C.c_int32, [_vp, C.c_uint32, _vp]),
    ("ctl_host_scene_set_environment_transform", C.c_int32, [_vp, _vp]),
    ("ctl_host_scene_set_bvh_params", C.c_int32, [_vp, C.c_float, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("ctl_host_scene_set_bvh_builder", C.c_int32, [_vp, C.c_uint32, C.c_float]),
    ("ctl_host_scene_compile", C.c_int32, [_vp, C.c_uint32, C.POINTER(SceneDesc)]),
    ("ctl_host_scene_add_animated_mesh", C.c_int32, [_vp, C.POINTER(AnimVertex), C.c_uint32, _vp, C.c_uint32, _vp,
                                                     _vp, C.POINTER(Material), C.c_uint32]),
    ("ctl_scene_animate", C.c_int32, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, C.c_float, _vp]),
    ("ctl_scene_read", C.c_int32, [_vp, C.c_uint32, C.c_uint64, C.c_uint64, _vp]),
    ("ctl_host_scene_add_xmsh", C.c_int32, [_vp, _vp, C.c_uint64, C.c_uint32, _vp, C.c_uint32]),
    ("ctl_host_scene_write_xmsh", C.c_int32, [_vp, C.c_uint32, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("ctl_host_last_error", C.c_char_p, []),
    ("ctl_host_scene_generate", C.c_int32, [_vp, C.c_int32, C.c_double, C.c_uint32, C.c_uint32]),
]

_lib = None


def load(path=LIB_PATH):
    """Load libctl_trace.so and bind every declared symbol.  Raises loudly if
    the HIP extension was not built: there is no fallback path."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libctl_trace.so not built ({path}); run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    for name, res, args in SYMBOLS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.ctl_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"{path} reports CTL_ABI_VERSION {v}, these bindings are for {ABI_VERSION}: rebuild it")
    if path == LIB_PATH:
        _lib = lib
    return lib

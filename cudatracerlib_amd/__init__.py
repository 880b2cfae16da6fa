"""cudatracerlib_amd — MI355X-native traversal backend for the CudaTracerLib
hot path (BVH traversal + Woop ray/triangle intersection driven by the
PathTracer pass loop).

The product is ``_lib/libctl_trace.so`` (hand-written gfx950 HIP kernels plus
the C-ABI of ``include/ctl_trace.h``).  This module is a thin host-side mirror
of the reference's surface for that path:

  reference                                   here
  ------------------------------------------- ---------------------------------
  DynamicScene (host scene, Engine/DynamicScene.h:40-188)   HostScene
  UpdateKernel / KernelDynamicScene upload                  Tracer.upload_scene
  __internal__IntersectBuffers (TraceHelper.cu:736-746)     Tracer.intersect_buffers
  PathTracer::DoPass (Kernel/Tracer.h:209-248)              PathTracer.do_pass
  k_getNumRaysTraced (TraceHelper.cu:309-314)               Tracer.rays_traced

Device memory, streams and torch.distributed come from PyTorch; no torch type
crosses the C-ABI (device pointers are passed as integers).  There is no CPU
fallback: every compute call goes through the HIP library and raises if it is
missing or fails.
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import (PTParams, WptParams, PrimParams, SceneDesc, Material, Pixel, Ray, Hit, CTL_SCENE_HALF_HOST_QUIRK, CTL_SCENE_BINARY_BVH,
                   CTL_BSDF_DIFFUSE, CTL_EDIFFUSE_REFLECTION, CTL_PT_MEGAKERNEL, CTL_PT_WAVEFRONT, CTL_PT_RENDER_AHEAD,
                   CTL_COMM_ID_BYTES)

__all__ = ["HostScene", "Tracer", "PathTracer", "WavefrontPathTracer", "PrimTracer", "PrimParams", "WptParams", "PTParams", "SceneDesc", "Material", "Pixel", "Ray", "Hit",
           "roughdielectric_material", "set_alpha_map", "comm_unique_id", "comm_init_rank", "comm_init_all",
           "comm_destroy",
           "CTL_SCENE_HALF_HOST_QUIRK", "CTL_SCENE_BINARY_BVH", "CTL_PT_MEGAKERNEL", "CTL_PT_WAVEFRONT", "CTL_PT_RENDER_AHEAD", "lib", "diffuse_material"]


def lib():
    return _abi.load()


class CTLError(RuntimeError):
    pass


def _check(status, ctx=None, what=""):
    if status != 0:
        L = lib()
        msg = L.ctl_last_error(ctx) if ctx is not None else L.ctl_host_last_error()
        raise CTLError(f"{what} failed (status {status}): {msg.decode() if msg else ''}")


def set_alpha_map(m, state, threshold, alpha_texture=None):
    """Material::AlphaMap (Engine/Material.h:14-36): state 1/2 = luminance/alpha of
    `alpha_texture`, 5/6 = luminance/alpha of the diffuse reflectance texture."""
    m.alpha_state = int(state)
    m.alpha_texture = 0xFFFFFFFF if alpha_texture is None else int(alpha_texture)
    m.alpha_threshold = float(threshold)
    return m


def diffuse_material(r, g, b, two_sided=True, texture=None):
    """diffuse BSDF (BSDF_Simple.cu:7-75); `texture` = ImageTexture index of
    m_reflectance (HostScene.add_texture), else the constant (r, g, b)."""
    m = Material()
    m.alpha_texture = 0xFFFFFFFF
    m.bsdf_type = CTL_BSDF_DIFFUSE
    m.combined_type = CTL_EDIFFUSE_REFLECTION
    m.two_sided = 1 if two_sided else 0
    m.node_light_index = 0xFFFFFFFF
    m.reflectance[:] = [r, g, b]
    m.texture = 0xFFFFFFFF if texture is None else int(texture)
    return m


def roughdielectric_material(distribution, eta, alpha_u, alpha_v=None, reflectance=(1.0, 1.0, 1.0),
                             transmittance=(1.0, 1.0, 1.0)):
    """roughdielectric BSDF (BSDF_Simple.cu:373-615) with constant textures;
    distribution = _abi.CTL_MICROFACET_BECKMANN or _abi.CTL_MICROFACET_GGX."""
    m = Material()
    m.alpha_texture = 0xFFFFFFFF
    m.bsdf_type = _abi.CTL_BSDF_ROUGHDIELECTRIC
    m.combined_type = _abi.CTL_EGLOSSY_REFLECTION | _abi.CTL_EGLOSSY_TRANSMISSION
    m.two_sided = 0
    m.node_light_index = 0xFFFFFFFF
    m.reflectance[:] = list(reflectance)
    m.texture = 0xFFFFFFFF
    m.transmittance[:] = list(transmittance)
    m.distribution = int(distribution)
    m.eta = float(eta)
    m.inv_eta = float(np.float32(1.0) / np.float32(eta))      # roughdielectric::Update
    m.alpha_u = float(alpha_u)
    m.alpha_v = float(alpha_u if alpha_v is None else alpha_v)
    m.sample_visible = 1                                         # getSampleVisible(Beckmann/GGX, true)
    return m


class HostScene:
    """Host-side scene compiler (the reference's DynamicScene + Mesh compile)."""

    def __init__(self):
        self._L = lib()
        self._h = self._L.ctl_host_scene_create()
        self.desc = None

    def close(self):
        if self._h:
            self._L.ctl_host_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def generate(self, config, scale=1.0, width=256, height=256):
        _check(self._L.ctl_host_scene_generate(self._h, int(config), float(scale), int(width), int(height)),
               None, "ctl_host_scene_generate")
        return self

    def add_mesh(self, vertices, indices, materials, mat_index=None, normals=None, uvs=None):
        import numpy as np
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        i = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 3)
        mats = (Material * len(materials))(*materials)
        mi = None if mat_index is None else np.ascontiguousarray(mat_index, dtype=np.uint8)
        n = None if normals is None else np.ascontiguousarray(normals, dtype=np.float32)
        uv = None if uvs is None else np.ascontiguousarray(uvs, dtype=np.float32)
        self._keep = getattr(self, "_keep", []) + [v, i, mi, n, uv, mats]
        r = self._L.ctl_host_scene_add_mesh(
            self._h, v.ctypes.data, v.shape[0], i.ctypes.data, i.shape[0],
            None if n is None else n.ctypes.data, None if uv is None else uv.ctypes.data,
            None if mi is None else mi.ctypes.data, mats, len(materials))
        if r < 0:
            _check(1, None, "add_mesh")
        return r

    def add_texture(self, rgba, filter=_abi.CTL_TEX_TRILINEAR, wrap=_abi.CTL_WRAP_REPEAT,
                    mapping=(1.0, 0.0, 0.0, 0.0, 1.0, 0.0), scale=(1.0, 1.0, 1.0)):
        """ImageTexture over an (h, w) uint32 RGBA8 image (r in the low byte); returns its index."""
        img = np.ascontiguousarray(rgba, dtype=np.uint32)
        h, w = img.shape
        self._keep = getattr(self, "_keep", []) + [img]
        r = self._L.ctl_host_scene_add_texture(self._h, img.ctypes.data, w, h, int(filter), int(wrap),
                                               (C.c_float * 6)(*mapping), (C.c_float * 3)(*scale))
        if r < 0:
            _check(1, None, "add_texture")
        return r

    def add_animated_mesh(self, vertices, normals, bone_indices, bone_weights, indices, materials, mat_index=None,
                          uvs=None):
        """Skinned mesh (AnimatedMesh): rest pose `vertices`/`normals` (n, 3), 8 bone
        indices and 8 weights (n, 8) uint8 per vertex (weight w means w/255)."""
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        nrm = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        bi = np.ascontiguousarray(bone_indices, dtype=np.uint8).reshape(-1, 8)
        bw = np.ascontiguousarray(bone_weights, dtype=np.uint8).reshape(-1, 8)
        dt = np.dtype([("pos", np.float32, 3), ("normal", np.float32, 3), ("bi", np.uint8, 8), ("bw", np.uint8, 8)])
        assert dt.itemsize == C.sizeof(_abi.AnimVertex)
        rec = np.zeros(v.shape[0], dt)
        rec["pos"], rec["normal"], rec["bi"], rec["bw"] = v, nrm, bi, bw
        av = C.cast(rec.ctypes.data, C.POINTER(_abi.AnimVertex))
        i = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 3)
        mats = (Material * len(materials))(*materials)
        mi = None if mat_index is None else np.ascontiguousarray(mat_index, dtype=np.uint8)
        uv = None if uvs is None else np.ascontiguousarray(uvs, dtype=np.float32)
        self._keep = getattr(self, "_keep", []) + [rec, i, mi, uv, mats]
        r = self._L.ctl_host_scene_add_animated_mesh(
            self._h, av, v.shape[0], i.ctypes.data, i.shape[0], None if uv is None else uv.ctypes.data,
            None if mi is None else mi.ctypes.data, mats, len(materials))
        if r < 0:
            _check(1, None, "add_animated_mesh")
        return r

    def add_xmsh(self, data, materials=None, material_record_size=_abi.CTL_XMSH_MATERIAL_RECORD_SIZE):
        """Compiled mesh from an .xmsh stream (bytes or a path) — Mesh::Mesh(path, IInStream&)
        (Engine/Mesh.cpp:46-98).  Reference files: pass sizeof(Material) of the writing build as
        material_record_size and the kernel materials in file order."""
        if isinstance(data, (str, os.PathLike)):
            with open(data, "rb") as f:
                data = f.read()
        buf = C.create_string_buffer(bytes(data), len(data))
        mats = None if materials is None else (Material * len(materials))(*materials)
        r = self._L.ctl_host_scene_add_xmsh(self._h, buf, len(data), int(material_record_size), mats,
                                            0 if materials is None else len(materials))
        if r < 0:
            _check(1, None, "add_xmsh")
        return r

    def write_xmsh(self, mesh, path=None):
        """Mesh `mesh` of the last compile as .xmsh bytes (written to `path` when given)."""
        n = C.c_uint64(0)
        _check(self._L.ctl_host_scene_write_xmsh(self._h, int(mesh), None, 0, C.byref(n)), None, "write_xmsh")
        buf = C.create_string_buffer(n.value)
        _check(self._L.ctl_host_scene_write_xmsh(self._h, int(mesh), buf, n.value, C.byref(n)), None, "write_xmsh")
        data = buf.raw[:n.value]
        if path is not None:
            with open(path, "wb") as f:
                f.write(data)
        return data

    def add_node(self, mesh, xf16=None):
        arr = None
        if xf16 is not None:
            arr = (C.c_float * 16)(*[float(x) for x in xf16])
        r = self._L.ctl_host_scene_add_node(self._h, mesh, arr)
        if r < 0:
            _check(1, None, "add_node")
        return r

    def add_area_light(self, node, local_material, radiance):
        arr = (C.c_float * 3)(*radiance)
        r = self._L.ctl_host_scene_add_area_light(self._h, node, local_material, arr)
        if r < 0:
            _check(1, None, "add_area_light")
        return r

    def set_camera(self, pos, target, up, fov_deg, width, height, near=1.0, far=100000.0):
        f3 = C.c_float * 3
        _check(self._L.ctl_host_scene_set_camera(self._h, f3(*pos), f3(*target), f3(*up), fov_deg, near, far,
                                                  width, height), None, "set_camera")

    def set_flags(self, flags):
        _check(self._L.ctl_host_scene_set_flags(self._h, flags), None, "set_flags")

    def set_environment(self, texture, scale=(1.0, 1.0, 1.0)):
        """DynamicScene::setEnvironementMap: an InfiniteLight over image texture
        `texture` (an add_texture index) with radiance `scale`; None removes it."""
        tex = 0xFFFFFFFF if texture is None else int(texture)
        _check(self._L.ctl_host_scene_set_environment(self._h, tex, (C.c_float * 3)(*scale)), None,
               "set_environment")
        return self

    def set_environment_transform(self, rot):
        """InfiniteLight::m_worldTransform (Light.h:307): a 3x3 rotation, world = rot @ local."""
        r = np.ascontiguousarray(rot, dtype=np.float32).reshape(9)
        _check(self._L.ctl_host_scene_set_environment_transform(self._h, (C.c_float * 9)(*r.tolist())), None,
               "set_environment_transform")
        return self

    def set_bvh_params(self, split_alpha=None, split_depth=8, bins=0, max_leaf=0):
        """BVH build knobs: reference splitting of large triangles (split_alpha = 0
        disables, None = library default), SAH bins per axis and max leaf size
        (0 = library default)."""
        if split_alpha is None:
            split_alpha = _abi.CTL_DEFAULT_SPLIT_ALPHA
        _check(self._L.ctl_host_scene_set_bvh_params(self._h, float(split_alpha), int(split_depth), int(bins),
                                                      int(max_leaf)), None, "set_bvh_params")
        return self

    def set_bvh_builder(self, builder="sbvh", split_alpha=1.0e-5):
        """Mesh BVH builder: "sbvh" (the reference's SplitBVHBuilder with in-build
        spatial splits, default) or "binned" (early split clipping + binned SAH)."""
        b = {"binned": _abi.CTL_BVH_BINNED, "sbvh": _abi.CTL_BVH_SBVH}[builder]
        _check(self._L.ctl_host_scene_set_bvh_builder(self._h, b, float(split_alpha)), None, "set_bvh_builder")
        return self

    def compile(self, threads=0):
        d = SceneDesc()
        _check(self._L.ctl_host_scene_compile(self._h, threads, C.byref(d)), None, "ctl_host_scene_compile")
        self.desc = d
        return d


def bvh_stack_bound(nodes, root_value=0):
    """(binary, 4-wide) worst-case traversal stack of a reference BVHNodeData
    tree (ctl_host_bvh_stack_bound); nodes = ctypes array / pointer of BVHNode."""
    out = (C.c_int32 * 2)()
    n = len(nodes)
    st = lib().ctl_host_bvh_stack_bound(C.cast(nodes, C.c_void_p), n, int(root_value), out)
    if st != 0:
        raise CTLError("ctl_host_bvh_stack_bound: " + (lib().ctl_host_last_error() or b"").decode())
    return out[0], out[1]


def host_wide_trees(desc):
    """The 4-wide trees ctl_scene_upload builds from desc (ctl_host_wide_trees):
    (mesh nodes (n, 32) float32, per-mesh first node (n_meshes,) uint32,
    instance-tree nodes (m, 32) float32), 128-B WideNode records as float32 rows
    (the child / pad words keep their int bits)."""
    L = lib()
    nm, ns = C.c_uint64(0), C.c_uint64(0)
    _check(L.ctl_host_wide_trees(C.byref(desc), None, 0, C.byref(nm), None, None, 0, C.byref(ns)), None,
           "ctl_host_wide_trees: " + (L.ctl_host_last_error() or b"").decode())
    mesh = np.zeros((nm.value, 32), np.float32)
    wbase = np.zeros(desc.n_meshes, np.uint32)
    scene = np.zeros((ns.value, 32), np.float32)
    _check(L.ctl_host_wide_trees(C.byref(desc), mesh.ctypes.data, nm.value, C.byref(nm), wbase.ctypes.data,
                                 scene.ctypes.data, ns.value, C.byref(ns)), None,
           "ctl_host_wide_trees: " + (L.ctl_host_last_error() or b"").decode())
    return mesh, wbase, scene


class Tracer:
    """Per-GPU traversal context (InitializeKernel/UpdateKernel/IntersectBuffers)."""

    def __init__(self, device=0):
        self._L = lib()
        self._ctx = self._L.ctl_create(int(device))
        if not self._ctx:
            raise CTLError("ctl_create failed: " + (self._L.ctl_last_error(None) or b"").decode())
        self.device = device

    def close(self):
        if self._ctx:
            self._L.ctl_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload_scene(self, desc):
        _check(self._L.ctl_scene_upload(self._ctx, C.byref(desc)), self._ctx, "ctl_scene_upload")

    def update_scene(self, desc, dirty=0, stream=0):
        """UpdateKernel / DynamicScene::UpdateScene (ctl_scene_update): the scene constants
        always, plus the array groups in `dirty` (_abi.CTL_DIRTY_*)."""
        _check(self._L.ctl_scene_update(self._ctx, C.byref(desc), int(dirty), stream), self._ctx, "ctl_scene_update")

    def set_transform(self, node, xf16, stream=0):
        """DynamicScene::SetNodeTransform on the device (ctl_scene_set_transform):
        xf16 = row-major object->world 4x4."""
        m = _abi.Float4x4()
        m.m[:] = [float(x) for x in np.asarray(xf16, dtype=np.float32).reshape(16)]
        _check(self._L.ctl_scene_set_transform(self._ctx, int(node), C.byref(m), stream), self._ctx,
               "ctl_scene_set_transform")

    def generate_samples(self, pass_index, stream=0):
        _check(self._L.ctl_sampler_generate(self._ctx, int(pass_index), stream), self._ctx, "ctl_sampler_generate")

    def intersect_buffers(self, n, rays_ptr, hits_ptr, any_hit=False, stream=0):
        _check(self._L.ctl_intersect(self._ctx, int(n), rays_ptr, hits_ptr, 1 if any_hit else 0, stream),
               self._ctx, "ctl_intersect")

    def occluded(self, n, rays_ptr, out_ptr, any_hit=False, stream=0):
        """KernelDynamicScene::Occluded(ray, 0, ray.tmax) per ray into uint32 out
        (ctl_occluded): the reference's closest-hit form or the any-hit query."""
        _check(self._L.ctl_occluded(self._ctx, int(n), rays_ptr, out_ptr, 1 if any_hit else 0, stream),
               self._ctx, "ctl_occluded")

    def intersect_stats(self, n, rays_ptr, hits_ptr, any_hit=False, stream=0):
        out = (C.c_uint64 * 4)()
        _check(self._L.ctl_intersect_stats(self._ctx, int(n), rays_ptr, hits_ptr, 1 if any_hit else 0, out, stream),
               self._ctx, "ctl_intersect_stats")
        return list(out)

    def animate(self, anim, frame0, frame1, lerp, stream=0):
        """AnimatedMesh::k_ComputeState on the device: frame0/frame1 = (n_bones, 4, 4) bone matrices."""
        f0 = np.ascontiguousarray(frame0, dtype=np.float32).reshape(-1, 16)
        f1 = np.ascontiguousarray(frame1, dtype=np.float32).reshape(-1, 16)
        if f0.shape != f1.shape:
            raise ValueError("frames differ in bone count")
        _check(self._L.ctl_scene_animate(self._ctx, int(anim), f0.ctypes.data, f1.ctypes.data, f0.shape[0],
                                         float(lerp), stream), self._ctx, "ctl_scene_animate")

    def read_array(self, which, first, count, dtype, width):
        """Device scene array slice (ctl_scene_read) as a (count, width) numpy array."""
        out = np.zeros((count, width), dtype)
        _check(self._L.ctl_scene_read(self._ctx, int(which), int(first), int(count), out.ctypes.data), self._ctx,
               "ctl_scene_read")
        return out

    def wide_trees(self, desc):
        """The uploaded scene's 4-wide trees as the device holds them (after any
        refit by animate / set_transform), in host_wide_trees' layout; float
        nodes only (not CTL_SCENE_WIDE_QUANT)."""
        if desc.flags & _abi.CTL_SCENE_WIDE_QUANT:
            raise ValueError("wide_trees: quantized trees are read as host_wide_trees' decoded boxes")
        mesh0, wbase0, scene0 = host_wide_trees(desc)
        mesh = self.read_array(_abi.CTL_ARRAY_WIDE_BVH, 0, mesh0.shape[0], np.float32, 32)
        wbase = self.read_array(_abi.CTL_ARRAY_MESH_WIDE_BASE, 0, wbase0.size, np.uint32, 1).reshape(-1)
        scene = self.read_array(_abi.CTL_ARRAY_SCENE_WIDE_BVH, 0, scene0.shape[0], np.float32, 32)
        return mesh, wbase, scene

    def rays_traced(self):
        return int(self._L.ctl_rays_traced(self._ctx))

    def reset_rays(self, stream=0):
        _check(self._L.ctl_reset_rays(self._ctx, stream), self._ctx, "ctl_reset_rays")

    def image_resolve(self, fb_ptr, width, height, out_ptr, splat_scale=0.0, stream=0):
        """applyImagePipeline without filter/post-process: RGBA8 sRGB output (ImagePipeline.cu)."""
        _check(self._L.ctl_image_resolve(self._ctx, fb_ptr, width, height, float(splat_scale), out_ptr, stream),
               self._ctx, "ctl_image_resolve")

    def variance_add_pass(self, fb_ptr, width, height, tile_samples, var_ptr, splat_scale=0.0, tile_size=64,
                          stream=0):
        """PixelVarianceBuffer::AddPass; tile_samples = uint8 samples per tile this pass."""
        flags = np.ascontiguousarray(tile_samples, dtype=np.uint8)
        _check(self._L.ctl_variance_add_pass(self._ctx, fb_ptr, width, height, float(splat_scale), int(tile_size),
                                             flags.ctypes.data, var_ptr, stream), self._ctx, "ctl_variance_add_pass")

    def variance_stats(self, var_ptr, n, err_ptr=None, variance_ptr=None, average_ptr=None, stream=0):
        _check(self._L.ctl_variance_stats(self._ctx, var_ptr, int(n), err_ptr, variance_ptr, average_ptr, stream),
               self._ctx, "ctl_variance_stats")

    def sync(self, stream=0):
        """Wait for the stream; raises CTLError if a traversal stack overflowed since the last reset_rays."""
        _check(self._L.ctl_sync(self._ctx, stream), self._ctx, "ctl_sync")

    def stack_bound(self):
        """Worst-case traversal stack (entries per lane) of the uploaded scene."""
        return int(self._L.ctl_scene_stack_bound(self._ctx))

    def fb_reduce(self, comm, fb_ptr, out_ptr, n_pixels, root=0, stream=0):
        """Sum every rank's PixelData framebuffer fb into out on the root (ctl_fb_reduce
        over an RCCL communicator from comm_init_all / comm_init_rank or the caller's);
        fb is only read, so it may be called after any step."""
        _check(self._L.ctl_fb_reduce(self._ctx, comm, fb_ptr, out_ptr, int(n_pixels), int(root), stream), self._ctx,
               "ctl_fb_reduce")


def comm_unique_id():
    """ncclGetUniqueId bytes (ctl_comm_unique_id) for comm_init_rank on every rank."""
    buf = (C.c_uint8 * CTL_COMM_ID_BYTES)()
    if lib().ctl_comm_unique_id(buf) != 0:
        raise CTLError("ctl_comm_unique_id failed")
    return bytes(buf)


def comm_init_rank(nranks, uid, rank, device):
    """One RCCL communicator of a one-process-per-GPU job (ctl_comm_init_rank)."""
    out = C.c_void_p()
    buf = (C.c_uint8 * CTL_COMM_ID_BYTES).from_buffer_copy(uid)
    if lib().ctl_comm_init_rank(C.byref(out), int(nranks), buf, int(rank), int(device)) != 0:
        raise CTLError("ctl_comm_init_rank failed")
    return out.value


def comm_init_all(devices):
    """RCCL communicators of one process driving `devices` (ctl_comm_init_all)."""
    n = len(devices)
    out = (C.c_void_p * n)()
    devs = (C.c_int32 * n)(*devices)
    if lib().ctl_comm_init_all(out, n, devs) != 0:
        raise CTLError("ctl_comm_init_all failed")
    return list(out)


def comm_destroy(comm):
    if lib().ctl_comm_destroy(comm) != 0:
        raise CTLError("ctl_comm_destroy failed")


class PathTracer(Tracer):
    """PathTracer (Integrators/PathTracer.h:7-24) parameters and pass loop.
    Defaults: Direct=1, MaxPathLength=50, RRStartDepth=5 (PathTracer.h:16-19)."""

    def __init__(self, device=0, max_path_length=50, rr_start_depth=5, shadow_any_hit=True, tile_size=64,
                 num_ranks=1, rank=0, schedule="persistent"):
        """schedule: "persistent" (regenerating path kernel, default), "megakernel"
        (one thread per pixel path) or "wavefront"; all bit-identical."""
        super().__init__(device)
        flags = {"persistent": 0, "megakernel": CTL_PT_MEGAKERNEL, "wavefront": CTL_PT_WAVEFRONT}[schedule]
        self.params = PTParams(1, max_path_length, rr_start_depth, 1 if shadow_any_hit else 0, tile_size,
                               num_ranks, rank, flags)

    def do_pass(self, fb_ptr, pass_index, stream=0):
        """UpdateKernel's sampler regeneration + one render pass into fb (device PixelData[w*h])."""
        self.generate_samples(pass_index, stream)
        _check(self._L.ctl_render_pass(self._ctx, C.byref(self.params), fb_ptr, stream), self._ctx,
               "ctl_render_pass")

    def render_pass(self, fb_ptr, stream=0):
        """One pass with the sampler tables already generated (generate_samples)."""
        _check(self._L.ctl_render_pass(self._ctx, C.byref(self.params), fb_ptr, stream), self._ctx,
               "ctl_render_pass")

    def render_passes(self, fb_ptr, first_pass, n_passes, stream=0):
        """Passes first_pass .. first_pass + n_passes - 1 in one launch (ctl_render_passes):
        the framebuffer of n_passes do_pass calls."""
        _check(self._L.ctl_render_passes(self._ctx, C.byref(self.params), int(first_pass), int(n_passes), fb_ptr,
                                         stream), self._ctx, "ctl_render_passes")

    def last_pass_ms(self):
        """Device time of the last render pass (Tracer::getLastTimeSpentRenderingSec)."""
        ms = C.c_float()
        _check(self._L.ctl_last_pass_ms(self._ctx, C.byref(ms)), self._ctx, "ctl_last_pass_ms")
        return ms.value

    def camera_rays(self, rays_ptr=None, capacity=0, stream=0):
        """Primary rays of the current pass (sampler tables from generate_samples) as a
        ctl_ray batch; returns the ray count (call with rays_ptr=None to query it)."""
        n = C.c_int64()
        _check(self._L.ctl_camera_rays(self._ctx, C.byref(self.params), rays_ptr, int(capacity), C.byref(n), stream),
               self._ctx, "ctl_camera_rays")
        return n.value

    def pass_stats(self, fb_ptr, pass_index, stream=0):
        self.generate_samples(pass_index, stream)
        out = (C.c_uint64 * 4)()
        _check(self._L.ctl_render_pass_stats(self._ctx, C.byref(self.params), fb_ptr, out, stream), self._ctx,
               "ctl_render_pass_stats")
        return list(out)


class WavefrontPathTracer(Tracer):
    """WavefrontPathTracer (Integrators/PseudoRealtime/WavefrontPathTracer.h:24-67): path
    tracing over a DoubleRayBuffer, the batch traversal's second caller.  Defaults
    Direct=1, MaxPathLength=50, RRStartDepth=5 (WavefrontPathTracer.h:32-37)."""

    def __init__(self, device=0, direct=True, max_path_length=50, rr_start_depth=5, shadow_any_hit=False):
        super().__init__(device)
        self.params = WptParams(1 if direct else 0, max_path_length, rr_start_depth, 0,
                                _abi.CTL_WPT_SHADOW_ANY_HIT if shadow_any_hit else 0)
        self.passes_done = 0

    def do_pass(self, fb_ptr, pass_index, new_trace=False, stream=0):
        """Tracer::DoPass (Kernel/Tracer.h:209-248): UpdateKernel's sampler tables of
        `pass_index`, m_uPassesDone++ (reset by new_trace), then DoRender into fb."""
        if new_trace:
            self.passes_done = 0
        self.generate_samples(pass_index, stream)
        self.passes_done += 1
        self.params.passes_done = self.passes_done
        _check(self._L.ctl_wpt_render_pass(self._ctx, C.byref(self.params), fb_ptr, stream), self._ctx,
               "ctl_wpt_render_pass")

    def last_pass_ms(self):
        ms = C.c_float()
        _check(self._L.ctl_last_pass_ms(self._ctx, C.byref(ms)), self._ctx, "ctl_last_pass_ms")
        return ms.value


class PrimTracer(Tracer):
    """PrimTracer (Integrators/PrimTracer.h:11-22): one primary ray per pixel and
    a first-hit draw mode (default first_f, PrimTracer.cu:246), non-progressive
    (every pass clears the image, Tracer<false>::DoPass)."""

    def __init__(self, device=0, draw_mode="first_f", max_path_length=7, near=1.0, far=100000.0):
        super().__init__(device)
        mode = _abi.PRIM_DRAW_MODES.index(draw_mode) if isinstance(draw_mode, str) else int(draw_mode)
        self.params = _abi.PrimParams(mode, max_path_length, near, far, 0)

    def do_pass(self, fb_ptr, pass_index, depth_ptr=None, stream=0):
        """UpdateKernel's sampler regeneration + DoRender into fb (device PixelData[w*h]);
        depth_ptr: optional device float[w*h] for the D3D-normalised depth image."""
        self.generate_samples(pass_index, stream)
        _check(self._L.ctl_prim_pass(self._ctx, C.byref(self.params), fb_ptr, depth_ptr, stream), self._ctx,
               "ctl_prim_pass")

    def last_pass_ms(self):
        ms = C.c_float()
        _check(self._L.ctl_last_pass_ms(self._ctx, C.byref(ms)), self._ctx, "ctl_last_pass_ms")
        return ms.value


"""C5 shading cost by material class: the C5 scene (HostScene.generate(5)) with its
rough-dielectric and / or textured materials swapped for constant diffuse ones of
the same reflectance, 4 passes per ctl_render_passes launch each.  C5SPLIT_ONLY
(';'-separated case names) runs a subset, e.g. under rocprofv3 --pmc."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import torch
import cudatracerlib_amd as ctl

hs = ctl.HostScene().generate(5, 1.0, 1920, 1080)
desc = hs.compile(threads=16)
n = desc.n_materials
orig = [ctl.Material.from_buffer_copy(desc.materials[i]) for i in range(n)]


def variant(keep_rough, keep_tex):
    out = []
    for m in orig:
        rough = m.bsdf_type != ctl._abi.CTL_BSDF_DIFFUSE
        tex = m.bsdf_type == ctl._abi.CTL_BSDF_DIFFUSE and m.texture != 0xFFFFFFFF
        if (rough and not keep_rough) or (tex and not keep_tex):
            d = ctl.diffuse_material(0.5, 0.5, 0.5, two_sided=bool(m.two_sided))
            d.node_light_index = m.node_light_index
            out.append(d)
        else:
            out.append(ctl.Material.from_buffer_copy(m))
    return (ctl.Material * n)(*out)


fb = torch.zeros((1920 * 1080, 7), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
nt = desc.n_textures
texs = [ctl._abi.Texture.from_buffer_copy(desc.textures[i]) for i in range(nt)]
print("texture filters:", [t.filter for t in texs], "levels:", [t.levels for t in texs])


def filtered(f):
    out = [ctl._abi.Texture.from_buffer_copy(t) for t in texs]
    for t in out:
        if f is not None:
            t.filter = f
    return (ctl._abi.Texture * nt)(*out)


def with_unused_textured(mats):
    """the same materials plus one unused textured material: the scene runs the
    full-shading kernel while every hit shades constant diffuse"""
    t = ctl.Material.from_buffer_copy(mats[0])
    t.texture = 0
    out = [ctl.Material.from_buffer_copy(m) for m in mats] + [t]
    return (ctl.Material * (n + 1))(*out)


CASES = (("C5", 1, 1, None), ("rough only", 1, 0, None), ("textures only", 0, 1, None),
         ("tex trilinear", 0, 1, ctl._abi.CTL_TEX_TRILINEAR), ("tex EWA", 0, 1, ctl._abi.CTL_TEX_EWA),
         ("tex bilinear", 0, 1, ctl._abi.CTL_TEX_BILINEAR), ("neither", 0, 0, None),
         ("neither, full", 0, 0, "full"))
only = [x for x in os.environ.get("C5SPLIT_ONLY", "").split(";") if x]
for name, kr, kt, flt in CASES:
    if only and name not in only:
        continue
    d = type(desc).from_buffer_copy(desc)
    mats = variant(kr, kt)
    if flt == "full":
        mats = with_unused_textured(mats)
        d.n_materials = n + 1
        flt = None
    d.materials = mats
    tx = filtered(flt)
    d.textures = tx
    pt = ctl.PathTracer(0, max_path_length=50, rr_start_depth=5, shadow_any_hit=True, tile_size=64)
    pt.upload_scene(d)
    pt.render_passes(fb.data_ptr(), 0, 4, s)
    torch.cuda.synchronize()
    pt.reset_rays(s)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(4):
        pt.render_passes(fb.data_ptr(), 10 + 4 * k, 4, s)
    e1.record(); pt.sync(s)
    ms = e0.elapsed_time(e1) / 16
    print(f"{name:14s} {ms:.3f} ms/pass {pt.rays_traced() / 16 / ms / 1e3:.1f} Mrays/s", flush=True)
    pt.close()

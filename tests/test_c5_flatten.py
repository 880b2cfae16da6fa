"""C5 materials through the drop-in: a material set
flattened field by field from the reference's records, the way a maintainer's
flattenMaterials writes it, uploaded through ctl_scene_upload and rendered
bit-exact against the oracle; and what the upload refuses.

Reference records: Material (Engine/Material.h:38), diffuse / roughdielectric
(SceneTypes/BSDF_Simple.h:127), ImageTexture + TextureMapping2D
(SceneTypes/Texture.h:15-40,159-183), KernelMIPMap (Engine/MIPMap_device.h:57-82),
AlphaBlendData (Engine/Material.h:14-30)."""
import ctypes as C

import numpy as np
import pytest

from helpers import oracle_render

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

EDIFF, EGLOSSY_R, EGLOSSY_T = 0x2, 0x8, 0x10


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def weight_lut():
    """KernelMIPMap::m_weightLut (MIPMap.cpp:88-93): exp(-2 r^2) - exp(-2) over 64
    entries, fp32 of the fp64 exponential (the oracle's and the library's cr_exp)."""
    r2 = np.arange(64, dtype=np.float32) / np.float32(63)
    e = np.exp((np.float32(-2.0) * r2).astype(np.float64)).astype(np.float32)
    return e - np.float32(np.exp(np.float64(np.float32(-2.0))))


def pyramid(rng, w, h):
    """A MIP pyramid given level by level (any data: the levels are part of the
    scene, as the reference's FreeImage-resampled ones are)."""
    levels, data, l = [], [], 0
    while (w >> l) >= 1 and (h >> l) >= 1 and l < 16:
        levels.append(sum(x.size for x in data))
        data.append(rng.integers(0, 2 ** 32, size=(h >> l) * (w >> l), dtype=np.uint64).astype(np.uint32))
        l += 1
    return levels, np.concatenate(data)


def flat_texture(ctl, mapping, scale, w, h, filt, wrap, base):
    t = ctl._abi.Texture()
    t.mapping[:] = mapping                   # TextureMapping2D m11 m12 m13 m21 m22 m23
    t.set_id = 0
    t.scale[:] = scale                       # ImageTexture::m_scale
    t.width, t.height = w, h                 # KernelMIPMap m_uWidth / m_uHeight
    t.filter, t.wrap = filt, wrap            # m_uFilterMode / m_uWrapMode, the reference's enum order
    t.weight_lut[:] = list(weight_lut())
    return t


def flat_scene(ctl):
    """Geometry and lights from the host compiler; materials, textures and texels
    replaced by hand-flattened records."""
    s = ctl.HostScene()
    verts, idx, mi, uv = [], [], [], []
    for k in range(6):
        x0 = -3.0 + k
        b = len(verts)
        verts += [(x0, -1, 0), (x0 + 0.9, -1, 0.25 * k), (x0 + 0.9, 1, 0.25 * k), (x0, 1, 0)]
        uv += [(0, 0), (1.5, 0), (1.5, 1.2), (0, 1.2)]
        idx += [(b, b + 1, b + 2), (b, b + 2, b + 3)]
        mi += [k, k]
    b = len(verts)
    verts += [(-2, 3, -2), (2, 3, -2), (2, 3, 2), (-2, 3, 2)]
    uv += [(0, 0)] * 4
    idx += [(b, b + 2, b + 1), (b, b + 3, b + 2)]
    mi += [6, 6]
    placeholder = [ctl.diffuse_material(0.5, 0.5, 0.5) for _ in range(7)]
    m = s.add_mesh(np.array(verts, np.float32), np.array(idx, np.uint32), placeholder,
                   mat_index=np.array(mi, np.uint8), uvs=np.array(uv, np.float32))
    node = s.add_node(m)
    s.add_area_light(node, 6, (25.0, 25.0, 25.0))
    s.set_camera((0.3, 0.2, -6.0), (0, 0, 0), (0, 1, 0), 60.0, 96, 64)
    d = s.compile()
    light_index = d.materials[6].node_light_index

    rng = np.random.default_rng(9)
    texels, recs = [], []
    for (w, h, filt, wrap, mapping) in [(64, 64, 3, 0, (3.0, 0.5, 0.1, -0.2, 2.0, 0.3)),    # trilinear, repeat
                                        (32, 64, 2, 2, (1.0, 0.0, 0.0, 0.0, 1.0, 0.0)),     # EWA, mirror
                                        (16, 16, 1, 1, (2.0, 0.0, 0.5, 0.0, 2.0, 0.0))]:    # bilinear, clamp
        base = sum(x.size for x in texels)
        offs, data = pyramid(rng, w, h)
        t = flat_texture(ctl, mapping, (0.9, 0.8, 1.0), w, h, filt, wrap, base)
        t.levels = len(offs)
        for l, o in enumerate(offs):
            t.offsets[l] = base + o
        recs.append(t)
        texels.append(data)
    tex = (ctl._abi.Texture * len(recs))(*recs)
    tex_data = np.concatenate(texels)

    mats = (ctl.Material * 7)()
    for k in range(7):
        c = mats[k]
        c.node_light_index = 0xFFFFFFFF
        c.texture = c.alpha_texture = 0xFFFFFFFF
    for k, ti in enumerate((0, 1, 2)):                     # diffuse with an ImageTexture m_reflectance
        c = mats[k]
        c.bsdf_type, c.combined_type, c.two_sided = 1, EDIFF, 1
        c.texture = ti
    mats[2].alpha_state, mats[2].alpha_threshold = 6, 0.5     # ReflectanceMap_Alpha on the bilinear one
    for k, (dist, eta, au, av) in ((3, (0, 1.5, 0.1, 0.1)), (4, (1, 1.33, 0.3, 0.15))):   # roughdielectric
        c = mats[k]
        c.bsdf_type, c.combined_type, c.two_sided = 5, EGLOSSY_R | EGLOSSY_T, 0
        c.reflectance[:] = [1.0, 0.95, 0.9]               # ConstantTexture m_specularReflectance
        c.transmittance[:] = [0.9, 1.0, 1.0]              # ConstantTexture m_specularTransmittance
        c.distribution = dist                              # MicrofacetDistribution::EType
        c.eta = eta
        c.inv_eta = float(np.float32(1.0) / np.float32(eta))   # roughdielectric::Update: m_invEta = 1 / m_eta
        c.alpha_u, c.alpha_v = au, av                     # ConstantTexture m_alphaU / m_alphaV
        c.sample_visible = 1                              # getSampleVisible(Beckmann / GGX, true)
    for k, rgb in ((5, (0.7, 0.6, 0.5)), (6, (0.8, 0.8, 0.8))):   # constant diffuse, the emitter's material
        c = mats[k]
        c.bsdf_type, c.combined_type, c.two_sided = 1, EDIFF, 1
        c.reflectance[:] = list(rgb)
    mats[6].node_light_index = light_index                # Material::NodeLightIndex from CreateNode
    d.materials, d.n_materials = C.cast(mats, C.POINTER(ctl.Material)), 7
    d.textures, d.n_textures = C.cast(tex, C.POINTER(ctl._abi.Texture)), len(recs)
    d.tex_data, d.n_tex_data = tex_data.ctypes.data_as(C.POINTER(C.c_uint32)), tex_data.size
    keep = (s, mats, tex, tex_data)
    return keep, d


def render(ctl, desc, dev, passes, w, h):
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(desc)
        pt.params = ctl.PTParams(1, 8, 3, 1, 64, 1, 0, 0)
        fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        for p in range(passes):
            pt.do_pass(fb.data_ptr(), p)
        pt.sync()
        return fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()


def test_hand_flattened_c5_materials_bit_exact(ctl, orc, dev):
    keep, d = flat_scene(ctl)
    got, grays = render(ctl, d, dev, 3, 96, 64)
    want, wrays = oracle_render(orc, d, ctl.PTParams(1, 8, 3, 1, 64, 1, 0, 0), 3, 96, 64)
    assert grays == wrays
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert want[:, 0].std() > 0.01
    del keep


@pytest.mark.parametrize("field,value,msg", [
    ("bsdf_type", 6, "only diffuse and roughdielectric"),             # conductor, TYPE_FUNC(6)
    ("sample_visible", 0, "visible-normal sampling"),
    ("distribution", 2, "Beckmann/GGX"),                              # EPhong
    ("texture", 7, "texture index out of range"),
    ("alpha_state", 3, "alpha state"),                                # ColorCompare (unsupported)
])
def test_upload_refuses_unsupported_material(ctl, dev, field, value, msg):
    keep, d = flat_scene(ctl)
    mats = keep[1]
    k = 0 if field in ("texture", "alpha_state") else 3
    setattr(mats[k], field, value)
    pt = ctl.PathTracer(0)
    try:
        with pytest.raises(ctl.CTLError, match=msg):
            pt.upload_scene(d)
    finally:
        pt.close()
    del keep


def test_upload_refuses_bad_texture_record(ctl, dev):
    keep, d = flat_scene(ctl)
    tex = keep[2]
    tex[1].levels = 0
    pt = ctl.PathTracer(0)
    try:
        with pytest.raises(ctl.CTLError, match="invalid texture record"):
            pt.upload_scene(d)
    finally:
        pt.close()
    del keep

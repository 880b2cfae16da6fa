"""Environment lighting (InfiniteLight: SceneTypes/Light.h:294-367,
Light.cu:350-511, Light.cpp:10-58; the miss terms of PathTracer.cu:98-111,
WavefrontPathTracer.cu:144-157 and PrimTracer.cu:102).

CPU: the host compile's sampling tables equal the oracle's restatement of the
InfiniteLight constructor bit for bit, and the restated sampling routine is a
normalized density that agrees with pdfDirect along its own samples.
GPU: every schedule (persistent, wavefront, megakernel), the
WavefrontPathTracer and the PrimTracer, with and without next-event
estimation, bit-exact against the oracle on open scenes lit by an
environment map.  The reference ships no InfiniteLight fixtures; parity of the
restatement itself is pinned by the reference's formulas only (parity
unpinned for this light beyond the self-consistency checks below)."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import oracle_render, tie_rule


def env_image(w=32, h=16, seed=5):
    """A sky gradient with a bright sun spot and noise (RGBA8, r in the low byte)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    r = 20 + 50 * (1 - yy / h) + rng.integers(0, 20, size=(h, w))
    g = 30 + 50 * (1 - yy / h) + rng.integers(0, 20, size=(h, w))
    b = 60 + 60 * (1 - yy / h) + rng.integers(0, 20, size=(h, w))
    sun = ((xx - w // 3) ** 2 + (yy - h // 4) ** 2) <= 2
    r, g, b = np.where(sun, 255, r), np.where(sun, 250, g), np.where(sun, 230, b)
    return (np.clip(r, 0, 255).astype(np.uint32) | (np.clip(g, 0, 255).astype(np.uint32) << 8) |
            (np.clip(b, 0, 255).astype(np.uint32) << 16) | (255 << 24)).astype(np.uint32)


def rotation(axis, angle):
    a = np.asarray(axis, np.float64)
    a /= np.linalg.norm(a)
    c, s = np.cos(angle), np.sin(angle)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return (np.eye(3) * c + s * K + (1 - c) * np.outer(a, a)).astype(np.float32)


ROT = rotation((0.3, 1.0, -0.2), 1.1)   # m_worldTransform of the rotated-map cases


def env_scene(ctl, textured=False, w=64, h=48, env_filter=None, with_area_light=True, scale=(2.0, 1.8, 1.6),
              rot=None):
    """An open scene: ground plane, two boxes (one rough glass or textured when
    `textured`), an area light; the camera sees the sky above the horizon."""
    s = ctl.HostScene()
    flt = ctl._abi.CTL_TEX_BILINEAR if env_filter is None else env_filter
    env_tex = s.add_texture(env_image(), filter=flt)
    mats = [ctl.diffuse_material(0.6, 0.6, 0.55), ctl.diffuse_material(0.7, 0.3, 0.2),
            ctl.diffuse_material(0.8, 0.8, 0.8)]
    if textured:
        rng = np.random.default_rng(7)
        img = rng.integers(0, 2 ** 32, size=(32, 32), dtype=np.uint64).astype(np.uint32)
        t = s.add_texture(img, filter=ctl._abi.CTL_TEX_TRILINEAR)
        mats[1] = ctl.diffuse_material(0.5, 0.5, 0.5, texture=t)
        mats.append(ctl.roughdielectric_material(1, 1.5, 0.2))
    verts, idx, mi, uv = [], [], [], []

    def quad(p, k):
        b = len(verts)
        verts.extend(p)
        uv.extend([(0, 0), (1, 0), (1, 1), (0, 1)])
        idx.extend([(b, b + 1, b + 2), (b, b + 2, b + 3)])
        mi.extend([k, k])

    def box(x0, y0, z0, x1, y1, z1, k):
        quad([(x0, y1, z0), (x0, y1, z1), (x1, y1, z1), (x1, y1, z0)], k)   # top
        quad([(x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0)], k)   # front
        quad([(x1, y0, z0), (x1, y0, z1), (x1, y1, z1), (x1, y1, z0)], k)   # right
        quad([(x0, y0, z1), (x0, y0, z0), (x0, y1, z0), (x0, y1, z1)], k)   # left
        quad([(x1, y0, z1), (x0, y0, z1), (x0, y1, z1), (x1, y1, z1)], k)   # back

    quad([(-8, 0, -8), (-8, 0, 8), (8, 0, 8), (8, 0, -8)], 0)
    box(-2.0, 0.0, -0.5, -0.6, 1.4, 0.9, 1)
    box(0.4, 0.0, -1.0, 1.8, 0.9, 0.4, 3 if textured else 1)
    quad([(-0.8, 3.0, -0.8), (0.8, 3.0, -0.8), (0.8, 3.0, 0.8), (-0.8, 3.0, 0.8)], 2)   # light, facing down
    m = s.add_mesh(np.array(verts, np.float32), np.array(idx, np.uint32), mats, mat_index=np.array(mi, np.uint8),
                   uvs=np.array(uv, np.float32))
    node = s.add_node(m)
    if with_area_light:
        s.add_area_light(node, 2, (12.0, 12.0, 12.0))
    s.set_environment(env_tex, scale)
    if rot is not None:
        s.set_environment_transform(rot)
    s.set_camera((0.5, 1.6, -6.0), (0.0, 1.2, 0.0), (0, 1, 0), 60.0, w, h)
    return s, s.compile()


def test_env_compile_record(ctl):
    s, d = env_scene(ctl)
    assert d.env_map_index == d.n_lights - 1 == 1
    assert d.lights[d.env_map_index].kind == ctl._abi.CTL_LIGHT_INFINITE
    assert d.lights[0].kind == ctl._abi.CTL_LIGHT_DIFFUSE
    e = d.env.contents
    assert (e.size[0], e.size[1]) == (32.0, 16.0)
    assert list(e.scale) == pytest.approx([2.0, 1.8, 1.6])
    # Update(): scene sphere = box centre, |box size| / 1.5
    lo, hi = np.array(d.box_min[:]), np.array(d.box_max[:])
    assert np.allclose(e.scene_center[:], (lo + hi) / 2)
    assert e.scene_radius == pytest.approx(np.linalg.norm(hi - lo) / 1.5, rel=1e-6)
    # the light CDF: unit weights over area light + environment
    assert list(d.light_cdf[:2]) == [0.5, 1.0]
    s.set_environment(None)
    d2 = s.compile()
    assert d2.env_map_index == 0xFFFFFFFF and d2.n_lights == 1 and not d2.env


def test_env_tables_match_oracle(ctl, orc):
    """InfiniteLight::InfiniteLight (Light.cpp:10-58): the compile's column / row
    CDFs, row weights, normalization and pixel size, bit-exact."""
    s, d = env_scene(ctl)
    e = d.env.contents
    w, h = int(e.size[0]), int(e.size[1])
    n = (w + 1) * h + (h + 1) + h
    assert d.n_env_data == n
    got = np.ctypeslib.as_array(d.env_data, shape=(n,)).copy()
    want = np.zeros(n, np.float32)
    want3 = np.zeros(3, np.float32)
    orc.oracle_env_tables(C.byref(d.textures[e.texture]), d.tex_data, oracle.ptr(want), oracle.ptr(want3))
    assert (e.cdf_cols, e.cdf_rows, e.row_weights) == (0, (w + 1) * h, (w + 1) * h + h + 1)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(np.array([e.normalization, e.pixel_size[0], e.pixel_size[1]], np.float32).view(np.uint32),
                          want3.view(np.uint32))
    cols = want[:(w + 1) * h].reshape(h, w + 1)
    assert (np.diff(cols, axis=1) >= 0).all() and (cols[:, -1] == 1).all() and (cols[:, 0] == 0).all()


def test_env_sampling_is_a_normalized_density(ctl, orc):
    """The restated internalSampleDirection / internalPdfDirection: on the half
    of the sphere where pdfDirect's lookups are not clamped it integrates to the
    sampler's probability of that half, agrees with the density the sampler
    reports along its own samples, and the sampler favours the bright texels."""
    _, d = env_scene(ctl)
    rng = np.random.default_rng(11)
    n = 200_000
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    out = np.zeros((n, 4), np.float32)
    orc.oracle_env_eval(C.byref(d), n, oracle.ptr(np.ascontiguousarray(v)), oracle.ptr(out))
    # over the d.x > 0 hemisphere (where the lookup is not clamped, see below)
    # the pdf integrates to the sampler's share of that half
    east = v[:, 0] > 0
    integral = out[east, 0].mean() * 2 * np.pi
    e = d.env.contents
    cols = np.ctypeslib.as_array(d.env_data, shape=(d.n_env_data,))[:(32 + 1) * 16].reshape(16, 33)
    rows = np.ctypeslib.as_array(d.env_data, shape=(d.n_env_data,))[e.cdf_rows:e.cdf_rows + 17]
    share = float(((cols[:, 16] - cols[:, 0]) * np.diff(rows)).sum())   # columns 0..15 = phi in (0, pi)
    assert abs(integral - share) < 0.03 * share, (integral, share)
    assert (out[:, 1:] >= 0).all()
    m = 20_000
    smp = rng.random((m, 2), dtype=np.float32)
    so = np.zeros((m, 7), np.float32)
    orc.oracle_env_sample(C.byref(d), m, oracle.ptr(smp), oracle.ptr(so))
    assert np.allclose(np.linalg.norm(so[:, :3], axis=1), 1.0, atol=1e-5)
    back = np.zeros((m, 4), np.float32)
    orc.oracle_env_eval(C.byref(d), m, oracle.ptr(np.ascontiguousarray(so[:, :3])), oracle.ptr(back))
    rel = np.abs(back[:, 0] - so[:, 3]) / so[:, 3]
    # internalPdfDirection maps atan2(d.x, -d.z) in (-pi, 0) to u < 0 and reads
    # the map through Sample(0, x, y), which clamps instead of wrapping: for
    # d.x < 0 the reference's pdf reads column 0.  Restated as is; the sampler
    # and pdfDirect agree on the d.x > 0 half.
    east = so[:, 0] > 1e-3
    assert np.quantile(rel[east], 0.9) < 1e-3
    assert np.quantile(rel[~east], 0.5) > 1e-2
    # importance sampling: the sun (brightest texels) draws far more than its area share
    sun = np.zeros((m,), bool)
    u = np.arctan2(so[:, 0], -so[:, 2]) / (2 * np.pi) % 1.0
    t = np.arccos(np.clip(so[:, 1], -1, 1)) / np.pi
    sun = (np.abs(u * 32 - (32 // 3 + 0.5)) < 2.0) & (np.abs(t * 16 - (16 // 4 + 0.5)) < 2.0)
    assert sun.mean() > 2 * (16 / (32 * 16))


def test_env_world_transform_rotates_the_map(ctl, orc):
    """m_worldTransform (Light.h:307; TransformDirection / TransformDirectionTranspose,
    Light.cu:342-510): with rotation R the radiance and pdf seen along R v are
    those of the identity map along v, and the sampled directions are R times
    the identity's (up to fp32 rounding of the rotation)."""
    s0, d0 = env_scene(ctl)
    s1, d1 = env_scene(ctl, rot=ROT)
    e0, e1 = d0.env.contents, d1.env.contents
    assert np.array_equal(np.array(e0.world, np.float32), np.eye(3, dtype=np.float32))
    assert np.array_equal(np.array(e1.world, np.float32), ROT)
    rng = np.random.default_rng(3)
    n = 50_000
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    rv = np.ascontiguousarray((v.astype(np.float64) @ ROT.T.astype(np.float64)).astype(np.float32))
    o0 = np.zeros((n, 4), np.float32)
    o1 = np.zeros((n, 4), np.float32)
    orc.oracle_env_eval(C.byref(d0), n, oracle.ptr(np.ascontiguousarray(v)), oracle.ptr(o0))
    orc.oracle_env_eval(C.byref(d1), n, oracle.ptr(rv), oracle.ptr(o1))
    # away from the lat-long seam and the poles the lookups agree to rounding
    keep = (np.abs(v[:, 0]) > 0.02) & (np.abs(v[:, 1]) < 0.98)
    rel = np.abs(o1[keep] - o0[keep]) / np.maximum(np.abs(o0[keep]), 1e-6)
    assert np.quantile(rel, 0.99) < 2e-2 and np.median(rel) < 1e-4
    m = 5000
    smp = rng.random((m, 2), dtype=np.float32)
    s0o = np.zeros((m, 7), np.float32)
    s1o = np.zeros((m, 7), np.float32)
    orc.oracle_env_sample(C.byref(d0), m, oracle.ptr(smp), oracle.ptr(s0o))
    orc.oracle_env_sample(C.byref(d1), m, oracle.ptr(smp), oracle.ptr(s1o))
    assert np.allclose(s1o[:, :3], s0o[:, :3] @ ROT.T, atol=1e-5)
    assert np.array_equal(s1o[:, 3:].view(np.uint32), s0o[:, 3:].view(np.uint32))   # pdf and value: local


def test_set_environment_rejects_bad_texture(ctl):
    s = ctl.HostScene()
    v = np.array([(0, 0, 0), (1, 0, 0), (0, 1, 0)], np.float32)
    s.add_mesh(v, np.array([(0, 1, 2)], np.uint32), [ctl.diffuse_material(0.5, 0.5, 0.5)])
    s.add_node(0)
    s.set_camera((0, 0, -3), (0, 0, 0), (0, 1, 0), 60.0, 8, 8)
    s.set_environment(3)
    with pytest.raises(RuntimeError):
        s.compile()


# ---- GPU parity ---------------------------------------------------------------

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def render_gpu(ctl, desc, params, passes, w, h, dev, first_pass=0):
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(desc)
        pt.params = params
        fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        for p in range(first_pass, first_pass + passes):
            pt.do_pass(fb.data_ptr(), p)
        torch.cuda.synchronize()
        return fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()


MODES = {"persistent": 0, "megakernel": "CTL_PT_MEGAKERNEL", "wavefront": "CTL_PT_WAVEFRONT"}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("direct", [1, 0])
@pytest.mark.parametrize("textured", [False, True])
def test_render_env_bit_exact(ctl, orc, dev, mode, direct, textured):
    """PathTrace<DIRECT> with an environment map: NEE picks the environment
    (importance-sampled direction, MIS against the BSDF) or the area light;
    escaping paths add misWeight * cf * EvalEnvironment(r)."""
    w, h = 64, 48
    _, d = env_scene(ctl, textured=textured, w=w, h=h)
    flags = 0 if mode == "persistent" else getattr(ctl, MODES[mode])
    p = ctl.PTParams(direct, 8, 3, 1, 64, 1, 0, flags)
    want, wrays = oracle_render(orc, d, p, 2, w, h)
    got, grays = render_gpu(ctl, d, p, 2, w, h, dev)
    assert grays == wrays
    assert np.isfinite(got).all()
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])
    # the sky shows up: without the environment the image differs
    s2, _ = env_scene(ctl, textured=textured, w=w, h=h)
    s2.set_environment(None)
    plain, _ = oracle_render(orc, s2.compile(), p, 2, w, h)
    assert not np.array_equal(plain.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("direct", [1, 0])
def test_render_env_rotated_bit_exact(ctl, orc, dev, mode, direct):
    """A rotated environment map (InfiniteLight::m_worldTransform): sampleDirect
    turns its directions into the world, pdfDirect and evalEnvironment turn the
    world direction back (Light.cu:355, 369, 483)."""
    w, h = 64, 48
    _, d = env_scene(ctl, textured=True, w=w, h=h, rot=ROT)
    flags = 0 if mode == "persistent" else getattr(ctl, MODES[mode])
    p = ctl.PTParams(direct, 8, 3, 1, 64, 1, 0, flags)
    want, wrays = oracle_render(orc, d, p, 2, w, h)
    got, grays = render_gpu(ctl, d, p, 2, w, h, dev)
    assert grays == wrays
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])
    _, d0 = env_scene(ctl, textured=True, w=w, h=h)
    plain, _ = oracle_render(orc, d0, p, 2, w, h)
    assert not np.array_equal(plain.view(np.uint32), want.view(np.uint32))   # the rotation shows


@pytest.mark.gpu
def test_upload_refuses_non_rotation_env_transform(ctl, dev):
    s, d = env_scene(ctl, rot=np.diag([2.0, 1.0, 1.0]).astype(np.float32))
    pt = ctl.PathTracer(0)
    try:
        with pytest.raises(ctl.CTLError, match="rotation"):
            pt.upload_scene(d)
    finally:
        pt.close()


@pytest.mark.gpu
def test_render_env_only_light(ctl, orc, dev):
    """The environment as the only emitter (light CDF = [1]): every NEE sample
    goes to the map."""
    w, h = 48, 32
    _, d = env_scene(ctl, w=w, h=h, with_area_light=False)
    assert d.n_lights == 1 and d.env_map_index == 0
    p = ctl.PTParams(1, 6, 3, 0, 64, 1, 0, 0)
    want, wrays = oracle_render(orc, d, p, 2, w, h)
    got, grays = render_gpu(ctl, d, p, 2, w, h, dev)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [1, 0])
@pytest.mark.parametrize("rotated", [False, True])
def test_wpt_env_bit_exact(ctl, orc, dev, direct, rotated):
    """WavefrontPathTracer (WavefrontPathTracer.cu:51-157) with the environment:
    sampleEmitterDirect over both lights, the escaped-ray term with its
    pathDepth / prev_normal MIS."""
    w, h = 64, 48
    _, d = env_scene(ctl, textured=True, w=w, h=h, rot=ROT if rotated else None)
    wt = ctl.WavefrontPathTracer(0, direct=direct, max_path_length=8, rr_start_depth=3)
    try:
        wt.upload_scene(d)
        fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
        wt.reset_rays()
        for k in range(2):
            wt.do_pass(fb.data_ptr(), 1 + k, new_trace=(k == 0))
        torch.cuda.synchronize()
        got, grays = fb.cpu().numpy(), wt.rays_traced()
    finally:
        wt.close()
    want = np.zeros((w * h, 7), np.float32)
    wrays = 0
    for k in range(2):
        wrays += orc.oracle_wpt_render_pass(C.byref(d), direct, 8, 3, k + 1, 1 + k, oracle.ptr(want), tie_rule(d), 0)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("env_filter", ["CTL_TEX_BILINEAR", "CTL_TEX_TRILINEAR", "CTL_TEX_EWA"])
@pytest.mark.parametrize("mode", ["first_f_direct", "uv"])
@pytest.mark.parametrize("rotated", [False, True])
def test_prim_env_bit_exact(ctl, orc, dev, env_filter, mode, rotated):
    """PrimTracer misses: EvalEnvironment(r, rX, rY), the map filtered over the
    primary ray differentials' footprint; first_f_direct also samples the
    environment for its UniformSampleOneLight."""
    _, d = env_scene(ctl, w=64, h=48, env_filter=getattr(ctl._abi, env_filter), rot=ROT if rotated else None)
    mi = ctl._abi.PRIM_DRAW_MODES.index(mode)
    pt = ctl.PrimTracer(0, draw_mode=mi)
    try:
        pt.upload_scene(d)
        fb = torch.zeros((64 * 48, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        pt.do_pass(fb.data_ptr(), 3)
        pt.sync()
        got, grays = fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()
    prm = ctl.PrimParams(mi, 7, 1.0, 100000.0, 0)
    want = np.zeros((64 * 48, 7), np.float32)
    depth = np.zeros(64 * 48, np.float32)
    wrays = orc.oracle_prim_pass(C.byref(d), C.byref(prm), 3, oracle.ptr(want), oracle.ptr(depth), tie_rule(d), 0)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))
    assert (want[:, 2] > 0.3).sum() > 100   # the sky is in frame

"""GPU parity: the gfx950 kernels (through the C-ABI) against the oracle on the
same inputs.  Bar: bit-exact for hit index/node/t/bary and for the per-pixel
PixelData framebuffer (fp32 sums of identical per-sample values in identical
pass order)."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import binary_bvh, camera_rays, oracle_intersect, oracle_render, random_rays, select_bvh, tie_rule

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def tracer(ctl, dev):
    return ctl.PathTracer(0)


SCENES = {}


def scene(ctl, config, scale, w, h):
    key = (config, scale, w, h)
    if key not in SCENES:
        s = ctl.HostScene().generate(config, scale, w, h)
        SCENES[key] = (s, s.compile())
    return SCENES[key][1]


def gpu_intersect(tracer, desc, rays, any_hit, dev):
    tracer.upload_scene(desc)
    r = torch.from_numpy(rays).to(dev)
    h = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
    tracer.intersect_buffers(rays.shape[0], r.data_ptr(), h.data_ptr(), any_hit=any_hit)
    torch.cuda.synchronize()
    return h.cpu().numpy()


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.25), (3, 0.004)])
@pytest.mark.parametrize("kind", ["random", "camera"])
@pytest.mark.parametrize("bvh", ["wide", "wideq", "binary"])
def test_intersect_closest_bit_exact(ctl, orc, tracer, dev, config, scale, kind, bvh):
    d = select_bvh(scene(ctl, config, scale, 96, 64), bvh)
    rays = random_rays(d, 50000, seed=config) if kind == "random" else camera_rays(d, 96, 64, seed=config)
    if kind == "random":
        rays[::3, 3] = np.float32(d.ray_eps)      # some rays with tmin > 0
        rays[1::5, 7] = np.float32(5.0)           # and short tmax
    want = oracle_intersect(orc, d, rays, any_hit=False)
    got = gpu_intersect(tracer, d, rays, False, dev)
    assert (want[:, 2] >= 0).sum() > 100
    bad = np.nonzero((want != got).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:5]], got[bad[:5]])


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.25)])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_intersect_any_hit(ctl, orc, tracer, dev, config, scale, bvh):
    """Any-hit returns *a* hit (order dependent, TraceHelper.cu:675-679): the
    hit/miss decision must equal the oracle's, and the reported triangle must
    really be hit inside (tmin, tmax) at the reported t."""
    d = select_bvh(scene(ctl, config, scale, 96, 64), bvh)
    rays = random_rays(d, 30000, seed=5)
    rays[:, 7] = np.float32(np.linalg.norm(np.array(d.box_max[:]) - np.array(d.box_min[:])) * 0.3)
    want = oracle_intersect(orc, d, rays, any_hit=True)
    got = gpu_intersect(tracer, d, rays, True, dev)
    assert np.array_equal(want[:, 2] >= 0, got[:, 2] >= 0)
    closest = oracle_intersect(orc, d, rays, any_hit=False)
    assert np.array_equal(closest[:, 2] >= 0, got[:, 2] >= 0)
    hit = got[:, 2] >= 0
    t = got[hit, 0].view(np.float32)
    assert np.all(t >= closest[hit, 0].view(np.float32)) and np.all(t < rays[hit, 7])


def render_gpu(ctl, tracer, desc, params, passes, w, h, dev, first_pass=0):
    tracer.upload_scene(desc)
    tracer.params = params
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    tracer.reset_rays()
    for p in range(first_pass, first_pass + passes):
        tracer.do_pass(fb.data_ptr(), p)
    torch.cuda.synchronize()
    return fb.cpu().numpy(), tracer.rays_traced()


@pytest.mark.parametrize("config,scale,w,h,passes", [(1, 1.0, 64, 64, 4), (2, 0.25, 96, 64, 2), (3, 0.003, 64, 48, 2)])
@pytest.mark.parametrize("any_hit", [1, 0])
@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("bvh", ["wide", "wideq", "binary"])
def test_render_pass_bit_exact(ctl, orc, tracer, dev, config, scale, w, h, passes, any_hit, mode, bvh):
    d = select_bvh(scene(ctl, config, scale, w, h), bvh)
    p = ctl.PTParams(1, 50, 5, any_hit, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                                 "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, passes, w, h)
    got, grays = render_gpu(ctl, tracer, d, p, passes, w, h, dev)
    assert grays == wrays
    assert want[:, 6].min() == passes          # every pixel got every sample
    assert np.isfinite(got).all()
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.mark.parametrize("config,scale,w,h", [(1, 1.0, 64, 64), (2, 0.25, 96, 64), (3, 0.003, 64, 48),
                                              (5, 0.003, 64, 48)])
@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_render_direct0_bit_exact(ctl, orc, tracer, dev, config, scale, w, h, mode, bvh):
    """PathTrace<false> (KEY_Direct = 0, PathTracer.h:16): no UniformSampleOneLight,
    emission unweighted (PathTracer.cu:62-70, 82-83), so no shadow rays at all."""
    d = select_bvh(scene(ctl, config, scale, w, h), bvh)
    p = ctl.PTParams(0, 50, 5, 1, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                           "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, 2, w, h)
    got, grays = render_gpu(ctl, tracer, d, p, 2, w, h, dev)
    assert grays == wrays
    assert want[:, :3].max() > 0.0
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])
    # fewer rays than Direct=1: no NEE shadow rays
    p1 = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, p.flags)
    _, wrays1 = oracle_render(orc, d, p1, 1, w, h)
    assert wrays < 2 * wrays1


@pytest.mark.parametrize("mode", ["megakernel", "wavefront"])
def test_render_long_paths_other_schedules(ctl, orc, tracer, dev, mode):
    """50 bounces without Russian roulette through the megakernel and wavefront
    schedules (their samplers wrap the 30-row tables as the persistent one does)."""
    d = scene(ctl, 1, 1.0, 64, 64)
    p = ctl.PTParams(1, 50, 50, 1, 64, 1, 0, ctl.CTL_PT_MEGAKERNEL if mode == "megakernel" else ctl.CTL_PT_WAVEFRONT)
    want, wrays = oracle_render(orc, d, p, 2, 64, 64)
    got, grays = render_gpu(ctl, tracer, d, p, 2, 64, 64, dev)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("mpl,rr", [(1, 5), (3, 1), (8, 2), (50, 50)])
def test_render_short_paths_and_rr(ctl, orc, tracer, dev, mpl, rr):
    """MaxPathLength / RRStartDepth edge values (PathTracer.h:16-19); (50, 50):
    no Russian roulette in the closed box, so paths run far past the sampler's
    30-row tables (the draw counters wrap, SamplerDev keeps them mod len)."""
    d = scene(ctl, 1, 1.0, 64, 64)
    p = ctl.PTParams(1, mpl, rr, 1, 64, 1, 0, 0)
    want, wrays = oracle_render(orc, d, p, 2, 64, 64)
    got, grays = render_gpu(ctl, tracer, d, p, 2, 64, 64, dev)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


def test_render_half_quirk_mode(ctl, orc, tracer, dev):
    s = ctl.HostScene().generate(1, 1.0, 48, 48)
    s.set_flags(ctl.CTL_SCENE_HALF_HOST_QUIRK)
    d = s.compile()
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    want, _ = oracle_render(orc, d, p, 2, 48, 48)
    got, _ = render_gpu(ctl, tracer, d, p, 2, 48, 48, dev)
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


def test_tile_sharding_exact_with_cross_rank_samples(ctl, orc, tracer, dev):
    """1920-wide image, 4 ranks, passes where a jittered sample rounds over a
    tile border onto another rank's pixel (floor(x + u) = x + 1).  The owner of
    the target pixel traces that foreign pixel's path (apron item) and sums the
    pixel in the 1-rank order, so the rank framebuffers sum to the 1-rank
    framebuffer bit for bit; each rank matches the oracle's rank render."""
    from helpers import cross_rank_strays
    w, h, R = 1920, 128, 4
    passes = [p for p in range(400) if cross_rank_strays(orc, p, w, h, R)][:3]
    assert len(passes) == 3
    d = scene(ctl, 2, 0.25, w, h)
    tracer.upload_scene(d)

    def render(nr, r):
        tracer.params = ctl.PTParams(1, 50, 5, 1, 64, nr, r, 0)
        fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
        for p in passes:
            tracer.do_pass(fb.data_ptr(), p)
        torch.cuda.synchronize()
        return fb.cpu().numpy()

    full = render(1, 0)
    acc = np.zeros_like(full)
    for r in range(R):
        part = render(R, r)
        acc += part
        if r == 1:
            want = np.zeros_like(full)
            prm = ctl.PTParams(1, 50, 5, 1, 64, R, r, 0)
            for p in passes:
                orc.oracle_render_pass(C.byref(d), C.byref(prm), p, oracle.ptr(want), tie_rule(d), 0, 1, None)
            assert np.array_equal(want.view(np.uint32), part.view(np.uint32))
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))


def test_tile_sharding_is_exact(ctl, orc, tracer, dev):
    """Rank r renders tiles with tile_id % R == r; the sum of the
    rank framebuffers equals the single-rank framebuffer bit for bit."""
    w, h = 200, 136
    d = scene(ctl, 2, 0.25, w, h)
    full, _ = render_gpu(ctl, tracer, d, ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0), 1, w, h, dev)
    acc = np.zeros_like(full)
    for r in range(3):
        part, _ = render_gpu(ctl, tracer, d, ctl.PTParams(1, 50, 5, 1, 64, 3, r, 0), 1, w, h, dev)
        assert ((part[:, 6] > 0) & (acc[:, 6] > 0)).sum() == 0     # disjoint owners
        acc += part
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))


def test_stats_counts(ctl, orc, tracer, dev):
    d = scene(ctl, 2, 0.25, 96, 64)
    rays = camera_rays(d, 96, 64)
    tracer.upload_scene(d)
    r = torch.from_numpy(rays).to(dev)
    hh = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
    st = tracer.intersect_stats(rays.shape[0], r.data_ptr(), hh.data_ptr())
    assert st[0] == rays.shape[0]
    # the kernel visits at least the nodes the CPU reference order visits on the same rays
    _, _, _, _, _, ost = __import__("helpers").oracle_trace(orc, d, rays, mode=1)
    assert st[1] >= ost[1] * 0.9 and st[2] >= ost[2] * 0.9 and st[3] == ost[3]


def test_full_size_c2_pass_properties(ctl, orc, tracer, dev):
    """BASELINE configs[1] at full size (100k tris, 1280x720): one pass; sampled
    pixels bit-exact against the oracle (every 97th pixel)."""
    w, h = 1280, 720
    d = scene(ctl, 2, 1.0, w, h)
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    got, grays = render_gpu(ctl, tracer, d, p, 1, w, h, dev)
    assert np.isfinite(got).all()
    # AddSample drops NaN/inf/negative samples (Image.cu:26-28); that must stay rare
    assert (got[:, 6] == 0).sum() < w * h * 1e-3
    want = np.zeros((w * h, 7), np.float32)
    orc.oracle_render_pass(C.byref(d), C.byref(p), 0, oracle.ptr(want), tie_rule(d), 0, 97, None)
    sel = np.arange(0, w * h, 97)
    assert np.array_equal(want[sel].view(np.uint32), got[sel].view(np.uint32))
    assert grays > w * h


def work_order_pixels(w, h, ts=64, num_ranks=1, rank=0):
    """numpy restatement of work_pixel(): work item -> (px, py, valid)."""
    tiles_x, tiles_y = -(-w // ts), -(-h // ts)
    num_tiles = tiles_x * tiles_y
    owned = (num_tiles - rank + num_ranks - 1) // num_ranks
    g = np.arange(owned * ts * ts, dtype=np.int64)
    j, wi = g // (ts * ts), g % (ts * ts)
    tile = j * num_ranks + rank
    grp, lane = wi // 64, wi % 64
    gpr = ts // 8
    px = (tile % tiles_x) * ts + (grp % gpr) * 8 + lane % 8
    py = (tile // tiles_x) * ts + (grp // gpr) * 8 + lane // 8
    return px, py, (px < w) & (py < h)


def test_camera_rays_and_batch_trace_bit_exact(ctl, orc, dev):
    """ctl_camera_rays == the oracle's first path ray per pixel (bit-exact), and
    ctl_intersect over them == the oracle's batch intersect."""
    w, h = 200, 136                        # partial tiles on both axes
    d = scene(ctl, 2, 0.25, w, h)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.generate_samples(3)
    n = pt.camera_rays()
    px, py, valid = work_order_pixels(w, h)
    assert n == px.size
    rays = torch.zeros((n, 8), dtype=torch.float32, device=dev)
    assert pt.camera_rays(rays.data_ptr(), n) == n
    hits = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(n, rays.data_ptr(), hits.data_ptr())
    torch.cuda.synchronize()
    got = rays.cpu().numpy()
    want = np.zeros((w * h, 8), np.float32)
    orc.oracle_camera_rays(C.byref(d), 3, oracle.ptr(want))
    lin = py[valid] * w + px[valid]
    assert np.array_equal(got[valid].view(np.uint32), want[lin].view(np.uint32))
    assert np.all(got[~valid][:, 7] == 0.0)
    wh = oracle_intersect(orc, d, want, any_hit=False)
    gh = hits.cpu().numpy()
    assert (wh[:, 2] >= 0).sum() > 1000
    assert np.array_equal(gh[valid], wh[lin])
    pt.close()


def test_intersect_large_batch_refill(ctl, orc, tracer, dev):
    """More rays than resident lanes: every lane refills from the work cursor."""
    d = scene(ctl, 2, 0.05, 64, 64)
    rays = random_rays(d, 1_500_000, seed=11)
    rays[::7, 3] = np.float32(d.ray_eps)
    for any_hit in (False, True):
        want = oracle_intersect(orc, d, rays, any_hit=any_hit)
        got = gpu_intersect(tracer, d, rays, any_hit, dev)
        if any_hit:
            assert np.array_equal(got[:, 2] >= 0, want[:, 2] >= 0)
        else:
            assert np.array_equal(got, want)


def test_last_pass_ms(ctl, dev):
    d = scene(ctl, 2, 0.05, 128, 128)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    fb = torch.zeros((128 * 128, 7), dtype=torch.float32, device=dev)
    pt.do_pass(fb.data_ptr(), 0)
    ms = pt.last_pass_ms()
    assert 0.0 < ms < 10_000.0
    pt.close()


@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("any_hit", [1, 0])
@pytest.mark.parametrize("bvh", ["wide"])
def test_render_c5_bit_exact(ctl, orc, tracer, dev, mode, any_hit, bvh):
    """C5 shading: roughdielectric (Beckmann + GGX, visible-normal
    sampling), image textures with trilinear and EWA MIP filtering driven by the
    first hit's ray differentials, diffuse elsewhere.  Bit-exact framebuffers."""
    w, h = 64, 48
    d = select_bvh(scene(ctl, 5, 0.003, w, h), bvh)
    assert d.n_textures == 2
    kinds = {d.materials[i].bsdf_type for i in range(d.n_materials)}
    assert kinds == {1, 5}
    p = ctl.PTParams(1, 50, 5, any_hit, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                                 "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, 2, w, h)
    got, grays = render_gpu(ctl, tracer, d, p, 2, w, h, dev)
    assert grays == wrays
    assert np.isfinite(got).all()
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.mark.parametrize("modes", [((0, 0), (1, 1), (3, 2), (2, 0), (2, 3)), ((2, 1), (2, 2), (3, 0), (1, 3), (0, 2))],
                         ids=["set_a", "ewa_clamp_mirror"])
def test_render_c5_textured_quad(ctl, orc, tracer, dev, modes):
    """A camera-facing textured quad per (filter, wrap) pair -- point,
    bilinear, trilinear, EWA; repeat, clamp, mirror, black -- plus rough
    Beckmann / GGX panels, lit by an area light: exercises every texture path
    at the first hit (EWA under every wrap mode across the two sets)."""
    s = ctl.HostScene()
    rng = np.random.default_rng(3)
    img = rng.integers(0, 2 ** 32, size=(64, 64), dtype=np.uint64).astype(np.uint32)
    tex = [s.add_texture(img, filter=f, wrap=wr, mapping=(3.0, 0.5, 0.1, -0.2, 2.0, 0.3)) for f, wr in modes]
    mats = [ctl.diffuse_material(0.5, 0.5, 0.5, texture=t) for t in tex]
    mats += [ctl.roughdielectric_material(0, 1.5, 0.1), ctl.roughdielectric_material(1, 1.5, 0.3, 0.2)]
    mats += [ctl.diffuse_material(0.8, 0.8, 0.8)]
    verts, idx, mi, uv = [], [], [], []
    for k in range(len(mats) - 1):
        x0 = -3.5 + k
        base = len(verts)
        verts += [(x0, -1, 0), (x0 + 0.9, -1, 0.3 * k), (x0 + 0.9, 1, 0.3 * k), (x0, 1, 0)]
        uv += [(0, 0), (1.3, 0), (1.3, 1.7), (0, 1.7)]
        idx += [(base, base + 1, base + 2), (base, base + 2, base + 3)]
        mi += [k, k]
    base = len(verts)   # light
    verts += [(-2, 3, -2), (2, 3, -2), (2, 3, 2), (-2, 3, 2)]
    uv += [(0, 0)] * 4
    idx += [(base, base + 2, base + 1), (base, base + 3, base + 2)]
    mi += [len(mats) - 1] * 2
    m = s.add_mesh(np.array(verts, np.float32), np.array(idx, np.uint32), mats, mat_index=np.array(mi, np.uint8),
                   uvs=np.array(uv, np.float32))
    node = s.add_node(m)
    s.add_area_light(node, len(mats) - 1, (20.0, 20.0, 20.0))
    s.set_camera((0.3, 0.2, -6.0), (0, 0, 0), (0, 1, 0), 60.0, 96, 64)
    d = s.compile()
    p = ctl.PTParams(1, 8, 3, 1, 64, 1, 0, 0)
    want, wrays = oracle_render(orc, d, p, 3, 96, 64)
    got, grays = render_gpu(ctl, tracer, d, p, 3, 96, 64, dev)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))
    assert want[:, 0].std() > 0.01                 # the textures show up


def test_image_resolve_and_variance_buffer(ctl, orc, dev):
    """Final-image stage: ctl_image_resolve and the
    PixelVarianceBuffer passes/statistics, bit-exact against the oracle over a
    few real render passes, with one tile skipped in a pass."""
    w, h = 160, 96
    d = scene(ctl, 2, 0.05, w, h)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    var = torch.zeros((w * h, 11), dtype=torch.float32, device=dev)   # 44-B records
    tiles = ((w + 63) // 64) * ((h + 63) // 64)
    var_o = np.zeros((w * h, 11), np.float32)
    for p in range(4):
        pt.do_pass(fb.data_ptr(), p)
        flags = np.ones(tiles, np.uint8)
        if p == 2:
            flags[1] = 0
        pt.variance_add_pass(fb.data_ptr(), w, h, flags, var.data_ptr(), splat_scale=0.5)
        torch.cuda.synchronize()
        orc.oracle_variance_add_pass(oracle.ptr(fb.cpu().numpy()), w, h, np.float32(0.5), 64, oracle.ptr(flags),
                                     oracle.ptr(var_o))
    assert np.array_equal(var.cpu().numpy().view(np.uint32), var_o.view(np.uint32))
    out = torch.zeros(w * h, dtype=torch.int32, device=dev)
    pt.image_resolve(fb.data_ptr(), w, h, out.data_ptr(), splat_scale=0.5)
    stats = torch.zeros((3, w * h), dtype=torch.float32, device=dev)
    pt.variance_stats(var.data_ptr(), w * h, stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr())
    torch.cuda.synchronize()
    want = np.zeros(w * h, np.uint32)
    orc.oracle_image_resolve(oracle.ptr(fb.cpu().numpy()), w, h, np.float32(0.5), oracle.ptr(want))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    so = np.zeros((3, w * h), np.float32)
    orc.oracle_variance_stats(oracle.ptr(var_o), w * h, oracle.ptr(so[0]), oracle.ptr(so[1]), oracle.ptr(so[2]))
    assert np.array_equal(stats.cpu().numpy().view(np.uint32), so.view(np.uint32))
    pt.close()


@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_render_alpha_tested_traversal(ctl, orc, tracer, dev, mode, bvh):
    """Alpha-tested traceRay (TraceHelper.cu:136-154, Material::AlphaTest):
    a checker alpha map (alpha channel), a luminance-thresholded texture and a
    reflectance-map alpha quad in front of a lit wall; camera, bounce and
    shadow rays all see through the cut-outs.  Bit-exact framebuffers."""
    s = ctl.HostScene()
    yy, xx = np.mgrid[0:64, 0:64]
    chk = (((xx // 8) + (yy // 8)) % 2).astype(np.uint32)
    img = (200 | (180 << 8) | (90 << 16) | ((chk * 255) << 24)).astype(np.uint32)
    lum = ((xx * 4) | ((yy * 4) << 8) | (128 << 16) | (255 << 24)).astype(np.uint32)
    ta = s.add_texture(img, filter=ctl._abi.CTL_TEX_BILINEAR)
    tl = s.add_texture(lum, filter=ctl._abi.CTL_TEX_POINT, mapping=(2.0, 0.0, 0.0, 0.0, 2.0, 0.0))
    m_alpha = ctl.set_alpha_map(ctl.diffuse_material(0.7, 0.3, 0.2), 2, 0.5, ta)
    m_lum = ctl.set_alpha_map(ctl.diffuse_material(0.2, 0.6, 0.3), 1, 0.35, tl)
    m_refl = ctl.set_alpha_map(ctl.diffuse_material(0.5, 0.5, 0.5, texture=ta), 6, 0.5)
    wall, light = ctl.diffuse_material(0.8, 0.8, 0.8), ctl.diffuse_material(0.8, 0.8, 0.8)
    mats = [m_alpha, m_lum, m_refl, wall, light]
    verts, idx, mi, uv = [], [], [], []

    def quad(p, k, uvs=((0, 0), (1, 0), (1, 1), (0, 1))):
        b = len(verts)
        verts.extend(p)
        uv.extend(uvs)
        idx.extend([(b, b + 1, b + 2), (b, b + 2, b + 3)])
        mi.extend([k, k])

    for k, x0 in enumerate((-2.2, -0.7, 0.8)):
        quad([(x0, -1, 0), (x0 + 1.4, -1, 0), (x0 + 1.4, 1, 0), (x0, 1, 0)], k)
    quad([(-4, -3, 2), (4, -3, 2), (4, 3, 2), (-4, 3, 2)], 3)
    quad([(-1, 3, -3), (-1, 3, -1), (1, 3, -1), (1, 3, -3)], 4)
    m = s.add_mesh(np.array(verts, np.float32), np.array(idx, np.uint32), mats, mat_index=np.array(mi, np.uint8),
                   uvs=np.array(uv, np.float32))
    node = s.add_node(m)
    s.add_area_light(node, 4, (30.0, 30.0, 30.0))
    s.set_camera((0.2, 0.1, -5.0), (0, 0, 0), (0, 1, 0), 55.0, 96, 64)
    d = select_bvh(s.compile(), bvh)
    p = ctl.PTParams(1, 10, 3, 1, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                            "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, 3, 96, 64)
    got, grays = render_gpu(ctl, tracer, d, p, 3, 96, 64, dev)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))
    # the cut-outs are visible: the oracle with alpha disabled renders differently
    d2 = type(d).from_buffer_copy(d)
    plain = (ctl.Material * 5)(*[ctl.diffuse_material(*mm.reflectance[:]) for mm in mats])
    d2.materials = plain
    no_alpha, _ = oracle_render(orc, d2, p, 3, 96, 64)
    assert not np.array_equal(no_alpha.view(np.uint32), want.view(np.uint32))


# ---- WavefrontPathTracer over the batch traversal ----------

def wpt_gpu(ctl, desc, direct, passes, w, h, dev, max_path_length=50, rr=5, first_pass=1, shadow_any_hit=False):
    wt = ctl.WavefrontPathTracer(0, direct=direct, max_path_length=max_path_length, rr_start_depth=rr,
                                 shadow_any_hit=shadow_any_hit)
    wt.upload_scene(desc)
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    wt.reset_rays()
    for k in range(passes):
        wt.do_pass(fb.data_ptr(), first_pass + k, new_trace=(k == 0))
    torch.cuda.synchronize()
    out = fb.cpu().numpy(), wt.rays_traced()
    wt.close()
    return out


def wpt_oracle(orc, desc, direct, passes, w, h, max_path_length=50, rr=5, first_pass=1):
    fb = np.zeros((w * h, 7), np.float32)
    rays = 0
    for k in range(passes):
        rays += orc.oracle_wpt_render_pass(C.byref(desc), int(direct), max_path_length, rr, k + 1, first_pass + k,
                                           oracle.ptr(fb), tie_rule(desc), 0)
    return fb, rays


@pytest.mark.parametrize("config,scale,w,h", [(1, 1.0, 64, 64), (2, 0.25, 96, 64), (3, 0.003, 64, 48),
                                              (5, 0.003, 64, 48)])
@pytest.mark.parametrize("direct", [1, 0])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_wpt_pass_bit_exact(ctl, orc, dev, config, scale, w, h, direct, bvh):
    """WavefrontPathTracer::DoRender with DoubleRayBuffer queues in fetch order:
    bit-exact framebuffer and the same number of traversed rays as the oracle."""
    d = scene(ctl, config, scale, w, h)
    if bvh == "binary":
        d = binary_bvh(d)
    want, wrays = wpt_oracle(orc, d, direct, 2, w, h)
    got, grays = wpt_gpu(ctl, d, direct, 2, w, h, dev)
    assert grays == wrays
    assert want[:, 6].min() == 2 and np.isfinite(got).all()
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.mark.parametrize("config,scale,w,h", [(1, 1.0, 64, 64), (2, 0.25, 96, 64), (3, 0.003, 64, 48),
                                              (5, 0.003, 64, 48)])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_wpt_shadow_any_hit_equals_reference(ctl, orc, dev, config, scale, w, h, bvh):
    """CTL_WPT_SHADOW_ANY_HIT: the secondary rays as the any-hit shadow query
    (tmax = dist (1 - eps), culled at tmax + slab slack) give the image of the
    reference's closest hit + distance compare (the oracle), bit for bit."""
    d = select_bvh(scene(ctl, config, scale, w, h), bvh)
    want, wrays = wpt_oracle(orc, d, 1, 2, w, h, first_pass=5)
    got, grays = wpt_gpu(ctl, d, 1, 2, w, h, dev, first_pass=5, shadow_any_hit=True)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("mpl,rr", [(1, 5), (2, 1), (7, 2), (50, 50)])
def test_wpt_short_paths(ctl, orc, dev, mpl, rr):
    d = scene(ctl, 2, 0.25, 96, 64)
    want, wrays = wpt_oracle(orc, d, 1, 2, 96, 64, mpl, rr, first_pass=3)
    got, grays = wpt_gpu(ctl, d, 1, 2, 96, 64, dev, mpl, rr, first_pass=3)
    assert grays == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("w,h", [(4096, 8), (8, 4200), (2500, 12)])
def test_wpt_wide_image_shared_targets(ctl, orc, dev, w, h):
    """Pixel coordinates travel as half (WavefrontPTRayData): above 2048 two or
    more source pixels round to one target pixel and their samples add into it
    (the reference's atomicAdd).  The pass is bit-exact against the oracle's
    sequential adds (bounce, then image order)."""
    d = scene(ctl, 2, 0.25, w, h)
    want, wrays = wpt_oracle(orc, d, 1, 2, w, h)
    got, grays = wpt_gpu(ctl, d, 1, 2, w, h, dev)
    assert grays == wrays
    assert want[:, 6].max() >= 4   # shared targets exist
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


def test_wpt_converges_to_path_tracer(ctl, orc, tracer, dev):
    """Different sample streams, same integral: the wavefront tracer's image mean
    matches the PathTracer's within Monte-Carlo noise (C1, 48 passes)."""
    w = h = 48
    d = scene(ctl, 1, 1.0, w, h)
    a, _ = wpt_gpu(ctl, d, 1, 48, w, h, dev)
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    b, _ = render_gpu(ctl, tracer, d, p, 48, w, h, dev, first_pass=1)
    ma = (a[:, :3] / a[:, 6:7]).mean(0)
    mb = (b[:, :3] / b[:, 6:7]).mean(0)
    assert np.all(np.abs(ma - mb) <= 0.03 * mb + 1e-4), (ma, mb)


@pytest.mark.parametrize("pass_index", [0, 1, 7, 1000, 123456])
def test_device_sampler_tables_bit_exact(ctl, orc, dev, pass_index):
    """sampler_kernel (wave-parallel XORWOW jumps) == the oracle's SequenceSampler
    tables of the same pass (CudaRNG(7539414) stream, Kernel/Sampler.h:36-55)."""
    pt = ctl.PathTracer(0)
    try:
        nseq, ln = 4096, 30
        pt.generate_samples(pass_index)
        got1 = np.zeros(nseq * ln, np.float32)
        got2 = np.zeros(nseq * ln * 2, np.float32)
        L = ctl.lib()
        assert L.ctl_scene_read(pt._ctx, ctl._abi.CTL_ARRAY_SAMPLES_1D, 0, nseq * ln, got1.ctypes.data) == 0
        assert L.ctl_scene_read(pt._ctx, ctl._abi.CTL_ARRAY_SAMPLES_2D, 0, nseq * ln, got2.ctypes.data) == 0
        want1 = np.zeros_like(got1)
        want2 = np.zeros_like(got2)
        orc.oracle_sampler_tables(pass_index, nseq, ln, oracle.ptr(want1), oracle.ptr(want2))
        assert np.array_equal(got1.view(np.uint32), want1.view(np.uint32))
        assert np.array_equal(got2.view(np.uint32), want2.view(np.uint32))
    finally:
        pt.close()


@pytest.mark.parametrize("ranks,rank,n", [(1, 0, 1), (1, 0, 4), (3, 1, 3), (8, 0, 8)])
@pytest.mark.parametrize("config,scale,w,h", [(2, 0.25, 200, 136), (3, 0.003, 136, 72)])
def test_render_passes_equals_sequential_passes(ctl, orc, tracer, dev, ranks, rank, n, config, scale, w, h):
    """ctl_render_passes(first, n) == n rounds of ctl_sampler_generate + ctl_render_pass
    (and the oracle's passes) bit for bit, on a shard of the tiles."""
    d = scene(ctl, config, scale, w, h)
    p = ctl.PTParams(1, 50, 5, 1, 64, ranks, rank, 0)
    first = 5
    want, wrays = oracle_render(orc, d, p, n, w, h, first_pass=first)
    seq, srays = render_gpu(ctl, tracer, d, p, n, w, h, dev, first_pass=first)
    tracer.params = p
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    tracer.reset_rays()
    tracer.render_passes(fb.data_ptr(), first, n)
    torch.cuda.synchronize()
    got = fb.cpu().numpy()
    assert tracer.rays_traced() == srays == wrays
    assert want[:, 6].sum() > 0
    assert np.array_equal(seq.view(np.uint32), want.view(np.uint32))
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
def test_colliding_samples_all_schedules(ctl, orc, tracer, dev, mode):
    """Pass 5 at 200x136 has a pixel that receives two samples (a jittered
    position rounds onto the neighbour, Image.cu:22-44): every schedule adds
    both, in image order, like the oracle."""
    w, h = 200, 136
    d = scene(ctl, 2, 0.25, w, h)
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                             "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, 2, w, h, first_pass=5)
    got, grays = render_gpu(ctl, tracer, d, p, 2, w, h, dev, first_pass=5)
    assert grays == wrays
    assert want[:, 6].max() > 2          # the collision is there
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))

"""How far the default (4-wide) traversal order lands from the reference's own
binary order, and that every traversal is a function of its ray alone.

The reference's semantics for a ray: TracerayTemplate's host branch
(Engine/SpatialStructures/BVH/BVHTraversal.h:122-232, the vote mask of a lone
lane) over the binary tree, first found wins a tie (Kernel/TraceHelper.cu:121),
boxes culled at the current hit (BVHTraversal.h:58-67).  CTL_SCENE_BINARY_BVH
runs exactly that on the GPU; the oracle's mode 0 restates it.  The default
device traversal walks 4-wide trees in its own per-ray order (DESIGN.md §5,
oracle mode 2 restates it); the two orders can pick different hits only when
two triangles tie at exactly the same t, or when a box's rounded slab entry
lies past a hit inside it (one order culls that box, the other has not found
the nearer hit yet).  These tests count both, on adversarial scenes on the CPU
and at full size (C3, 10 M triangles) on the GPU, and hold the GPU to its own
stated order bit for bit, under any permutation of the rays.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle
from helpers import (binary_bvh, camera_rays, classify_orders, grazing_rays, grid_room, oracle_intersect,
                     random_rays, select_bvh, tie_rule)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Bounds on the distance to the reference order.  Measured: 0
# differing rays on every small scene below, and on the full-size C3 rays of
# test_full_size_c3_reference_order_distance a rate well under these.
MAX_DIFFER_FRAC = 2e-5          # rays whose hit differs from the reference's
MAX_PIXEL_OVER_FRAC = 2e-3      # full-pass pixels beyond 1e-4 relative radiance

SCENES = {}


def scene(ctl, config, scale, w=96, h=64):
    key = (config, scale, w, h)
    if key not in SCENES:
        s = ctl.HostScene().generate(config, scale, w, h)
        SCENES[key] = (s, s.compile())
    return SCENES[key][1]


def room(ctl, offset):
    key = ("room", tuple(offset))
    if key not in SCENES:
        SCENES[key] = grid_room(ctl, offset)
    return SCENES[key][1]


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.25), (3, 0.004), (5, 0.003)])
def test_wide_order_vs_reference_order_small(ctl, orc, config, scale):
    """Random (some with tmin > 0 and a short tmax) and camera rays: the 4-wide
    order against the reference order, and both against an exhaustive scan."""
    d = scene(ctl, config, scale)
    rays = np.concatenate([random_rays(d, 40000, seed=config), camera_rays(d, 96, 64, seed=config)])
    rays[:40000:3, 3] = np.float32(d.ray_eps)
    rays[1:40000:5, 7] = np.float32(5.0)
    ref = oracle_intersect(orc, d, rays, tie=0)
    wide = oracle_intersect(orc, d, rays)
    c = classify_orders(ref, wide)
    assert c["differ"] <= MAX_DIFFER_FRAC * c["rays"], c
    assert c["hit_miss"] == 0 and c["same_hit_other_fields"] == 0, c
    bt = np.zeros(rays.shape[0], np.float32)
    btri = np.zeros(rays.shape[0], np.uint32)
    orc.oracle_brute_force(C.byref(d), rays.shape[0], oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
    full = (rays[:, 3] <= d.ray_eps) & (rays[:, 7] > 1e30)     # the scan's window: (eps, inf)
    hit = full & (wide[:, 2] >= 0)
    assert hit.sum() > 1000
    # the tree finds the scan's closest t on all but a sliver of rays (the float slab test can
    # exclude a box whose triangle the scan hits; the reference's tree does the same)
    assert (wide[hit, 0].view(np.float32) != bt[hit]).mean() < 1e-3


@pytest.mark.parametrize("offset", [(0.0, 0.0, 0.0), (1.0e4, 1.0e4, 1.0e4), (-3.0e4, 2.0e3, 5.0e4)])
def test_wide_order_vs_reference_order_grazing_translated(ctl, orc, offset):
    """Axis-aligned walls of touching grid triangles, moved up to 5e4 from the
    origin; rays leaving the walls nearly parallel to them (|d| component
    1e-7 .. 1e-2 of the others).  The slab entry's error grows with |o| / |d|,
    so this is where a box holding the hit can round past it."""
    d = room(ctl, offset)
    rays = grazing_rays(d, offset, 150000, seed=7)
    ref = oracle_intersect(orc, d, rays, tie=0)
    wide = oracle_intersect(orc, d, rays)
    c = classify_orders(ref, wide)
    assert (ref[:, 2] >= 0).sum() > 50000
    assert c["differ"] <= MAX_DIFFER_FRAC * c["rays"], c
    assert c["hit_miss"] == 0, c


def test_refraction_rays_wide_vs_reference_order_small(ctl, orc):
    """The C5 ray class refraction adds (transmitted-like rays that start on a
    roughdielectric surface and cross it), on a small C5 scene: the 4-wide order
    against the reference order."""
    d = scene(ctl, 5, 0.003, 192, 128)
    prim = camera_rays(d, 192, 128, seed=5)
    ph = oracle_intersect(orc, d, prim)
    refr = refraction_rays(d, prim, ph, np.random.default_rng(3), 20000)
    assert refr.shape[0] > 1000
    ref = oracle_intersect(orc, d, refr, tie=0)
    wide = oracle_intersect(orc, d, refr)
    c = classify_orders(ref, wide)
    assert (ref[:, 2] >= 0).sum() > 300          # an open scene: most transmitted rays leave it
    assert c["differ"] <= MAX_DIFFER_FRAC * c["rays"], c
    assert c["hit_miss"] == 0, c


def test_host_wide_trees_shape(ctl):
    d = scene(ctl, 2, 0.25)
    mesh, wbase, sc = ctl.host_wide_trees(d)
    assert mesh.shape[1] == 32 and mesh.shape[0] > 0 and wbase.shape == (d.n_meshes,)
    ch = mesh[:, 24:28].view(np.int32)
    inner = (ch >= 0) & (ch != 0x76543210)
    assert ch[inner].max() < mesh.shape[0]
    # every binary leaf value reaches a wide leaf (counted: first entry << 3 | count)
    assert (ch < 0).sum() > 0


# ---------------------------------------------------------------------------
# GPU: the device order is its stated one, bit for bit, in any ray order
# ---------------------------------------------------------------------------
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def gpu_hits(pt, rays, dev, any_hit=False):
    r = torch.from_numpy(rays).to(dev)
    h = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(rays.shape[0], r.data_ptr(), h.data_ptr(), any_hit=any_hit)
    torch.cuda.synchronize()
    return h.cpu().numpy()


@pytest.mark.gpu
def test_device_wide_trees_equal_host(ctl, dev):
    """The trees ctl_scene_upload builds (read back, CTL_ARRAY_WIDE_BVH ...) are
    ctl_host_wide_trees' bit for bit: the oracle's mode 2 walks what the GPU walks."""
    from test_gpu_instances import instanced_scene
    for d in (scene(ctl, 2, 0.25), instanced_scene(ctl, 64, 48)):
        pt = ctl.PathTracer(0)
        try:
            pt.upload_scene(d)
            got = pt.wide_trees(d)
        finally:
            pt.close()
        want = ctl.host_wide_trees(d)
        for g, w in zip(got, want):
            assert g.shape == w.shape and np.array_equal(g.view(np.uint32), w.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["c3_random", "c3_camera", "room_origin", "room_1e4", "room_far"])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_hits_independent_of_ray_order(ctl, orc, dev, case, bvh):
    """ctl_intersect on the same rays in their original order and under three
    random permutations: identical per-ray hits (a ray's result does not depend
    on which rays share its wave), equal to the oracle's statement of the same
    order; any-hit decisions equal too.  Includes walls 1e4 / 5e4 from the
    origin and grazing rays, the cases where culling is most fragile."""
    if case.startswith("c3"):
        d = scene(ctl, 3, 0.02, 128, 96)
        rays = random_rays(d, 200000, seed=3) if case == "c3_random" else camera_rays(d, 512, 384, seed=3)
    else:
        off = {"room_origin": (0.0, 0.0, 0.0), "room_1e4": (1.0e4, 1.0e4, 1.0e4),
               "room_far": (-3.0e4, 2.0e3, 5.0e4)}[case]
        d = room(ctl, off)
        rays = grazing_rays(d, off, 200000, seed=11)
    d = select_bvh(d, bvh)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        base = gpu_hits(pt, rays, dev)
        base_any = gpu_hits(pt, rays, dev, any_hit=True)
        rng = np.random.default_rng(5)
        for _ in range(3):
            perm = rng.permutation(rays.shape[0])
            got = gpu_hits(pt, rays[perm], dev)
            assert np.array_equal(got, base[perm])
            got_any = gpu_hits(pt, rays[perm], dev, any_hit=True)
            assert np.array_equal(got_any[:, 2] >= 0, base_any[perm][:, 2] >= 0)
    finally:
        pt.close()
    want = oracle_intersect(orc, d, rays)
    bad = np.nonzero((want != base).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], base[bad[:3]])
    assert (base[:, 2] >= 0).sum() > 10000


def secondary_rays(desc, prim, hits, rng, n):
    """Bounce- and shadow-like rays from the camera rays' hit points: origins
    o + t d (fp32), bounce directions uniform on the sphere (tmin = eps), shadow
    segments towards random points of the scene box (tmin = eps, tmax = 0.999 of
    the distance)."""
    hit = np.nonzero(hits[:, 2] >= 0)[0]
    sel = rng.choice(hit, size=min(n, hit.size), replace=False)
    t = hits[sel, 0].view(np.float32)[:, None]
    p = prim[sel, 0:3] + t * prim[sel, 4:7]
    m = sel.size
    b = np.zeros((m, 8), np.float32)
    b[:, 0:3] = p
    b[:, 3] = np.float32(desc.ray_eps)
    dd = rng.normal(size=(m, 3))
    b[:, 4:7] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
    b[:, 7] = 3.0e38
    lo, hi = np.array(desc.box_min[:]), np.array(desc.box_max[:])
    q = lo + (hi - lo) * rng.random((m, 3))
    v = q - p
    dist = np.linalg.norm(v, axis=1)
    s = np.zeros((m, 8), np.float32)
    s[:, 0:3] = p
    s[:, 3] = np.float32(desc.ray_eps)
    s[:, 4:7] = v / dist[:, None]
    s[:, 7] = dist * 0.999
    return b, s


def nee_shadow_rays(desc, prim, hits, rng, n):
    """NEE-like shadow rays (ctl_ray: o, d, tmax = dist) from camera-ray hit
    points to points drawn uniformly by area on the scene's light triangles
    (ShapeSet::SamplePosition's distribution, fp64 inputs), as EstimateDirect
    hands them to Occluded(Ray(p, d), 0, dist)."""
    hit = np.nonzero(hits[:, 2] >= 0)[0]
    sel = rng.choice(hit, size=min(n, hit.size), replace=False)
    t = hits[sel, 0].view(np.float32)[:, None]
    p = (prim[sel, 0:3] + t * prim[sel, 4:7]).astype(np.float32)
    lt = [desc.light_tris[i] for i in range(desc.n_light_tris)]
    P = np.array([[list(x.p[k]) for k in range(3)] for x in lt], np.float64)        # (L, 3, 3)
    area = np.array([x.area for x in lt], np.float64)
    k = rng.choice(len(lt), size=sel.size, p=area / area.sum())
    u, v = rng.random(sel.size), rng.random(sel.size)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    q = P[k, 0] + u[:, None] * (P[k, 1] - P[k, 0]) + v[:, None] * (P[k, 2] - P[k, 0])
    w = q - p
    dist = np.linalg.norm(w, axis=1)
    s = np.zeros((sel.size, 8), np.float32)
    s[:, 0:3] = p
    s[:, 4:7] = w / dist[:, None]
    s[:, 7] = dist
    return s[dist > 1e-3]


def pixel_distance(img, want):
    a, b = img[:, :3].astype(np.float64), want[:, :3].astype(np.float64)
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    rel[(a == b)] = 0.0
    over = (rel > 1e-4).any(axis=1) | (img[:, 6] != want[:, 6])
    return {"pixels": int(img.shape[0]), "pixels_over_1e-4_rel": int(over.sum()),
            "pixels_differing": int((img.view(np.uint32) != want.view(np.uint32)).any(axis=1).sum()),
            "max_rel": float(rel.max())}


def build_stamp():
    """Hashes of the library and of its sources (buildid.py), so a record can be
    matched to the binary that produced it (bench.py reference_order_record)."""
    import hashlib
    import sys
    sys.path.insert(0, ROOT)
    from buildid import source_fingerprint
    lib = os.path.join(ROOT, "cudatracerlib_amd", "_lib", "libctl_trace.so")
    return {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "src_sha256": source_fingerprint(ROOT)}


def refraction_rays(desc, prim, hits, rng, n):
    """Transmitted-like rays from camera-ray hits on roughdielectric triangles
    (the C5 population that refraction adds, BSDF_Simple.cu:491-615): origin
    o + t d (fp32), direction Snell-refracted (eta 1.5, entering or leaving by
    the side the ray arrives from) about a microfacet normal tilted from the
    triangle's plane normal (the Woop row a, TriIntersectorData.cu:5-18) by a
    random alpha in [0.05, 0.5]; total internal reflection reflects.  tmin =
    eps, as traceRay's; the ray crosses the surface it starts on."""
    A = __import__("cudatracerlib_amd")._abi
    nt, ni, nw = int(desc.n_tri_data), int(desc.n_tri_indices), int(desc.n_woop_tris)
    td = np.ctypeslib.as_array(C.cast(desc.tri_data, C.POINTER(C.c_uint32)), shape=(nt * 8,)).reshape(nt, 8)
    idx = np.ctypeslib.as_array(C.cast(desc.tri_indices, C.POINTER(C.c_uint32)), shape=(ni,))
    woop = np.ctypeslib.as_array(C.cast(desc.woop_tris, C.POINTER(C.c_float)), shape=(nw * 12,)).reshape(nw, 12)
    assert desc.n_meshes == 1 and desc.meshes[0].triangle_offset == 0 and desc.meshes[0].bvh_indices_offset == 0
    mats = np.array([desc.materials[i].bsdf_type for i in range(desc.n_materials)])
    mat_off = desc.nodes[0].material_offset if desc.n_nodes else 0
    hit = np.nonzero(hits[:, 2] >= 0)[0]
    tri = hits[hit, 2].astype(np.int64)
    m = ((td[tri, 1] >> 16) & 0xFF).astype(np.int64) + mat_off
    hit = hit[mats[m] == A.CTL_BSDF_ROUGHDIELECTRIC]
    # fewer dielectric hits than rays wanted: hit points repeat, each with its own microfacet normal
    sel = rng.choice(hit, size=n, replace=True) if hit.size < n else rng.choice(hit, size=n, replace=False)
    slot = np.empty(nt, np.int64)
    slot[idx >> 1] = np.arange(ni)
    a = woop[slot[hits[sel, 2]], 0:3].astype(np.float64)
    ng = a / np.linalg.norm(a, axis=1, keepdims=True)
    d = prim[sel, 4:7].astype(np.float64)
    t = hits[sel, 0].view(np.float32)[:, None]
    p = (prim[sel, 0:3] + t * prim[sel, 4:7]).astype(np.float32)
    front = (d * ng).sum(1) < 0
    eta = np.where(front, 1.0 / 1.5, 1.5)[:, None]
    ng = np.where(front[:, None], ng, -ng)                       # facing the incoming ray
    alpha = rng.uniform(0.05, 0.5, size=(sel.size, 1))
    mn = ng + alpha * rng.normal(size=(sel.size, 3))
    mn /= np.linalg.norm(mn, axis=1, keepdims=True)
    ci = -(d * mn).sum(1, keepdims=True)
    bad = ci[:, 0] <= 0
    mn[bad], ci[bad] = ng[bad], -(d[bad] * ng[bad]).sum(1, keepdims=True)
    k = 1.0 - eta ** 2 * (1.0 - ci ** 2)
    refr = eta * d + (eta * ci - np.sqrt(np.maximum(k, 0.0))) * mn
    refl = d + 2.0 * ci * mn
    w = np.where(k >= 0, refr, refl)
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    r = np.zeros((sel.size, 8), np.float32)
    r[:, 0:3] = p
    r[:, 3] = np.float32(desc.ray_eps)
    r[:, 4:7] = w
    r[:, 7] = 3.0e38
    return r


# BASELINE configs of the PathTracer at their full size: (generate config, width, height)
FULL = {"c2": (2, 1280, 720), "c3": (3, 1920, 1080), "c5": (5, 1920, 1080)}


@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_full_size_reference_order_distance(ctl, orc, dev, cfg):
    """C2 / C3 / C5 at full size against the reference's own CPU path.  (1) One
    pass's camera rays plus a million bounce-like and a million shadow-like rays
    from their hits (C5: and a million transmitted-like rays through its
    roughdielectric surfaces), through ctl_intersect (default 4-wide order):
    bit-exact to the oracle's statement of that order, classified against the
    reference's binary order.  (2) A million NEE shadow rays to points on the
    lights: the shipped any-hit query (ctl_occluded) against the reference's
    closest-hit Occluded in its binary order (visibility flips).  (3) One full
    PathTracer pass of the shipped default (4-wide order, any-hit shadow rays)
    against the oracle's render of the reference's CPU path (binary order,
    closest-hit Occluded, KernelDynamicScene.cu:70-80) and against the binary
    order with any-hit shadows, per pixel at 1e-4 relative.  The counts and the
    build's hashes go to gpurun_out/reference_order_<cfg>.json (bench.py reports
    the committed copies under profiles/)."""
    config, W, H = FULL[cfg]
    hs = ctl.HostScene().generate(config, 1.0, W, H)
    d = hs.compile()
    rng = np.random.default_rng(2024)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        pt.generate_samples(3)
        n = pt.camera_rays()
        rays = torch.zeros((n, 8), dtype=torch.float32, device=dev)
        pt.camera_rays(rays.data_ptr(), n)
        torch.cuda.synchronize()
        prim = rays.cpu().numpy()
        del rays
        prim = prim[prim[:, 7] > 0]
        ph = gpu_hits(pt, prim, dev)
        bounce, shadow = secondary_rays(d, prim, ph, rng, 1_000_000)
        classes = [("camera", prim, ph), ("bounce", bounce, gpu_hits(pt, bounce, dev)),
                   ("shadow_closest", shadow, gpu_hits(pt, shadow, dev))]
        if config == 5:
            refr = refraction_rays(d, prim, ph, rng, 1_000_000)
            classes.append(("refraction", refr, gpu_hits(pt, refr, dev)))
        nee = nee_shadow_rays(d, prim, ph, rng, 1_000_000)
        nr = torch.from_numpy(nee).to(dev)
        occ = torch.zeros(nee.shape[0], dtype=torch.int32, device=dev)
        pt.occluded(nee.shape[0], nr.data_ptr(), occ.data_ptr(), True)
        torch.cuda.synchronize()
        nee_any = occ.cpu().numpy().astype(np.uint8)
        del nr, occ
        # one full pass, default schedule, order and shadow query
        pt.params = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        pt.do_pass(fb.data_ptr(), 0)
        pt.sync()
        img, grays = fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()
    out = {"config": cfg, "scene": f"{cfg.upper()} {d.n_tri_data} tris, {W}x{H}", "build": build_stamp(),
           "classes": {}}
    for name, r, g in classes:
        wide = oracle_intersect(orc, d, r, threads=16)
        bad = np.nonzero((wide != g).any(axis=1))[0]
        assert bad.size == 0, (name, bad[:10], wide[bad[:3]], g[bad[:3]])
        ref = oracle_intersect(orc, d, r, tie=0, threads=16)
        out["classes"][name] = classify_orders(ref, g)
    tot = {k: sum(c[k] for c in out["classes"].values()) for k in next(iter(out["classes"].values()))}
    out["total"] = tot
    # NEE visibility: the shipped query against the reference's Occluded
    tie = tie_rule(d, orc)

    def occ_oracle(any_hit, order, cull=oracle.CULL_SLAB):
        o = np.zeros(nee.shape[0], np.uint8)
        orc.oracle_occluded(C.byref(d), nee.shape[0], oracle.ptr(nee), oracle.ptr(o), int(any_hit), order, cull, 16)
        return o
    assert np.array_equal(nee_any, occ_oracle(True, tie))           # ctl_occluded states the product's query
    ref_occ = occ_oracle(False, 0)
    out["nee_visibility"] = {"rays": int(nee.shape[0]), "reference_occluded": int(ref_occ.sum()),
                             "visibility_flips": int((nee_any != ref_occ).sum()),
                             "flips_round4_rule": int((occ_oracle(True, tie, oracle.CULL_AT_ACCEPT) != ref_occ).sum())}
    # the pass, against the reference's CPU path and against the binary order with any-hit shadows
    renders = {}
    for key, any_hit in (("reference_cpu_path", 0), ("binary_order_any_hit", 1)):
        want = np.zeros((W * H, 7), np.float32)
        wr = orc.oracle_render_pass(C.byref(d), C.byref(ctl.PTParams(1, 50, 5, any_hit, 64, 1, 0, 0)), 0,
                                    oracle.ptr(want), 0, 16, 1, None)
        renders[key] = pixel_distance(img, want)
        renders[key]["rays_reference"] = int(wr)
    renders["rays_gpu"] = int(grays)
    out["pass"] = renders
    hs.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"reference_order_{cfg}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    assert tot["hit_miss"] == 0 and tot["same_hit_other_fields"] == 0, out
    assert tot["differ"] <= MAX_DIFFER_FRAC * tot["rays"], out
    assert out["nee_visibility"]["visibility_flips"] <= MAX_DIFFER_FRAC * nee.shape[0], out
    for key in ("reference_cpu_path", "binary_order_any_hit"):
        assert renders[key]["pixels_over_1e-4_rel"] <= MAX_PIXEL_OVER_FRAC * W * H, out

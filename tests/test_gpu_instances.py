"""Two-level traversal with real instance transforms (SceneBVH.cpp:77-100,
TraceHelper.cu:91-100, 528-561): one mesh instanced three times with
distinct rotation, non-uniform scale and translation, a second mesh (the
ground), and an area light on a rotated + scaled + translated node.  The
non-SINGLE wide and binary traversals, batch closest / any hit and the
three PathTracer schedules, bit-exact against the oracle."""
import ctypes as C

import numpy as np
import pytest

import oracle

from helpers import binary_bvh, device_wide_trees, oracle_intersect, oracle_render, random_rays

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def uv_sphere(nu=24, nv=12):
    verts, nrm, uv, idx = [], [], [], []
    for j in range(nv + 1):
        th = np.pi * j / nv
        for i in range(nu + 1):
            ph = 2 * np.pi * i / nu
            p = (np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph))
            verts.append(p)
            nrm.append(p)
            uv.append((i / nu, j / nv))
    for j in range(nv):
        for i in range(nu):
            a, b = j * (nu + 1) + i, j * (nu + 1) + i + 1
            c, d = a + nu + 1, b + nu + 1
            if j > 0:
                idx.append((a, b, c))
            if j < nv - 1:
                idx.append((b, d, c))
    return (np.array(verts, np.float32), np.array(idx, np.uint32), np.array(nrm, np.float32),
            np.array(uv, np.float32))


def xform(axis, angle, scale, trans):
    """Row-major float4x4 = T * R * S (translation in the last column)."""
    a = np.asarray(axis, np.float64)
    a /= np.linalg.norm(a)
    c, s = np.cos(angle), np.sin(angle)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) * c + s * K + (1 - c) * np.outer(a, a)
    M = np.eye(4)
    M[:3, :3] = R @ np.diag(scale)
    M[:3, 3] = trans
    return M.astype(np.float32).ravel()


SCENE = {}


def instanced_scene(ctl, w=96, h=64):
    if "d" in SCENE:
        return SCENE["d"]
    s = ctl.HostScene()
    v, i, n, uv = uv_sphere()
    mats = [ctl.diffuse_material(0.7, 0.3, 0.2), ctl.diffuse_material(0.2, 0.6, 0.8)]
    mi = (np.arange(i.shape[0]) % 3 == 0).astype(np.uint8)
    sphere = s.add_mesh(v, i, mats, mat_index=mi, normals=n, uvs=uv)
    g = np.array([(-8, 0, -8), (8, 0, -8), (8, 0, 8), (-8, 0, 8)], np.float32)
    ground = s.add_mesh(g, np.array([(0, 2, 1), (0, 3, 2)], np.uint32), [ctl.diffuse_material(0.6, 0.6, 0.6)])
    q = np.array([(-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1)], np.float32)
    light = s.add_mesh(q, np.array([(0, 1, 2), (0, 2, 3)], np.uint32), [ctl.diffuse_material(0.8, 0.8, 0.8)])
    s.add_node(sphere, xform((0, 1, 0), 0.3, (1.0, 1.6, 0.7), (-2.5, 1.6, 0.5)))
    s.add_node(sphere, xform((1, 0, 1), 1.1, (0.5, 0.5, 1.8), (0.4, 0.9, -1.0)))
    s.add_node(sphere, xform((0.3, 0.2, 1), -0.7, (1.3, 0.6, 0.9), (2.6, 0.8, 1.4)))
    s.add_node(ground)
    ln = s.add_node(light, xform((1, 0, 0.2), 0.35, (1.5, 1.0, 0.6), (0.3, 5.0, 0.5)))
    s.add_area_light(ln, 0, (14.0, 13.0, 11.0))
    s.set_camera((0.5, 3.0, -8.5), (0.0, 1.0, 0.0), (0, 1, 0), 55.0, w, h)
    d = s.compile()
    assert d.n_nodes == 5 and d.n_meshes == 3 and d.scene_start_node >= 0   # two-level, not SINGLE
    SCENE["s"], SCENE["d"] = s, d
    return d


@pytest.mark.parametrize("bvh", ["wide", "binary"])
@pytest.mark.parametrize("any_hit", [False, True])
def test_instanced_intersect_bit_exact(ctl, orc, dev, bvh, any_hit):
    d = instanced_scene(ctl)
    d = binary_bvh(d) if bvh == "binary" else d
    rays = random_rays(d, 60000, seed=21)
    rays[::4, 3] = np.float32(d.ray_eps)
    want = oracle_intersect(orc, d, rays, any_hit=any_hit)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    r = torch.from_numpy(rays).to(dev)
    hh = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(rays.shape[0], r.data_ptr(), hh.data_ptr(), any_hit=any_hit)
    pt.sync()
    got = hh.cpu().numpy()
    pt.close()
    hit_nodes = set(np.unique(want[want[:, 2] >= 0, 1]).tolist())
    assert {0, 1, 2, 3} <= hit_nodes          # every transformed instance is hit
    if any_hit:
        assert np.array_equal(want[:, 2] >= 0, got[:, 2] >= 0)
    else:
        bad = np.nonzero((want != got).any(axis=1))[0]
        assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.mark.parametrize("mode", ["persistent", "wavefront", "megakernel"])
@pytest.mark.parametrize("bvh", ["wide", "binary"])
@pytest.mark.parametrize("direct", [1, 0])
def test_instanced_render_bit_exact(ctl, orc, dev, mode, bvh, direct):
    w, h = 96, 64
    d = instanced_scene(ctl, w, h)
    d = binary_bvh(d) if bvh == "binary" else d
    p = ctl.PTParams(direct, 50, 5, 1, 64, 1, 0, {"persistent": 0, "megakernel": ctl.CTL_PT_MEGAKERNEL,
                                                   "wavefront": ctl.CTL_PT_WAVEFRONT}[mode])
    want, wrays = oracle_render(orc, d, p, 3, w, h)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.params = p
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    for k in range(3):
        pt.do_pass(fb.data_ptr(), k)
    pt.sync()
    got, grays = fb.cpu().numpy(), pt.rays_traced()
    pt.close()
    assert grays == wrays
    assert want[:, :3].max() > 0.0            # the light reaches the image
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])


def instanced_scene_xf(ctl, xfs, w=96, h=64):
    """instanced_scene with the transforms of `xfs` ({node: xf16}) replaced, compiled anew."""
    s = ctl.HostScene()
    v, i, n, uv = uv_sphere()
    mats = [ctl.diffuse_material(0.7, 0.3, 0.2), ctl.diffuse_material(0.2, 0.6, 0.8)]
    mi = (np.arange(i.shape[0]) % 3 == 0).astype(np.uint8)
    sphere = s.add_mesh(v, i, mats, mat_index=mi, normals=n, uvs=uv)
    g = np.array([(-8, 0, -8), (8, 0, -8), (8, 0, 8), (-8, 0, 8)], np.float32)
    ground = s.add_mesh(g, np.array([(0, 2, 1), (0, 3, 2)], np.uint32), [ctl.diffuse_material(0.6, 0.6, 0.6)])
    q = np.array([(-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1)], np.float32)
    light = s.add_mesh(q, np.array([(0, 1, 2), (0, 2, 3)], np.uint32), [ctl.diffuse_material(0.8, 0.8, 0.8)])
    base = [(sphere, xform((0, 1, 0), 0.3, (1.0, 1.6, 0.7), (-2.5, 1.6, 0.5))),
            (sphere, xform((1, 0, 1), 1.1, (0.5, 0.5, 1.8), (0.4, 0.9, -1.0))),
            (sphere, xform((0.3, 0.2, 1), -0.7, (1.3, 0.6, 0.9), (2.6, 0.8, 1.4))),
            (ground, None),
            (light, xform((1, 0, 0.2), 0.35, (1.5, 1.0, 0.6), (0.3, 5.0, 0.5)))]
    for k, (m, xf) in enumerate(base):
        s.add_node(m, xfs.get(k, xf))
    s.add_area_light(4, 0, (14.0, 13.0, 11.0))
    s.set_camera((0.5, 3.0, -8.5), (0.0, 1.0, 0.0), (0, 1, 0), 55.0, w, h)
    return s, s.compile()


MOVES = {1: xform((0.2, 1, 0.1), 2.0, (0.7, 1.4, 0.6), (-0.8, 1.2, -2.2)),
         4: xform((0.3, 0, 1), -0.25, (1.2, 1.0, 0.9), (-0.6, 4.6, -0.4))}


@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_set_transform_on_device_matches_recompiled_scene(ctl, orc, dev, bvh):
    """DynamicScene::SetNodeTransform (DynamicScene.cpp:433-443, SceneBVH.cpp:77-89)
    on the device: a sphere instance and the light's node move without a
    re-upload.  Transforms, inverse transforms, the light's ShapeSet (world
    triangles, areas, CDF, sumArea), the ray epsilon and the rendered image equal
    those of the scene compiled on the host with the new transforms (bit-exact;
    the instance tree is refit on the device, rebuilt on the host)."""
    w, h = 96, 64
    d = instanced_scene(ctl, w, h)
    hs2, d2 = instanced_scene_xf(ctl, MOVES, w, h)   # hs2 owns d2's arrays
    d, d2 = (binary_bvh(d), binary_bvh(d2)) if bvh == "binary" else (d, d2)
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        pt.params = p
        for node, xf in MOVES.items():
            pt.set_transform(node, xf)
        A = ctl._abi
        xf = pt.read_array(A.CTL_ARRAY_NODE_XF, 0, d2.n_nodes, np.float32, 16)
        ixf = pt.read_array(A.CTL_ARRAY_NODE_INV_XF, 0, d2.n_nodes, np.float32, 16)
        lt = pt.read_array(A.CTL_ARRAY_LIGHT_TRIS, 0, d2.n_light_tris, np.uint32, 16)
        cdf = pt.read_array(A.CTL_ARRAY_LIGHT_CDF, 0, d2.n_light_tri_cdf, np.float32, 1)
        lights = pt.read_array(A.CTL_ARRAY_LIGHTS, 0, d2.n_lights, np.uint32, 12)
        eps = pt.read_array(A.CTL_ARRAY_RAY_EPS, 0, 1, np.float32, 1)
        box = pt.read_array(A.CTL_ARRAY_SCENE_BOX, 0, 1, np.float32, 6)
        sbvh = pt.read_array(A.CTL_ARRAY_SCENE_BVH, 0, d.n_scene_bvh_nodes, np.uint32, 16)
        trees = None if bvh == "binary" else device_wide_trees(pt, d)   # instance tree refit on the device
        fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        for k in range(3):
            pt.update_scene(d, 0)    # UpdateKernel each DoPass: the device's epsilon stays
            pt.do_pass(fb.data_ptr(), k)
        pt.sync()
        got, grays = fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()

    def arr(ptr, n, dt, width):
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n * width * 4,)).view(dt).reshape(n, width)
    assert np.array_equal(xf.view(np.uint32), arr(d2.node_xf, d2.n_nodes, np.uint32, 16))
    assert np.array_equal(ixf.view(np.uint32), arr(d2.node_inv_xf, d2.n_nodes, np.uint32, 16))
    assert np.array_equal(lt, arr(d2.light_tris, d2.n_light_tris, np.uint32, 16))
    assert np.array_equal(cdf.view(np.uint32), arr(d2.light_tri_cdf, d2.n_light_tri_cdf, np.uint32, 1))
    assert np.array_equal(lights, arr(d2.lights, d2.n_lights, np.uint32, 12))
    assert eps.view(np.uint32)[0, 0] == np.float32(d2.ray_eps).view(np.uint32)
    assert np.array_equal(box.view(np.uint32)[0], np.array(list(d2.box_min) + list(d2.box_max), np.float32).view(np.uint32))
    # the instance tree: SceneBVH::Build after each SetNodeTransform, along the moved
    # node's path with BVHRebuilder's rotations, from the previous call's tree
    scene = arr(d.scene_bvh_nodes, d.n_scene_bvh_nodes, np.float32, 16).copy()
    xfs = arr(d.node_xf, d.n_nodes, np.float32, 16).copy()
    mb = arr(d.mesh_boxes, d.n_meshes, np.float32, 6).copy()
    oeps = np.zeros(1, np.float32)
    for node, m in MOVES.items():
        xfs[node] = np.asarray(m, np.float32).reshape(16)
        orc.oracle_scene_set_transform(C.byref(d), oracle.ptr(scene), oracle.ptr(mb), oracle.ptr(xfs), node,
                                       oracle.ptr(oeps))
    assert np.array_equal(sbvh, scene.view(np.uint32))
    assert oeps[0] == eps[0, 0]
    want, wrays = oracle_render(orc, d2, p, 3, w, h, trees=trees)
    old, _ = oracle_render(orc, d, p, 3, w, h)
    assert not np.array_equal(old.view(np.uint32), want.view(np.uint32))   # the move is visible
    assert grays == wrays
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])

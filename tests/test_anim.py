"""Animated (skinned) meshes: AnimatedMesh::k_ComputeState (Engine/AnimatedMesh.cpp:163-184,
AnimatedMesh.cu:13-70) on the device through ctl_scene_animate, against the
oracle's restatement (skinning, TriangleData::setData on the device, Woop
data, box refit of the compiled trees, instance boxes, ray epsilon).  The
reference ships no animation fixture: the skinned tube below is synthetic
(parity pinned by the reference source, checked bit for bit against the
oracle, and BVH-independently against brute-force traversal)."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle
from helpers import binary_bvh, device_wide_trees, oracle_intersect, oracle_render, random_rays


def skinned_tube(nseg=24, nring=16, radius=0.5, length=4.0):
    """Cylinder along +y, two bones blended linearly along its length."""
    V, Nrm, BI, BW, UV = [], [], [], [], []
    for i in range(nseg + 1):
        y = length * i / nseg
        f = i / nseg
        w0 = int(round(255 * (1 - f)))
        for j in range(nring):
            a = 2 * math.pi * j / nring
            V.append([radius * math.cos(a), y, radius * math.sin(a)])
            Nrm.append([math.cos(a), 0.0, math.sin(a)])
            BI.append([0, 1, 0, 0, 0, 0, 0, 0])
            BW.append([w0, 255 - w0, 0, 0, 0, 0, 0, 0])
            UV.append([j / nring, f])
    T = []
    for i in range(nseg):
        for j in range(nring):
            a, b = i * nring + j, i * nring + (j + 1) % nring
            c, d = a + nring, b + nring
            T += [[a, c, b], [b, c, d]]
    return (np.array(V, np.float32), np.array(Nrm, np.float32), np.array(BI, np.uint8), np.array(BW, np.uint8),
            np.array(T, np.uint32), np.array(UV, np.float32))


def rot_z(deg, pivot):
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    R = np.eye(4, dtype=np.float32)
    R[0, 0], R[0, 1], R[1, 0], R[1, 1] = c, -s, s, c
    P = np.eye(4, dtype=np.float32); P[:3, 3] = pivot
    Pi = np.eye(4, dtype=np.float32); Pi[:3, 3] = [-p for p in pivot]
    return (P @ R @ Pi).astype(np.float32)


def frames():
    f0 = np.stack([np.eye(4, dtype=np.float32), rot_z(20, [0, 2, 0])])
    t = np.eye(4, dtype=np.float32); t[:3, 3] = [0.1, 0.0, -0.05]
    f1 = np.stack([t, rot_z(55, [0, 2, 0])])
    return f0, f1


def build_scene(ctl, w=64, h=48, light_on_tube=False):
    v, n, bi, bw, tris, uv = skinned_tube()
    s = ctl.HostScene()
    m_tube = s.add_animated_mesh(v, n, bi, bw, tris, [ctl.diffuse_material(0.7, 0.5, 0.3)], uvs=uv)
    ground = np.array([[-6, -0.5, -6], [6, -0.5, -6], [6, -0.5, 6], [-6, -0.5, 6]], np.float32)
    m_g = s.add_mesh(ground, [[0, 2, 1], [0, 3, 2]], [ctl.diffuse_material(0.5, 0.5, 0.5)])
    lq = np.array([[-1, 6, -1], [1, 6, -1], [1, 6, 1], [-1, 6, 1]], np.float32)
    m_l = s.add_mesh(lq, [[0, 1, 2], [0, 2, 3]], [ctl.diffuse_material(0.0, 0.0, 0.0)])
    n_tube = s.add_node(m_tube)
    s.add_node(m_tube, [1, 0, 0, 2.5, 0, 1, 0, 0, 0, 0, 1, 0.5, 0, 0, 0, 1])   # second instance
    s.add_node(m_g)
    nl = s.add_node(m_l)
    s.add_area_light(n_tube if light_on_tube else nl, 0, [20.0, 18.0, 15.0])
    s.set_camera([1.2, 2.5, -9], [1.2, 1.8, 0], [0, 1, 0], 50, w, h)
    return s


def _arr(ptr, ctype, n):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), shape=(n,)).copy()


def oracle_animated(ctl, orc, d, f0, f1, lerp, state=None):
    """Arrays after k_ComputeState, and a desc pointing at them.  The trees'
    shape persists between frames (BVHRebuilder rotates the tree it is given):
    pass the `keep` of the previous frame as `state` to continue from it."""
    A = ctl._abi
    tri = _arr(d.tri_data, C.c_uint32, d.n_tri_data * 8)
    woop = _arr(d.woop_tris, C.c_float, d.n_woop_tris * 12)
    if state is None:
        nodes = _arr(d.bvh_nodes, C.c_float, d.n_bvh_nodes * 16)
        scene = _arr(d.scene_bvh_nodes, C.c_float, max(1, d.n_scene_bvh_nodes) * 16)
        boxes = _arr(d.mesh_boxes, C.c_float, d.n_meshes * 6)
    else:
        nodes, scene, boxes = state[2].copy(), state[3].copy(), state[4].copy()
    eps = np.zeros(1, np.float32)
    b0 = np.ascontiguousarray(f0, np.float32)
    b1 = np.ascontiguousarray(f1, np.float32)
    orc.oracle_animate(C.byref(d), 0, oracle.ptr(b0), oracle.ptr(b1), lerp, oracle.ptr(tri), oracle.ptr(woop),
                       oracle.ptr(nodes), oracle.ptr(scene), oracle.ptr(boxes), oracle.ptr(eps))
    d2 = type(d).from_buffer_copy(d)
    d2.tri_data = C.cast(tri.ctypes.data, C.POINTER(A.TriangleData))
    d2.woop_tris = C.cast(woop.ctypes.data, C.POINTER(A.WoopTri))
    d2.bvh_nodes = C.cast(nodes.ctypes.data, C.POINTER(A.BVHNode))
    d2.scene_bvh_nodes = C.cast(scene.ctypes.data, C.POINTER(A.BVHNode))
    d2.mesh_boxes = C.cast(boxes.ctypes.data, C.POINTER(C.c_float))
    d2.ray_eps = float(eps[0])
    keep = (tri, woop, nodes, scene, boxes)
    return d2, keep, eps[0]


def check_tree(nodes, n_nodes, idx, root=0):
    """BVHRebuilder::validateTree (BVHRebuilder.cpp:575-606) on a mesh tree in
    the reference layout: parent words, every entry in exactly one leaf, every
    slot box containing what it bounds (leaf slots: the leaf's entries are
    checked by traversal elsewhere).  Returns the objects under the root."""
    n = nodes.view(np.int32).reshape(-1, 16)
    f = nodes.view(np.float32).reshape(-1, 16)
    seen = np.zeros(idx.size, bool)

    def walk(k, parent):
        assert n[k, 14] == parent
        total = 0
        for c in range(2):
            v = n[k, 12 + c]
            if v == 0x76543210:
                continue
            if v < 0:
                e = ~v
                while True:
                    assert not seen[e]
                    seen[e] = True
                    total += 1
                    if idx[e] & 1:
                        break
                    e += 1
            else:
                ch = v >> 2
                lo = np.array([f[ch, [0, 2, 8]], f[ch, [4, 6, 10]]]).min(0)
                hi = np.array([f[ch, [1, 3, 9]], f[ch, [5, 7, 11]]]).max(0)
                slot = f[k, [0, 2, 8]] if c == 0 else f[k, [4, 6, 10]]
                sloth = f[k, [1, 3, 9]] if c == 0 else f[k, [5, 7, 11]]
                assert (slot <= lo).all() and (sloth >= hi).all()
                total += walk(ch, k * 4)
        return total
    total = walk(root, -1)
    assert seen.all()
    return total


# ---------------------------------------------------------------------------- CPU

def test_animated_mesh_compiles_like_a_static_mesh(ctl):
    """Rest pose: the same arrays as add_mesh without reference splitting, plus
    the AnimatedVertex / triangle / mesh records of the desc."""
    v, n, bi, bw, tris, uv = skinned_tube()
    mats = [ctl.diffuse_material(0.7, 0.5, 0.3)]
    a = ctl.HostScene()
    a.add_animated_mesh(v, n, bi, bw, tris, mats, uvs=uv)
    a.add_node(0)
    a.set_camera([0, 2, -9], [0, 2, 0], [0, 1, 0], 50, 16, 16)
    da = a.compile()
    b = ctl.HostScene()
    b.set_bvh_builder("binned").set_bvh_params(0.0, 0)
    b.add_mesh(v, tris, mats, normals=n, uvs=uv)
    b.add_node(0)
    b.set_camera([0, 2, -9], [0, 2, 0], [0, 1, 0], 50, 16, 16)
    db = b.compile()
    for f, ct, w in [("tri_data", C.c_uint32, 8), ("woop_tris", C.c_uint32, 12), ("bvh_nodes", C.c_uint32, 16)]:
        cnt = {"tri_data": da.n_tri_data, "woop_tris": da.n_woop_tris, "bvh_nodes": da.n_bvh_nodes}[f]
        assert np.array_equal(_arr(getattr(da, f), ct, cnt * w), _arr(getattr(db, f), ct, cnt * w)), f
    assert da.n_anim_meshes == 1 and da.n_anim_vertices == len(v) and da.n_anim_triangles == len(tris)
    am = da.anim_meshes[0]
    assert (am.mesh, am.vertex_first, am.vertex_count, am.tri_first, am.tri_count, am.max_bone) == \
        (0, 0, len(v), 0, len(tris), 1)
    av = da.anim_vertices[5]
    assert list(av.pos) == v[5].tolist() and av.bone_weights == int(bw[5].view(np.uint64)[0])
    assert db.n_anim_meshes == 0


def test_area_light_on_animated_mesh_refused(ctl):
    s = build_scene(ctl, light_on_tube=True)
    with pytest.raises(ctl.CTLError, match="animated"):
        s.compile()


def test_oracle_refit_at_rest_reproduces_the_build(ctl, orc):
    """Identity bones, lerp 0: the refit boxes equal the builder's child boxes and
    the Woop data the compile's (both are exact functions of the vertices)."""
    eye = np.stack([np.eye(4, dtype=np.float32)] * 2)
    v, n, bi, bw, tris, uv = skinned_tube()
    # weights (w0, 255 - w0) blend the identity to a matrix that is not exactly
    # the identity: one bone at weight 255 keeps the rest pose exact
    s = ctl.HostScene()
    s.add_animated_mesh(v, n, np.zeros_like(bi), np.array([[255, 0, 0, 0, 0, 0, 0, 0]] * len(v), np.uint8), tris,
                        [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=uv)
    s.add_node(0)
    s.add_node(0, [1, 0, 0, 3, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    s.set_camera([0, 2, -9], [0, 2, 0], [0, 1, 0], 50, 16, 16)
    d = s.compile()
    d3, keep3, eps3 = oracle_animated(ctl, orc, d, eye[:1], eye[:1], 0.0)
    assert np.array_equal(keep3[1].view(np.uint32), _arr(d.woop_tris, C.c_uint32, d.n_woop_tris * 12))
    assert np.array_equal(keep3[2].view(np.uint32), _arr(d.bvh_nodes, C.c_uint32, d.n_bvh_nodes * 16))
    assert np.array_equal(keep3[3][:d.n_scene_bvh_nodes * 16].view(np.uint32),
                          _arr(d.scene_bvh_nodes, C.c_uint32, d.n_scene_bvh_nodes * 16))
    assert np.float32(eps3) == np.float32(d.ray_eps)


def test_oracle_refit_traversal_matches_brute_force(ctl, orc):
    """The refit tree bounds the moved triangles: traceRay over it finds what a
    scan over every triangle finds (BVH-independent truth)."""
    from helpers import oracle_trace
    s = build_scene(ctl)
    d = s.compile()
    f0, f1 = frames()
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.8)
    rays = random_rays(d2, 20000, seed=5)
    t, u, v, tri, node, st = oracle_trace(orc, d2, rays, mode=0)
    bt = np.zeros(rays.shape[0], np.float32)
    btri = np.zeros(rays.shape[0], np.uint32)
    orc.oracle_brute_force(C.byref(d2), rays.shape[0], oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
    assert (tri != 0xFFFFFFFF).sum() > 2000
    assert np.array_equal(t, bt) and np.array_equal(tri, btri)


def test_oracle_rebuild_rotates_and_keeps_a_valid_tree(ctl, orc):
    """BVHRebuilder's rotations (BVHRebuilder.cpp:306-334) on the animated tube,
    frame after frame from the last frame's tree: subtrees move (children and
    parent words change), the tree stays valid (validateTree) and traversal
    over it still finds what a scan over every triangle finds."""
    from helpers import oracle_trace
    s = build_scene(ctl)
    d = s.compile()
    f0, f1 = frames()
    idx = _arr(d.tri_indices, C.c_uint32, d.n_tri_indices)
    k0 = d.meshes[0].bvh_indices_offset
    k1 = d.meshes[1].bvh_indices_offset
    n1 = d.meshes[1].bvh_node_offset // 4
    rest = _arr(d.bvh_nodes, C.c_int32, d.n_bvh_nodes * 16).reshape(-1, 16)
    keep = None
    moved = 0
    for lerp in (0.2, 0.5, 0.9, 0.3):
        d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, lerp, keep)
        tube = keep[2][:n1 * 16].view(np.int32)
        assert check_tree(tube, n1, idx[k0:k1]) == k1 - k0
        moved = max(moved, int((tube.reshape(-1, 16)[:, 12:14] != rest[:n1, 12:14]).any(1).sum()))
        rays = random_rays(d2, 5000, seed=int(lerp * 10))
        t, u, v, tri, node, st = oracle_trace(orc, d2, rays, mode=0)
        bt = np.zeros(rays.shape[0], np.float32)
        btri = np.zeros(rays.shape[0], np.uint32)
        orc.oracle_brute_force(C.byref(d2), rays.shape[0], oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
        assert np.array_equal(t, bt) and np.array_equal(tri, btri)
    assert moved > 20


def test_oracle_rebuild_grid_moves_inner_nodes(ctl, orc):
    """On a deeper tree (a skinned grid) rotations move inner subtrees too: their
    parent words change, and the tree stays valid."""
    V, N, BI, BW, T, UV = skinned_grid(64)
    s = ctl.HostScene()
    s.add_animated_mesh(V, N, BI, BW, T, [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=UV)
    s.add_node(0)
    s.add_node(0, [1, 0, 0, 25, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    s.set_camera([0, 8, -20], [0, 0, 0], [0, 1, 0], 50, 16, 16)
    d = s.compile()
    idx = _arr(d.tri_indices, C.c_uint32, d.n_tri_indices)
    rest = _arr(d.bvh_nodes, C.c_int32, d.n_bvh_nodes * 16).reshape(-1, 16)
    keep = None
    for t in (0.5, 1.5, 2.5):
        d2, keep, eps = oracle_animated(ctl, orc, d, grid_frames(16, 0.0), grid_frames(16, t), 1.0, keep)
        nodes = keep[2].view(np.int32)
        assert check_tree(nodes, d.n_bvh_nodes, idx) == d.n_tri_indices
    parents = int((nodes.reshape(-1, 16)[:, 14] != rest[:, 14]).sum())
    assert parents > 10


# ---------------------------------------------------------------------------- GPU

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_animate_arrays_bit_exact(ctl, orc, dev, bvh):
    A = ctl._abi
    s = build_scene(ctl)
    d = s.compile()
    if bvh == "binary":
        d = binary_bvh(d)
    f0, f1 = frames()
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.animate(0, f0, f1, 0.25)      # a first pose, then the one compared: the tree's shape carries over
    pt.animate(0, f0, f1, 0.4)
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.25)
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.4, keep)
    tri, woop, nodes, scene, boxes = keep
    got = pt.read_array(A.CTL_ARRAY_TRI_DATA, 0, d.n_tri_data, np.uint32, 8)
    assert np.array_equal(got.ravel(), tri)
    assert not np.array_equal(tri, _arr(d.tri_data, C.c_uint32, d.n_tri_data * 8))   # it moved
    got = pt.read_array(A.CTL_ARRAY_WOOP, 0, d.n_woop_tris, np.uint32, 12)
    assert np.array_equal(got.ravel(), woop.view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_BVH_NODES, 0, d.n_bvh_nodes, np.uint32, 16)
    assert np.array_equal(got.ravel(), nodes.view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_SCENE_BVH, 0, d.n_scene_bvh_nodes, np.uint32, 16)
    assert np.array_equal(got.ravel(), scene[:d.n_scene_bvh_nodes * 16].view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
    assert np.array_equal(got.ravel().view(np.uint32), boxes.view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_RAY_EPS, 0, 1, np.float32, 1)
    assert got[0, 0] == eps
    pt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_animated_traversal_and_render_bit_exact(ctl, orc, dev, bvh):
    """Refit trees (binary and the 4-wide copy) traverse to the oracle's hits on
    the oracle's animated arrays; hits agree with brute force; a 2-pass render
    is bit-exact."""
    w, h = 64, 48
    s = build_scene(ctl, w, h)
    d = s.compile()
    if bvh == "binary":
        d = binary_bvh(d)
    f0, f1 = frames()
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.animate(0, f0, f1, 0.6)
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.6)
    rays = random_rays(d2, 20000, seed=3, tmin=d2.ray_eps)   # batch tmin = traceRay's eps (brute force below)
    trees = None if bvh == "binary" else device_wide_trees(pt, d)   # refit boxes, the upload's topology
    want = oracle_intersect(orc, d2, rays, trees=trees)
    r = torch.from_numpy(rays).to(dev)
    hits = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(rays.shape[0], r.data_ptr(), hits.data_ptr(), False)
    torch.cuda.synchronize()
    got = hits.cpu().numpy()
    assert np.array_equal(got, want)
    hit = want[:, 2] != -1
    assert hit.sum() > 1000
    bt = np.zeros(rays.shape[0], np.float32)
    btri = np.zeros(rays.shape[0], np.uint32)
    orc.oracle_brute_force(C.byref(d2), rays.shape[0], oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
    assert np.array_equal(got[:, 0].view(np.float32)[hit], bt[hit])
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    want_fb, wrays = oracle_render(orc, d2, p, 2, w, h, trees=trees)
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    pt.params = p
    pt.reset_rays()
    for k in range(2):
        pt.do_pass(fb.data_ptr(), k)
    torch.cuda.synchronize()
    got_fb = fb.cpu().numpy()
    assert pt.rays_traced() == wrays
    assert np.array_equal(got_fb.view(np.uint32), want_fb.view(np.uint32))
    pt.close()


@pytest.mark.gpu
def test_cull_bound_covers_animated_boxes_and_follows_instance_update(ctl, orc, dev):
    """DevScene::cull_m bounds every box the any-hit shadow query tests (the
    slack of traverse.h slab_slack).  The tube is moved 40 along x: after
    ctl_scene_animate the bound covers the moved mesh boxes.  An instance-only
    ctl_scene_update (CTL_DIRTY_NODES) re-derives the bound from the desc; it
    also returns every device-edited array to the desc (commit re-uploads the
    trees with the instances), so the boxes on the device are the rest pose's
    again and the desc's bound holds for them (advisor round 5: a NODES-only
    update never leaves moved trees behind a rest-pose bound)."""
    A = ctl._abi
    s = build_scene(ctl)
    d = s.compile()
    bump = np.stack([np.eye(4, dtype=np.float32)] * 2)
    bump[:, 0, 3] = 40.0                                     # both bones: the tube moves 40 along x
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        rest = pt.read_array(A.CTL_ARRAY_CULL_BOUND, 0, 1, np.float32, 3)[0].copy()
        rest_boxes = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
        pt.animate(0, bump, bump, 0.0)
        boxes = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
        moved = np.abs(boxes).reshape(-1, 2, 3).max(axis=(0, 1))
        assert moved[0] > 40.0 > rest[0]
        after_anim = pt.read_array(A.CTL_ARRAY_CULL_BOUND, 0, 1, np.float32, 3)[0].copy()
        assert (after_anim >= moved).all()
        pt.update_scene(d, A.CTL_DIRTY_NODES)
        back = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
        assert np.array_equal(back.view(np.uint32), rest_boxes.view(np.uint32))
        nodes = pt.read_array(A.CTL_ARRAY_BVH_NODES, 0, d.n_bvh_nodes, np.uint32, 16)
        assert np.array_equal(nodes.ravel(), _arr(d.bvh_nodes, C.c_uint32, d.n_bvh_nodes * 16))
        after_nodes = pt.read_array(A.CTL_ARRAY_CULL_BOUND, 0, 1, np.float32, 3)[0]
        assert np.array_equal(after_nodes, rest)
        assert (after_nodes >= np.abs(back).reshape(-1, 2, 3).max(axis=(0, 1))).all()
    finally:
        pt.close()


def skinned_grid(n, bones=16):
    """n x n quads in the xz plane (2 n^2 triangles), 4 random bone influences per
    vertex: a mesh tree deep and wide enough for every refit stage (one-block
    subtrees, per-level launches above them, the single-block top)."""
    xs = np.linspace(-10, 10, n + 1, dtype=np.float32)
    X, Z = np.meshgrid(xs, xs, indexing="xy")
    V = np.stack([X.ravel(), np.zeros(X.size, np.float32), Z.ravel()], 1).astype(np.float32)
    N = np.tile(np.array([[0, 1, 0]], np.float32), (V.shape[0], 1))
    rng = np.random.default_rng(0)
    BI = np.zeros((V.shape[0], 8), np.uint8)
    BI[:, :4] = rng.integers(0, bones, size=(V.shape[0], 4), dtype=np.uint8)
    BW = np.zeros((V.shape[0], 8), np.uint8)
    BW[:, :4] = [64, 64, 64, 63]
    q = np.arange(n * n, dtype=np.uint32)
    i, j = q // n, q % n
    a = i * (n + 1) + j
    b, c, d = a + 1, a + n + 1, a + n + 2
    T = np.concatenate([np.stack([a, c, b], 1), np.stack([b, c, d], 1)]).astype(np.uint32)
    UV = np.stack([(X.ravel() + 10) / 20, (Z.ravel() + 10) / 20], 1).astype(np.float32)
    return V, N, BI, BW, T, UV


def grid_frames(bones, t):
    out = []
    for k in range(bones):
        a = math.radians(5 * math.sin(t + k))
        m = np.eye(4, dtype=np.float32)
        m[0, 0], m[0, 1], m[1, 0], m[1, 1] = math.cos(a), -math.sin(a), math.sin(a), math.cos(a)
        m[1, 3] = 0.2 * math.sin(t * 0.5 + k)
        out.append(m)
    return np.stack(out)


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_animate_large_grid_bit_exact(ctl, orc, dev, bvh):
    """The 2 M-triangle skinned grid of tools/tools_anim_bench.py: ~1 M binary
    nodes rebuilt by ~0.5 M leaf threads climbing with arrival counters and
    rotating on the way (two frames, the second from the first's tree); every
    array equals the oracle's bit for bit, and traversal over the 4-wide copy
    (refit in its upload topology) equals the oracle's over the same trees."""
    A = ctl._abi
    V, N, BI, BW, T, UV = skinned_grid(1024)
    s = ctl.HostScene()
    s.add_animated_mesh(V, N, BI, BW, T, [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=UV)
    s.add_node(0)
    s.add_node(0, [1, 0, 0, 25, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    s.set_camera([0, 8, -20], [0, 0, 0], [0, 1, 0], 50, 16, 16)
    d = s.compile()
    assert d.n_bvh_nodes > 500000
    if bvh == "binary":
        d = binary_bvh(d)
    f0, f1 = grid_frames(16, 0.0), grid_frames(16, 1.0)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.animate(0, f0, f1, 0.3)
    pt.animate(0, f0, f1, 0.7)
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.3)
    d2, keep, eps = oracle_animated(ctl, orc, d, f0, f1, 0.7, keep)
    tri, woop, nodes, scene, boxes = keep
    got = pt.read_array(A.CTL_ARRAY_BVH_NODES, 0, d.n_bvh_nodes, np.uint32, 16)
    assert np.array_equal(got.ravel(), nodes.view(np.uint32))
    assert not np.array_equal(nodes.view(np.uint32), _arr(d.bvh_nodes, C.c_uint32, d.n_bvh_nodes * 16))   # it moved
    got = pt.read_array(A.CTL_ARRAY_WOOP, 0, d.n_woop_tris, np.uint32, 12)
    assert np.array_equal(got.ravel(), woop.view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_SCENE_BVH, 0, d.n_scene_bvh_nodes, np.uint32, 16)
    assert np.array_equal(got.ravel(), scene[:d.n_scene_bvh_nodes * 16].view(np.uint32))
    got = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
    assert np.array_equal(got.ravel().view(np.uint32), boxes.view(np.uint32))
    if bvh == "wide":   # the 4-wide copy, refit in the topology the upload collapsed
        trees = device_wide_trees(pt, d)
        rays = random_rays(d2, 20000, seed=7, tmin=d2.ray_eps)
        want = oracle_intersect(orc, d2, rays, trees=trees)
        r = torch.from_numpy(rays).to(dev)
        hits = torch.zeros((rays.shape[0], 4), dtype=torch.int32, device=dev)
        pt.intersect_buffers(rays.shape[0], r.data_ptr(), hits.data_ptr(), False)
        torch.cuda.synchronize()
        assert np.array_equal(hits.cpu().numpy(), want)
        assert (want[:, 2] != -1).sum() > 1000
    pt.close()


@pytest.mark.gpu
def test_rebuild_deterministic_across_contexts(ctl, dev):
    """The rebuild's threads climb the tree in whatever order they arrive, on every
    XCD: the result must not depend on it.  Two contexts animate the 512 x 512
    skinned grid through the same 4 frames (each frame from the last one's tree);
    their node arrays, Woop data, 4-wide trees and mesh boxes are identical after
    every frame."""
    A = ctl._abi
    V, N, BI, BW, T, UV = skinned_grid(512)
    s = ctl.HostScene()
    s.add_animated_mesh(V, N, BI, BW, T, [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=UV)
    s.add_node(0)
    s.add_node(0, [1, 0, 0, 25, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    s.set_camera([0, 8, -20], [0, 0, 0], [0, 1, 0], 50, 16, 16)
    d = s.compile()
    nw = ctl.host_wide_trees(d)[0].shape[0]
    pts = [ctl.PathTracer(0), ctl.PathTracer(0)]
    try:
        for pt in pts:
            pt.upload_scene(d)
        for t in (0.4, 1.3, 2.2, 3.1):
            got = []
            for pt in pts:
                pt.animate(0, grid_frames(16, 0.0), grid_frames(16, t), 0.9)
                got.append((pt.read_array(A.CTL_ARRAY_BVH_NODES, 0, d.n_bvh_nodes, np.uint32, 16),
                            pt.read_array(A.CTL_ARRAY_WOOP, 0, d.n_woop_tris, np.uint32, 12),
                            pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.uint32, 6),
                            pt.read_array(A.CTL_ARRAY_WIDE_BVH, 0, nw, np.uint32, 32)))
            for a, b in zip(*got):
                assert np.array_equal(a, b), t
    finally:
        for pt in pts:
            pt.close()


@pytest.mark.gpu
def test_animate_rejects_bad_bones(ctl, dev):
    s = build_scene(ctl)
    d = s.compile()
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    eye = np.stack([np.eye(4, dtype=np.float32)])
    with pytest.raises(ctl.CTLError, match="bone"):
        pt.animate(0, eye, eye, 0.5)         # the tube uses bone 1
    with pytest.raises(ctl.CTLError):
        pt.animate(1, eye, eye, 0.5)         # one animated mesh only
    pt.close()


def expected_wide(upload, wbase, d, nodes):
    """The 4-wide mesh trees as the rebuild must leave them: the upload's
    topology, each leaf slot the leaf's box (read from the binary tree's slot
    that holds it: BVHNodeData's leaf box is its triangles' boxes extended from
    AABB::Identity), each inner slot the union of the child node's occupied slots
    in slot order (from AABB::Identity, `a < b ? a : b`), empty slots as
    uploaded."""
    out = upload.copy()
    wi = out.view(np.int32)
    f = nodes.view(np.float32).reshape(-1, 16)
    n = nodes.view(np.int32).reshape(-1, 16)
    nw = upload.shape[0]
    for m in range(d.n_meshes):
        k0 = d.meshes[m].bvh_node_offset // 4
        k1 = d.meshes[m + 1].bvh_node_offset // 4 if m + 1 < d.n_meshes else d.n_bvh_nodes
        w0, w1 = int(wbase[m]), int(wbase[m + 1]) if m + 1 < d.n_meshes else nw
        leaf = {}
        for k in range(k0, k1):
            for c in range(2):
                v = n[k, 12 + c]
                if v < 0:
                    leaf[~v] = (f[k, [0, 2, 8]] if c == 0 else f[k, [4, 6, 10]],
                                f[k, [1, 3, 9]] if c == 0 else f[k, [5, 7, 11]])
        post, st = [], [w0]
        while st:
            k = st.pop()
            post.append(k)
            st += [w0 + v for v in wi[k, 24:28] if 0 <= v != 0x76543210]
        for k in reversed(post):
            for q in range(4):
                v = wi[k, 24 + q]
                if v == 0x76543210:
                    continue
                if v < 0:
                    lo, hi = leaf[(~v) >> 3]
                else:
                    ch = w0 + v
                    lo = np.full(3, np.finfo(np.float32).max, np.float32)
                    hi = -lo
                    for r in range(4):
                        if wi[ch, 24 + r] == 0x76543210:
                            continue
                        clo, chi = out[ch, [r, 8 + r, 16 + r]], out[ch, [4 + r, 12 + r, 20 + r]]
                        lo, hi = np.where(lo < clo, lo, clo), np.where(hi > chi, hi, chi)
                out[k, [q, 8 + q, 16 + q]] = lo
                out[k, [4 + q, 12 + q, 20 + q]] = hi
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_small_and_several_animated_meshes_bit_exact(ctl, orc, dev, bvh):
    """Three animated meshes (1 triangle: a root with one empty slot; 3
    triangles; the tube) animated in turn over three rounds, each frame from the
    last one's trees: every array equals the oracle's, and the 4-wide copy equals
    its upload topology refit from the oracle's leaf boxes (expected_wide)."""
    A = ctl._abi
    s = ctl.HostScene()
    one = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    three = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0.5], [2, 0, 0.2]], np.float32)
    small = []
    for V, T in ((one, [[0, 1, 2]]), (three, [[0, 1, 2], [1, 3, 2], [1, 4, 3]])):
        nv = V.shape[0]
        bi = np.zeros((nv, 8), np.uint8)
        bi[:, 1] = 1
        bw = np.zeros((nv, 8), np.uint8)
        bw[:, 0], bw[:, 1] = 200, 55
        nrm = np.tile(np.array([[0, 0, 1]], np.float32), (nv, 1))
        small.append(s.add_animated_mesh(V, nrm, bi, bw, np.array(T, np.uint32), [ctl.diffuse_material(0.6, 0.6, 0.6)],
                                         uvs=V[:, :2].copy()))
    v, nrm, bi, bw, tris, uv = skinned_tube()
    m_tube = s.add_animated_mesh(v, nrm, bi, bw, tris, [ctl.diffuse_material(0.7, 0.5, 0.3)], uvs=uv)
    ground = np.array([[-6, -0.5, -6], [6, -0.5, -6], [6, -0.5, 6], [-6, -0.5, 6]], np.float32)
    m_g = s.add_mesh(ground, [[0, 2, 1], [0, 3, 2]], [ctl.diffuse_material(0.5, 0.5, 0.5)])
    for i, m in enumerate(small + [m_tube]):
        s.add_node(m, [1, 0, 0, 2.0 * i, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
    nl = s.add_node(m_g)
    s.add_area_light(nl, 0, [5.0, 5.0, 5.0])
    s.set_camera([1.2, 2.5, -9], [1.2, 1.8, 0], [0, 1, 0], 50, 32, 24)
    d = s.compile()
    if bvh == "binary":
        d = binary_bvh(d)
    f0, f1 = frames()
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    upload = None if bvh == "binary" else pt.wide_trees(d)
    keep = None
    for rnd in range(3):
        for anim in range(3):
            lerp = 0.2 + 0.25 * rnd + 0.05 * anim
            pt.animate(anim, f0, f1, lerp)
            tri = _arr(d.tri_data, C.c_uint32, d.n_tri_data * 8) if keep is None else keep[0]
            woop = _arr(d.woop_tris, C.c_float, d.n_woop_tris * 12) if keep is None else keep[1]
            if keep is None:
                nodes = _arr(d.bvh_nodes, C.c_float, d.n_bvh_nodes * 16)
                scene = _arr(d.scene_bvh_nodes, C.c_float, max(1, d.n_scene_bvh_nodes) * 16)
                boxes = _arr(d.mesh_boxes, C.c_float, d.n_meshes * 6)
            else:
                nodes, scene, boxes = keep[2], keep[3], keep[4]
            eps = np.zeros(1, np.float32)
            orc.oracle_animate(C.byref(d), anim, oracle.ptr(f0), oracle.ptr(f1), lerp, oracle.ptr(tri),
                               oracle.ptr(woop), oracle.ptr(nodes), oracle.ptr(scene), oracle.ptr(boxes),
                               oracle.ptr(eps))
            keep = (tri, woop, nodes, scene, boxes)
            got = pt.read_array(A.CTL_ARRAY_BVH_NODES, 0, d.n_bvh_nodes, np.uint32, 16)
            assert np.array_equal(got.ravel(), nodes.view(np.uint32)), (rnd, anim)
            got = pt.read_array(A.CTL_ARRAY_WOOP, 0, d.n_woop_tris, np.uint32, 12)
            assert np.array_equal(got.ravel(), woop.view(np.uint32)), (rnd, anim)
            got = pt.read_array(A.CTL_ARRAY_TRI_DATA, 0, d.n_tri_data, np.uint32, 8)
            assert np.array_equal(got.ravel(), tri), (rnd, anim)
            got = pt.read_array(A.CTL_ARRAY_SCENE_BVH, 0, d.n_scene_bvh_nodes, np.uint32, 16)
            assert np.array_equal(got.ravel(), scene[:d.n_scene_bvh_nodes * 16].view(np.uint32)), (rnd, anim)
            got = pt.read_array(A.CTL_ARRAY_MESH_BOXES, 0, d.n_meshes, np.float32, 6)
            assert np.array_equal(got.ravel().view(np.uint32), boxes.view(np.uint32)), (rnd, anim)
            assert pt.read_array(A.CTL_ARRAY_RAY_EPS, 0, 1, np.float32, 1)[0, 0] == eps[0]
            if upload is not None:
                mesh, wbase, _ = pt.wide_trees(d)
                want = expected_wide(upload[0], upload[1], d, nodes)
                assert np.array_equal(mesh.view(np.uint32), want.view(np.uint32)), (rnd, anim)
    n = nodes.view(np.int32).reshape(-1, 16)
    assert (n[:, 12:14] == 0x76543210).any()   # the 1-triangle mesh's root keeps an empty slot
    pt.close()

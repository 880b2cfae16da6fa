"""The reference's per-pass UpdateKernel and its incremental DynamicScene::
UpdateScene through ctl_scene_update (Kernel/Tracer.h:229,
Kernel/TraceHelper.cu:182-217, Engine/DynamicScene.cpp:480-554): the scene
constants every call, the arrays the caller marks dirty and nothing else.
Each case renders after the update and compares with the oracle over the
updated desc, bit for bit (full-size C3 DoPass loop: test_gpu_fullsize.py)."""
import ctypes as C
import time

import numpy as np
import pytest

from helpers import binary_bvh, oracle_render

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

W, H = 96, 64


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def scene(ctl, config=2, scale=0.05, builder="sbvh"):
    hs = ctl.HostScene().generate(config, scale, W, H)
    hs.set_bvh_builder(builder)
    return hs, hs.compile()


def copy_desc(d):
    return type(d).from_buffer_copy(d)


def render(ctl, pt, dev, passes, first=0):
    fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
    pt.reset_rays()
    for k in range(passes):
        pt.do_pass(fb.data_ptr(), first + k)
    pt.sync()
    return fb.cpu().numpy(), pt.rays_traced()


def same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


P = None


def params(ctl):
    return ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)


@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_update_clean_scene_is_cheap_and_exact(ctl, orc, dev, bvh):
    """dirty = 0 (the reference's UpdateKernel every DoPass): no copy, no sync,
    microseconds, and the passes equal those of a context that never updated."""
    hs, d = scene(ctl)
    d = binary_bvh(d) if bvh == "binary" else d
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        times = []
        for k in range(10):
            t0 = time.perf_counter()
            pt.update_scene(d, 0)
            times.append(time.perf_counter() - t0)
            pt.do_pass(fb.data_ptr(), k)
        pt.sync()
        got = fb.cpu().numpy()
    finally:
        pt.close()
    want, _ = oracle_render(orc, d, params(ctl), 10, W, H)
    assert same(got, want)
    assert max(times) < 1e-3, times


def test_update_camera_and_materials(ctl, orc, dev):
    """A moved camera (scene constant, dirty = 0) and edited materials
    (CTL_DIRTY_MATERIALS): the next pass is the oracle's over the edited desc."""
    hs, d = scene(ctl)
    hs2, d2 = scene(ctl)
    hs2.set_camera((3.0, 2.5, -14.0), (0.0, 1.0, 0.0), (0, 1, 0), 50.0, W, H)
    d2 = hs2.compile()
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        e = copy_desc(d)
        e.camera = d2.camera                      # DoPass after the sensor moved
        pt.update_scene(e, 0)
        got, grays = render(ctl, pt, dev, 2)
        want, wrays = oracle_render(orc, e, params(ctl), 2, W, H)
        assert grays == wrays and same(got, want)
        # edit every material's reflectance in the host array, then mark it dirty
        for i in range(d.n_materials):
            m = d.materials[i]
            m.reflectance[0], m.reflectance[2] = m.reflectance[2] * 0.5, min(1.0, m.reflectance[0] * 1.2)
        pt.update_scene(d, ctl._abi.CTL_DIRTY_MATERIALS)
        got, grays = render(ctl, pt, dev, 2, first=5)
        want, wrays = oracle_render(orc, d, params(ctl), 2, W, H, first_pass=5)
        assert grays == wrays and same(got, want)
    finally:
        pt.close()


def test_update_refuses_unmarked_size_change(ctl, orc, dev):
    """An array whose count changed without its dirty bit is refused and the
    uploaded scene stays as it was."""
    hs, d = scene(ctl)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        e = copy_desc(d)
        e.n_tri_data = d.n_tri_data - 1
        with pytest.raises(ctl.CTLError, match="tri_data"):
            pt.update_scene(e, 0)
        got, _ = render(ctl, pt, dev, 1)
        want, _ = oracle_render(orc, d, params(ctl), 1, W, H)
        assert same(got, want)
    finally:
        pt.close()


@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_update_rebuilt_geometry(ctl, orc, dev, bvh):
    """A new BVH (another builder: every tree array changes size) through
    ctl_scene_update(CTL_DIRTY_ALL): arrays reallocated, 4-wide trees rebuilt."""
    hs, d = scene(ctl, builder="sbvh")
    hs2, d2 = scene(ctl, builder="binned")
    assert d2.n_bvh_nodes != d.n_bvh_nodes
    d, d2 = (binary_bvh(d), binary_bvh(d2)) if bvh == "binary" else (d, d2)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        render(ctl, pt, dev, 1)
        pt.update_scene(d2, ctl._abi.CTL_DIRTY_ALL)
        got, grays = render(ctl, pt, dev, 2, first=3)
        assert pt.stack_bound() > 0
    finally:
        pt.close()
    want, wrays = oracle_render(orc, d2, params(ctl), 2, W, H, first_pass=3)
    assert grays == wrays and same(got, want)


def test_update_switches_tree_format(ctl, orc, dev):
    """CTL_SCENE_BINARY_BVH toggled between updates: the device trees follow the
    flag without any dirty bit (the format is a scene constant)."""
    hs, d = scene(ctl)
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        b = binary_bvh(d)
        pt.update_scene(b, 0)
        got, grays = render(ctl, pt, dev, 1, first=2)
        want, wrays = oracle_render(orc, b, params(ctl), 1, W, H, first_pass=2)
        assert grays == wrays and same(got, want)
        pt.update_scene(d, 0)
        got, grays = render(ctl, pt, dev, 1, first=2)
        want, wrays = oracle_render(orc, d, params(ctl), 1, W, H, first_pass=2)
        assert grays == wrays and same(got, want)
    finally:
        pt.close()


@pytest.mark.parametrize("bvh", ["wide"])
def test_update_tri_indices_alone_rebuilds_trees(ctl, orc, dev, bvh):
    """CTL_DIRTY_TRI_INDICES alone, same size: the 4-wide trees
    carry per-leaf entry counts and relaid entries derived from the
    TriIntersectorData2 flags, so they are rebuilt.  The update merges leaves
    (a cleared last-in-leaf flag) and renames triangles; the image equals the
    oracle's over the new arrays in the device order and in the reference's."""
    from helpers import select_bvh, tie_rule
    hs, d = scene(ctl)
    d = select_bvh(d, bvh)
    idx = np.ctypeslib.as_array(C.cast(d.tri_indices, C.POINTER(C.c_uint32)), shape=(d.n_tri_indices,)).copy()
    ends = np.nonzero(idx[:-1] & 1)[0]
    merge = ends[::5]
    idx2 = idx.copy()
    idx2[merge] &= ~np.uint32(1)                        # the leaf runs on into the next one's entries
    ntri = int(d.n_tri_data)
    idx2 = ((((idx2 >> 1) + 7) % ntri) << 1) | (idx2 & 1)   # and names other triangles
    d2 = copy_desc(d)
    d2.tri_indices = idx2.ctypes.data_as(C.POINTER(C.c_uint32))
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        render(ctl, pt, dev, 1)
        pt.update_scene(d2, ctl._abi.CTL_DIRTY_TRI_INDICES)
        got, grays = render(ctl, pt, dev, 2, first=3)
    finally:
        pt.close()
    want, wrays = oracle_render(orc, d2, params(ctl), 2, W, H, first_pass=3)
    assert grays == wrays and same(got, want)
    ref = np.zeros_like(want)
    import oracle
    for p in (3, 4):
        orc.oracle_render_pass(C.byref(d2), C.byref(params(ctl)), p, oracle.ptr(ref), 0, 0, 1, None)
    assert same(got, ref)                               # and the reference order agrees
    old, _ = oracle_render(orc, d, params(ctl), 2, W, H, first_pass=3)
    assert not same(old, want)                          # the update is visible
    del idx2


def test_set_transform_then_tree_update_returns_to_desc(ctl, orc, dev):
    """After ctl_scene_set_transform, an update that re-uploads a tree group
    (CTL_DIRTY_MESHES) returns the transforms, the instance tree, the moved
    light's ShapeSet and the epsilon to the desc together: the image and the
    light records equal those of the unmoved scene."""
    from test_gpu_instances import MOVES, instanced_scene
    d = instanced_scene(ctl, W, H)
    A = ctl._abi
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        lt0 = pt.read_array(A.CTL_ARRAY_LIGHT_TRIS, 0, d.n_light_tris, np.uint32, 16)
        for node, xf in MOVES.items():
            pt.set_transform(node, xf)
        moved = pt.read_array(A.CTL_ARRAY_LIGHT_TRIS, 0, d.n_light_tris, np.uint32, 16)
        assert not np.array_equal(moved, lt0)
        pt.update_scene(d, A.CTL_DIRTY_MESHES)
        lt = pt.read_array(A.CTL_ARRAY_LIGHT_TRIS, 0, d.n_light_tris, np.uint32, 16)
        xf = pt.read_array(A.CTL_ARRAY_NODE_XF, 0, d.n_nodes, np.float32, 16)
        pt.params = params(ctl)
        got, grays = render(ctl, pt, dev, 2)
    finally:
        pt.close()
    assert np.array_equal(lt, lt0)
    want_xf = np.ctypeslib.as_array(C.cast(d.node_xf, C.POINTER(C.c_float)), shape=(d.n_nodes * 16,))
    assert np.array_equal(xf.ravel().view(np.uint32), want_xf.view(np.uint32))
    want, wrays = oracle_render(orc, d, params(ctl), 2, W, H)
    assert grays == wrays and same(got, want)

"""The product's host scene compiler (libctl_trace.so, no GPU) against the
oracle's restatement of the reference host code: bit-exact."""
import ctypes as C

import numpy as np
import pytest

import oracle


def test_woop_bit_exact(ctl, orc):
    L = ctl.lib()
    rng = np.random.default_rng(7)
    for _ in range(500):
        v = (rng.normal(size=(3, 3)) * rng.choice([1e-2, 1, 100])).astype(np.float32)
        a = np.zeros(12, np.float32)
        orc.oracle_woop_set(oracle.ptr(v[0]), oracle.ptr(v[1]), oracle.ptr(v[2]), oracle.ptr(a))
        w = ctl._abi.WoopTri()
        L.ctl_woop_set(v[0].ctypes.data, v[1].ctypes.data, v[2].ctypes.data, C.byref(w))
        assert np.array_equal(np.array(w.v[:], np.float32).view(np.uint32), a.view(np.uint32))


@pytest.mark.parametrize("pass_index", [0, 1, 7, 1000])
def test_sampler_tables_bit_exact(ctl, orc, pass_index):
    L = ctl.lib()
    nseq, ln = 4096, 30
    a1 = np.zeros(nseq * ln, np.float32)
    a2 = np.zeros(nseq * ln * 2, np.float32)
    b1, b2 = a1.copy(), a2.copy()
    orc.oracle_sampler_tables(pass_index, nseq, ln, oracle.ptr(a1), oracle.ptr(a2))
    assert L.ctl_host_sampler_tables(pass_index, nseq, ln, b1.ctypes.data, b2.ctypes.data) == 0
    assert np.array_equal(a1.view(np.uint32), b1.view(np.uint32))
    assert np.array_equal(a2.view(np.uint32), b2.view(np.uint32))
    assert a1.min() >= 0 and a1.max() < 1


@pytest.mark.parametrize("config", [1, 2, 3])
def test_camera_bit_exact(ctl, orc, config):
    s = ctl.HostScene()
    pos, tar, up = [1.5, 2.25, -7.0], [0.3, 0.1, 4.0], [0.0, 1.0, 0.2]
    s.add_mesh([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]], [ctl.diffuse_material(0.5, 0.5, 0.5)])
    s.add_node(0)
    w, h = [(256, 256), (1280, 720), (1920, 1080)][config - 1]
    s.set_camera(pos, tar, up, 53.0, w, h, near=0.5, far=5000.0)
    d = s.compile()
    cam = ctl._abi.Camera()
    f3 = C.c_float * 3
    orc.oracle_camera(f3(*pos), f3(*tar), f3(*up), 53.0, 0.5, 5000.0, w, h, C.byref(cam))
    assert bytes(cam) == bytes(d.camera)


def test_triangle_data_and_lights_bit_exact(ctl, orc):
    rng = np.random.default_rng(11)
    ntri = 300
    v = rng.normal(size=(ntri * 3, 3)).astype(np.float32) * 5
    idx = np.arange(ntri * 3, dtype=np.uint32).reshape(-1, 3)
    nrm = rng.normal(size=(ntri * 3, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    uv = rng.random((ntri * 3, 2)).astype(np.float32)
    uv[::7] = 0.0   # exercise the half-decode quirk and degenerate UV determinants
    mats = [ctl.diffuse_material(0.5, 0.4, 0.3), ctl.diffuse_material(0.9, 0.9, 0.9)]
    mi = (np.arange(ntri) % 2).astype(np.uint8)
    s = ctl.HostScene()
    s.add_mesh(v, idx, mats, mat_index=mi, normals=nrm, uvs=uv)
    xf = [1.0, 0.1, 0.0, 3.0, 0.0, 2.0, 0.2, -1.0, 0.05, 0.0, 0.5, 0.25, 0.0, 0.0, 0.0, 1.0]
    s.add_node(0, xf)
    s.add_area_light(0, 1, [5.0, 4.0, 3.0])
    s.set_camera([0, 0, -20], [0, 0, 0], [0, 1, 0], 60, 32, 32)
    d = s.compile()
    td = np.ctypeslib.as_array(C.cast(d.tri_data, C.POINTER(C.c_uint32)), shape=(ntri * 8,)).reshape(ntri, 8)
    for t in range(ntri):
        P = v[idx[t]].ravel().copy()
        T = uv[idx[t]].ravel().copy()
        N = nrm[idx[t]].ravel().copy()
        out = np.zeros(8, np.uint32)
        orc.oracle_triangle_data_set(oracle.ptr(P), int(mi[t]), oracle.ptr(T), oracle.ptr(N), oracle.ptr(out))
        assert np.array_equal(out, td[t]), t
    # node inverse transform = float4x4::inverse
    inv = np.zeros(16, np.float32)
    orc.oracle_matrix_inverse(oracle.ptr(np.array(xf, np.float32)), oracle.ptr(inv))
    assert np.array_equal(np.array(d.node_inv_xf[0].m[:], np.float32).view(np.uint32), inv.view(np.uint32))
    # ShapeSet triangles of the light (light material = 1 -> odd triangles)
    assert d.n_lights == 1 and d.lights[0].tri_count == ntri // 2
    woop = np.ctypeslib.as_array(C.cast(d.woop_tris, C.POINTER(C.c_float)), shape=(d.n_woop_tris * 12,)).reshape(-1, 12)
    areas = []
    for k in range(d.n_light_tris):
        lt = d.light_tris[k]
        p9 = np.zeros(9, np.float32)
        n3 = np.zeros(3, np.float32)
        ar = np.zeros(1, np.float32)
        wo = woop[lt.i_dat].copy()
        tdk = td[lt.t_dat].copy()
        orc.oracle_light_tri(oracle.ptr(wo), oracle.ptr(tdk), oracle.ptr(np.array(xf, np.float32)), oracle.ptr(p9),
                             oracle.ptr(n3), oracle.ptr(ar))
        got = np.array([list(r) for r in lt.p], np.float32).ravel()
        assert np.array_equal(got.view(np.uint32), p9.view(np.uint32))
        assert np.array_equal(np.array(lt.n[:], np.float32).view(np.uint32), n3.view(np.uint32))
        assert np.float32(lt.area).view(np.uint32) == ar.view(np.uint32)[0]
        areas.append(ar[0])
    cdf = np.array([d.light_tri_cdf[i] for i in range(d.n_light_tri_cdf)], np.float32)
    assert cdf[0] == 0 and abs(cdf[-1] - 1) < 1e-6 and np.all(np.diff(cdf) >= 0)


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 1.0), (3, 0.01)])
@pytest.mark.parametrize("split", [False, True, "sbvh"])
def test_bvh_layout_contract(ctl, config, scale, split):
    """Reference layout contract (SplitBVHBuilder.cpp:163-203): DFS inner nodes
    (child = index*4), leaves = ~first entry, every triangle referenced (exactly
    once without reference splitting; at least once with it and with the SBVH's
    spatial splits), leaf <= 8, last-in-leaf flags, depth bounded for the
    64-entry stacks.  split: binned builder without / with early split
    clipping, or the SBVH builder (leaf <= 8, the reference's Platform)."""
    s = ctl.HostScene().generate(config, scale, 64, 64)
    if split == "sbvh":
        s.set_bvh_builder("sbvh").set_bvh_params(0.0, 0, 0, 8)
    else:
        s.set_bvh_builder("binned").set_bvh_params(1.0 if split else 0.0, 4 if split else 0, 0, 0)
    d = s.compile()
    for m in range(d.n_meshes):
        km = d.meshes[m]
        nb = km.bvh_node_offset // 4
        nxt = d.meshes[m + 1].bvh_node_offset // 4 if m + 1 < d.n_meshes else d.n_bvh_nodes
        nodes = np.ctypeslib.as_array(C.cast(d.bvh_nodes, C.POINTER(C.c_float)), shape=(d.n_bvh_nodes * 16,)).reshape(-1, 16)[nb:nxt]
        ch = nodes[:, 12:14].copy().view(np.int32)
        e0 = km.bvh_indices_offset
        e1 = d.meshes[m + 1].bvh_indices_offset if m + 1 < d.n_meshes else d.n_tri_indices
        idx = np.ctypeslib.as_array(C.cast(d.tri_indices, C.POINTER(C.c_uint32)), shape=(d.n_tri_indices,))[e0:e1]
        t0 = km.triangle_offset
        t1 = d.meshes[m + 1].triangle_offset if m + 1 < d.n_meshes else d.n_tri_data
        if split:
            assert set((idx >> 1).tolist()) == set(range(t1 - t0))   # each triangle at least once
            assert idx.size <= 16 * (t1 - t0)
        else:
            assert sorted((idx >> 1).tolist()) == list(range(t1 - t0))   # each triangle exactly once
        seen_inner = set()
        stack = [(0, 0)]
        maxdepth = 0
        leaves = 0
        while stack:
            k, dep = stack.pop()
            maxdepth = max(maxdepth, dep)
            assert k not in seen_inner
            seen_inner.add(k)
            for c in ch[k]:
                if c == 0x76543210:
                    continue
                if c >= 0:
                    assert c % 4 == 0
                    stack.append((c // 4, dep + 1))
                else:
                    first = ~c
                    j = first
                    while not (idx[j] & 1):
                        j += 1
                    assert j - first + 1 <= 8
                    leaves += 1
        assert len(seen_inner) == nxt - nb
        assert maxdepth <= 62


def test_wide_bvh_collapse_is_exercised_by_upload_contract(ctl):
    """The scene flag that keeps the reference's binary order is part of the ABI."""
    assert ctl.CTL_SCENE_BINARY_BVH == 2

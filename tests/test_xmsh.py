"""Compiled-mesh files (.xmsh): ctl_host_scene_add_xmsh / ctl_host_scene_write_xmsh
against the reference's byte layout (Engine/Mesh.cpp:46-98 reader, Mesh.cpp:279-288 +
MeshLoader/BVHBuilderHelper.cpp:129-147 writer, leading MeshCompileType from
MeshCompiler.cpp:94).  The reference ships no .xmsh fixture, so the golden stream
below is assembled field by field with `struct` from that layout (parity of the
byte format is pinned by the reference source, not by a file it wrote)."""
import ctypes as C
import struct

import numpy as np
import pytest

from helpers import oracle_render


def _arr(ptr, ctype, n):
    if n == 0:
        return np.zeros(0, np.dtype(ctype))
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), shape=(n,)).copy()


def _desc_arrays(d):
    return {
        "tri": _arr(d.tri_data, C.c_uint32, d.n_tri_data * 8),
        "woop": _arr(d.woop_tris, C.c_uint32, d.n_woop_tris * 12),
        "nodes": _arr(d.bvh_nodes, C.c_uint32, d.n_bvh_nodes * 16),
        "idx": _arr(d.tri_indices, C.c_uint32, d.n_tri_indices),
        "mats": bytes(C.string_at(d.materials, d.n_materials * 80)),
        "scene_bvh": _arr(d.scene_bvh_nodes, C.c_uint32, d.n_scene_bvh_nodes * 16),
        "lights": bytes(C.string_at(d.lights, d.n_lights * C.sizeof(d.lights[0]))) if d.n_lights else b"",
        "light_tris": bytes(C.string_at(d.light_tris, d.n_light_tris * C.sizeof(d.light_tris[0])))
        if d.n_light_tris else b"",
        "box": np.array(list(d.box_min) + list(d.box_max), np.float32),
        "start": d.scene_start_node,
    }


def _random_mesh(rng, ntri):
    v = (rng.normal(size=(ntri * 3, 3)) * 3).astype(np.float32)
    idx = np.arange(ntri * 3, dtype=np.uint32).reshape(-1, 3)
    uv = rng.random((ntri * 3, 2)).astype(np.float32)
    mi = (np.arange(ntri) % 3).astype(np.uint8)
    return v, idx, uv, mi


XF = [1.0, 0.0, 0.2, 1.0, 0.0, 1.5, 0.0, -0.5, 0.1, 0.0, 1.0, 2.0, 0.0, 0.0, 0.0, 1.0]


def _source_scene(ctl, split):
    rng = np.random.default_rng(5)
    v, idx, uv, mi = _random_mesh(rng, 700)
    mats = [ctl.diffuse_material(0.7, 0.6, 0.5), ctl.diffuse_material(0.2, 0.8, 0.3),
            ctl.roughdielectric_material(ctl._abi.CTL_MICROFACET_GGX, 1.5, 0.2)]
    s = ctl.HostScene()
    s.set_bvh_params(0.5 if split else 0.0, 8 if split else 0)
    m = s.add_mesh(v, idx, mats, mat_index=mi, uvs=uv)
    n = s.add_node(m, XF)
    s.add_area_light(n, 1, [4.0, 3.0, 2.0])
    s.set_camera([0, 0, -15], [0, 0, 0], [0, 1, 0], 50, 48, 40)
    return s, s.compile()


@pytest.mark.parametrize("split", [False, True])
def test_write_read_round_trip_bit_exact(ctl, split):
    """write_xmsh -> add_xmsh -> compile reproduces every kernel array, and the
    MeshPartLight written for the lit material recreates the node's light."""
    s, d = _source_scene(ctl, split)
    data = s.write_xmsh(0)
    assert struct.unpack_from("<I", data, 0)[0] == 0          # MeshCompileType::Static
    s2 = ctl.HostScene()
    m = s2.add_xmsh(data)
    s2.add_node(m, XF)                                        # light comes from the file
    s2.set_camera([0, 0, -15], [0, 0, 0], [0, 1, 0], 50, 48, 40)
    d2 = s2.compile()
    a, b = _desc_arrays(d), _desc_arrays(d2)
    for k in a:
        if isinstance(a[k], bytes):
            assert a[k] == b[k], k
        else:
            assert np.array_equal(a[k], b[k]), k
    assert d2.n_lights == 1
    # the stream written from the reloaded scene is the same file
    assert s2.write_xmsh(0) == data


def _golden_stream(ctl, mat_record_size, light_name=b"glow", names=(b"base", b"glow")):
    """An .xmsh built from the reference layout alone: 3 triangles, root inner
    node -> (leaf {0, 1}, leaf {2}), 2 materials with Name at offset 0 of a
    `mat_record_size`-byte record, one MeshPartLight."""
    L = ctl.lib()
    P = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0],
                  [0, 0, 1], [1, 0, 1], [0, 1, 1],
                  [2, 0, 0], [3, 0, 0], [2, 1, 0]], np.float32)
    woop = []
    for t in range(3):
        w = ctl._abi.WoopTri()
        L.ctl_woop_set(P[3 * t].ctypes.data, P[3 * t + 1].ctypes.data, P[3 * t + 2].ctypes.data, C.byref(w))
        woop.append(bytes(w))
    rng = np.random.default_rng(3)
    tri = rng.integers(0, 2 ** 32, size=(3, 8), dtype=np.uint64).astype(np.uint32)
    for t, m in enumerate([0, 1, 0]):
        tri[t, 1] = (tri[t, 1] & ~np.uint32(0xff0000)) | np.uint32(m << 16)
    # BVHNodeData: [lo.x hi.x lo.y hi.y] left, [..] right, [lo.z hi.z lo.z hi.z], [left right 0 0]
    node = struct.pack("<16f", 0, 1, 0, 1, 2, 3, 0, 1, 0, 1, 0, 0, 0, 0, 0, 0)
    node = node[:48] + struct.pack("<iiii", ~0, ~2, 0, 0)
    idx = struct.pack("<III", 0 << 1, (1 << 1) | 1, (2 << 1) | 1)

    def fixed(s, cap):
        return struct.pack("<I", len(s) + 1) + s + b"\0" * (cap - len(s))

    out = struct.pack("<I", 0)
    out += struct.pack("<6f", 0, 0, 0, 3, 1, 1)
    out += struct.pack("<I", 1) + fixed(light_name, 32) + struct.pack("<3f", 6.0, 5.0, 4.0)
    out += struct.pack("<I", 3) + tri.tobytes()
    recs = b""
    for nm in names:
        rec = fixed(nm, 64)
        recs += rec + bytes((0xA5 + i) & 0xff for i in range(mat_record_size - len(rec)))
    out += struct.pack("<I", 2) + recs
    out += struct.pack("<Q", 1) + node
    out += struct.pack("<Q", 3) + b"".join(woop)
    out += struct.pack("<Q", 3) + idx
    return out, tri, node, woop, idx


@pytest.mark.parametrize("record", [148, 1344])
def test_reference_layout_stream(ctl, record):
    data, tri, node, woop, idx = _golden_stream(ctl, record)
    mats = [ctl.diffuse_material(0.5, 0.5, 0.5), ctl.diffuse_material(0.1, 0.1, 0.1)]
    s = ctl.HostScene()
    m = s.add_xmsh(data, materials=mats, material_record_size=record)
    s.add_node(m)
    s.set_camera([1.5, 0.5, -5], [1.5, 0.5, 0], [0, 1, 0], 40, 16, 16)
    d = s.compile()
    a = _desc_arrays(d)
    assert np.array_equal(a["tri"], tri.ravel())
    assert a["nodes"].tobytes() == node
    assert a["woop"].tobytes() == b"".join(woop)
    assert a["idx"].tobytes() == idx
    assert s.write_xmsh(0)[4:28] == data[4:28]       # m_sLocalBox kept as read
    assert np.allclose(a["box"], [0, 0, 0, 3, 1, 1], atol=1e-5)
    # the MeshPartLight "glow" became a DiffuseLight on material 1 of the node
    assert d.n_lights == 1 and list(d.lights[0].radiance) == [6.0, 5.0, 4.0]
    assert d.materials[1].node_light_index == 0 and d.materials[0].node_light_index == 0xffffffff
    assert d.lights[0].tri_count == 1               # one triangle carries material 1


def test_rejects_malformed_streams(ctl):
    good, *_ = _golden_stream(ctl, 148)
    mats = [ctl.diffuse_material(0.5, 0.5, 0.5)] * 2

    def load(data, **kw):
        kw.setdefault("materials", mats)
        kw.setdefault("material_record_size", 148)
        return ctl.HostScene().add_xmsh(data, **kw)

    load(good)
    for bad in (good[:-1], good + b"\0", good[:10], b""):
        with pytest.raises(ctl.CTLError):
            load(bad)
    with pytest.raises(ctl.CTLError, match="Animated|animated"):
        load(struct.pack("<I", 1) + good[4:])
    with pytest.raises(ctl.CTLError, match="material name"):
        load(_golden_stream(ctl, 148, light_name=b"nope")[0])
    with pytest.raises(ctl.CTLError, match="count"):
        load(good, materials=mats[:1])
    with pytest.raises(ctl.CTLError):                # reference records need kernel materials
        load(_golden_stream(ctl, 1344)[0], materials=None, material_record_size=1344)
    # the structure checks: patch the root's children / the entry flags
    node_at = len(good) - (8 + 4 * 3) - (8 + 48 * 3) - 64
    assert struct.unpack_from("<i", good, node_at + 48)[0] == ~0

    def patched(off, fmt, *val):
        b = bytearray(good)
        struct.pack_into(fmt, b, off, *val)
        return bytes(b)

    for kids in [(4, ~2), (0, ~2), (~7, ~2), (3, ~2)]:   # out of range / cycle / bad leaf / misaligned
        with pytest.raises(ctl.CTLError):
            load(patched(node_at + 48, "<ii", *kids))
    with pytest.raises(ctl.CTLError):                  # last entry without its last-in-leaf flag
        load(patched(len(good) - 4, "<I", 2 << 1))
    with pytest.raises(ctl.CTLError):                  # triangle index out of range
        load(patched(len(good) - 4, "<I", (9 << 1) | 1))


def test_write_requires_compile(ctl):
    s = ctl.HostScene()
    s.add_mesh([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]], [ctl.diffuse_material(0.5, 0.5, 0.5)])
    with pytest.raises(ctl.CTLError):
        s.write_xmsh(0)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
def test_xmsh_scene_renders_like_source(ctl, orc, split):
    """A scene loaded from .xmsh renders bit-identically to the scene it was
    written from, on the GPU and in the oracle."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s, d = _source_scene(ctl, split)
    s2 = ctl.HostScene()
    s2.add_node(s2.add_xmsh(s.write_xmsh(0)), XF)
    s2.set_camera([0, 0, -15], [0, 0, 0], [0, 1, 0], 50, 48, 40)
    d2 = s2.compile()
    w, h, passes = 48, 40, 2
    p = ctl.PTParams(1, 8, 3, 1, 64, 1, 0, 0)
    want, wrays = oracle_render(orc, d, p, passes, w, h)
    tr = ctl.PathTracer(0)
    tr.upload_scene(d2)
    tr.params = p
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device="cuda:0")
    tr.reset_rays()
    for i in range(passes):
        tr.do_pass(fb.data_ptr(), i)
    torch.cuda.synchronize()
    got = fb.cpu().numpy()
    assert tr.rays_traced() == wrays
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))

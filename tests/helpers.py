"""Shared helpers for the parity tests (test infrastructure)."""
import ctypes as C

import numpy as np

import oracle


def random_rays(desc, n, seed=0, tmin=0.0, tmax=3.0e38, inside=True):
    """Rays with origins inside the scene box and uniformly random directions (ctl_ray layout)."""
    rng = np.random.default_rng(seed)
    lo = np.array(desc.box_min[:], np.float64)
    hi = np.array(desc.box_max[:], np.float64)
    o = lo + (hi - lo) * rng.random((n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = o
    r[:, 3] = tmin
    r[:, 4:7] = d
    r[:, 7] = tmax
    return r


def camera_rays(desc, w, h, seed=0):
    """Primary rays through jittered pixel centres (PerspectiveSensor, numpy fp64: only inputs)."""
    cam = desc.camera
    tw = np.array(cam.to_world.m[:], np.float64).reshape(4, 4)
    s2c = np.array(cam.sample_to_camera.m[:], np.float64).reshape(4, 4)
    rng = np.random.default_rng(seed)
    ys, xs = np.mgrid[0:h, 0:w]
    px = (xs.ravel() + rng.random(w * h)) / w
    py = (ys.ravel() + rng.random(w * h)) / h
    p = np.stack([px, py, np.zeros_like(px), np.ones_like(px)], 1) @ s2c.T
    p = p[:, :3] / p[:, 3:4]
    d = p / np.linalg.norm(p, axis=1, keepdims=True)
    d = d @ tw[:3, :3].T
    r = np.zeros((w * h, 8), np.float32)
    r[:, 0:3] = tw[:3, 3]
    r[:, 4:7] = d
    r[:, 7] = 3.0e38
    return r


def oracle_intersect(orc, desc, rays, any_hit=False, tie=None, threads=0, trees=None):
    tie = tie_rule(desc, orc, trees) if tie is None else tie
    n = rays.shape[0]
    hits = np.zeros((n, 4), np.int32)
    orc.oracle_intersect(C.byref(desc), n, oracle.ptr(rays), oracle.ptr(hits), 1 if any_hit else 0, tie, threads)
    return hits


def oracle_trace(orc, desc, rays, mode=0, tie=0, threads=0):
    n = rays.shape[0]
    t = np.zeros(n, np.float32)
    u = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    tri = np.zeros(n, np.uint32)
    node = np.zeros(n, np.uint32)
    st = np.zeros(4, np.uint64)
    orc.oracle_trace(C.byref(desc), n, oracle.ptr(rays), mode, tie, oracle.ptr(t), oracle.ptr(u), oracle.ptr(v),
                     oracle.ptr(tri), oracle.ptr(node), oracle.ptr(st), threads)
    return t, u, v, tri, node, st


_WIDE_KEY = [None]


def _addr(p):
    return C.cast(p, C.c_void_p).value or 0


def _sample_digest(desc):
    """Digest of the first and last binary nodes and of the mesh records (a freed
    scene's addresses can be reused by the next one)."""
    import hashlib
    h = hashlib.sha1()
    n = int(desc.n_bvh_nodes)
    for first in (0, max(0, n - 64)):
        k = min(64, n - first)
        if k > 0:
            h.update(C.string_at(_addr(desc.bvh_nodes) + 64 * first, 64 * k))
    if desc.n_meshes:
        h.update(C.string_at(_addr(desc.meshes), 20 * desc.n_meshes))
    if desc.n_scene_bvh_nodes:
        h.update(C.string_at(_addr(desc.scene_bvh_nodes), 64 * min(64, desc.n_scene_bvh_nodes)))
    return h.hexdigest()


def device_wide_trees(tracer, uploaded):
    """The 4-wide trees as the device holds them (after a refit by animate /
    set_transform, whose topology is the uploaded desc's), for tie_rule(trees=)."""
    return tracer.wide_trees(uploaded)


def register_wide(orc, desc, trees=None):
    """Hand the scene's 4-wide trees to the oracle (oracle_set_wide): the given
    (device read-back) trees, else the library's host collapse of desc, which is
    what the upload builds (tests/test_reference_order.py checks the two agree)."""
    import cudatracerlib_amd as ctl
    mesh, wbase, sc = trees if trees is not None else ctl.host_wide_trees(desc)
    orc.oracle_set_wide(C.byref(desc), oracle.ptr(mesh), mesh.shape[0], oracle.ptr(wbase), wbase.size,
                        oracle.ptr(sc), sc.shape[0])


def tie_rule(desc, orc=None, trees=None):
    """Oracle traversal mode matching the device traversal the scene selects:
    the reference's own binary order for CTL_SCENE_BINARY_BVH (0); else the
    product's 4-wide per-ray order (oracle.TRAVERSE_WIDE = 2) over the same
    trees, registered here."""
    if desc.flags & 2:
        return 0
    orc = orc or oracle.load()
    key = (_addr(desc.bvh_nodes), desc.n_bvh_nodes, _addr(desc.scene_bvh_nodes), desc.n_scene_bvh_nodes,
           _addr(desc.tri_indices), desc.n_tri_indices, _addr(desc.meshes), desc.flags & 4, desc.scene_start_node,
           _sample_digest(desc))
    if trees is not None or _WIDE_KEY[0] != key:
        register_wide(orc, desc, trees)
        _WIDE_KEY[0] = None if trees is not None else key
    return 2


def binary_bvh(desc):
    """Copy of a compiled scene desc that selects the reference's binary visit order."""
    d = type(desc).from_buffer_copy(desc)
    d.flags |= 2
    return d


def wide_quant(desc):
    """Copy of a compiled scene desc that selects the 64-B quantized 4-wide nodes."""
    d = type(desc).from_buffer_copy(desc)
    d.flags |= 4
    return d


def select_bvh(desc, bvh):
    return {"wide": desc, "wideq": wide_quant(desc) if bvh == "wideq" else desc,
            "binary": binary_bvh(desc) if bvh == "binary" else desc}[bvh]


def oracle_render(orc, desc, params, passes, w, h, threads=0, fb=None, first_pass=0, trees=None):
    if fb is None:
        fb = np.zeros((w * h, 7), np.float32)
    rays = 0
    for p in range(first_pass, first_pass + passes):
        rays += orc.oracle_render_pass(C.byref(desc), C.byref(params), p, oracle.ptr(fb), tie_rule(desc, orc, trees),
                                       threads, 1,
                                       None)
    return fb, rays


def jitter_landing(orc, pass_index, w, h):
    """Pixel each pixel's pass sample lands on: floor((x, y) + the first 2-D
    SequenceSampler draw), as PathTrace / AddSample compute it (fp32)."""
    nseq, ln = 4096, 30
    s1 = np.zeros(nseq * ln, np.float32)
    s2 = np.zeros(nseq * ln * 2, np.float32)
    orc.oracle_sampler_tables(pass_index, nseq, ln, oracle.ptr(s1), oracle.ptr(s2))
    t = s2.reshape(ln, nseq, 2)[0]
    idx = np.arange(w * h, dtype=np.int64)
    a, b = idx % nseq, (idx // nseq) % nseq
    u = (np.float32(0) + t[a]) + t[b]          # two fp32 adds, as next2()
    u = u - np.floor(u)                        # fracf
    px = (idx % w).astype(np.float32) + u[:, 0]
    py = (idx // w).astype(np.float32) + u[:, 1]
    return np.floor(px).astype(np.int64), np.floor(py).astype(np.int64)


def cross_rank_strays(orc, pass_index, w, h, ranks, tile=64):
    """Number of pixels whose pass sample lands on another rank's tile."""
    lx, ly = jitter_landing(orc, pass_index, w, h)
    idx = np.arange(w * h, dtype=np.int64)
    tx = -(-w // tile)
    own = ((idx // w) // tile * tx + (idx % w) // tile) % ranks
    inside = (lx < w) & (ly < h)
    land = ((ly // tile) * tx + lx // tile) % ranks
    return int(((own != land) & inside).sum())


def grid_room(ctl, offset, n=24, size=4.0, w=64, h=64):
    """Axis-aligned box room translated to `offset`: six walls and three inner
    slabs, each an n x n grid of quads (two triangles), one diffuse material.
    Flat walls made of many triangles whose boxes touch, far from the origin
    when offset is large: the worst case for the slab arithmetic
    (lo * idir - o * idir) and for the Woop t of grazing rays.  Returns
    (host scene, desc); the host scene owns the desc's arrays."""
    verts, idx = [], []
    o = np.array(offset, np.float64)

    def wall(origin, u, v):
        b = len(verts)
        for j in range(n + 1):
            for i in range(n + 1):
                verts.append(origin + u * (i / n) + v * (j / n))
        for j in range(n):
            for i in range(n):
                a = b + j * (n + 1) + i
                idx.append((a, a + 1, a + n + 2))
                idx.append((a, a + n + 2, a + n + 1))

    ex, ey, ez = np.eye(3) * size
    wall(o, ex, ey); wall(o + ez, ey, ex); wall(o, ey, ez)
    wall(o + ex, ez, ey); wall(o, ez, ex); wall(o + ey, ex, ez)
    for k in range(1, 4):
        wall(o + ex * (k / 4) + ey * 0.1 + ez * 0.1, ey * 0.5, ez * 0.5)
    s = ctl.HostScene()
    m = s.add_mesh(np.array(verts, np.float32), np.array(idx, np.uint32), [ctl.diffuse_material(0.5, 0.5, 0.5)])
    s.add_node(m)
    c = o + size / 2
    s.set_camera(tuple(c - [0, 0, size * 0.4]), tuple(c), (0, 1, 0), 60.0, w, h)
    return s, s.compile()


def grazing_rays(desc, offset, n, seed, size=4.0):
    """Rays starting on (or 1e-4 off) the room's walls, nearly parallel to the
    wall they start on (that axis' direction component scaled by 1e-7..1e-2)."""
    rng = np.random.default_rng(seed)
    o = np.array(offset, np.float64)
    orig = o + rng.random((n, 3)) * size
    ax = rng.integers(0, 3, n)
    orig[np.arange(n), ax] = (o[ax] + np.where(rng.random(n) < 0.5, 0.0, size)
                              + rng.normal(0, 1e-4, n) * (rng.random(n) < 0.5))
    d = rng.normal(size=(n, 3))
    d[np.arange(n), ax] *= 10.0 ** rng.uniform(-7, -2, n)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = orig
    r[:, 3] = np.float32(desc.ray_eps)
    r[:, 4:7] = d
    r[:, 7] = 3.0e38
    return r


def classify_orders(ref, other):
    """Per-ray comparison of two batch results (ctl_hit rows): the reference's
    binary order vs another traversal order over the same scene.  ties: same t,
    another triangle (both exact-t candidates; first found differs);
    ref_culled: the other order found a strictly closer hit (a box whose rounded
    slab entry lies past a hit inside it was culled on the reference's path);
    other_culled: the reference found a strictly closer hit; hit_miss: one
    side hit, the other missed."""
    rt, ot = ref[:, 0].view(np.float32), other[:, 0].view(np.float32)
    rh, oh = ref[:, 2] >= 0, other[:, 2] >= 0
    diff = (ref != other).any(axis=1)
    both = rh & oh
    return {"rays": int(ref.shape[0]), "differ": int(diff.sum()),
            "ties": int((diff & both & (rt == ot) & (ref[:, 2] != other[:, 2])).sum()),
            "ref_culled": int((diff & both & (ot < rt)).sum()),
            "other_culled": int((diff & both & (rt < ot)).sum()),
            "hit_miss": int((diff & (rh != oh)).sum()),
            "same_hit_other_fields": int((diff & both & (rt == ot) & (ref[:, 2] == other[:, 2])).sum())}

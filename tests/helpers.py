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


def oracle_intersect(orc, desc, rays, any_hit=False, tie=None, threads=0):
    tie = tie_rule(desc) if tie is None else tie
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


def tie_rule(desc):
    """Oracle tie rule matching the device traversal the scene selects: the
    reference's first-found order for CTL_SCENE_BINARY_BVH, else the wide
    BVH's lowest-(triangle, node) rule (oracle TIE_MIN_INDEX = 1)."""
    return 0 if desc.flags & 2 else 1


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


def oracle_render(orc, desc, params, passes, w, h, threads=0, fb=None, first_pass=0):
    if fb is None:
        fb = np.zeros((w * h, 7), np.float32)
    rays = 0
    for p in range(first_pass, first_pass + passes):
        rays += orc.oracle_render_pass(C.byref(desc), C.byref(params), p, oracle.ptr(fb), tie_rule(desc), threads, 1,
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

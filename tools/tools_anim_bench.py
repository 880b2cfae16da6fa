"""Animated-mesh throughput (ctl_scene_animate): a skinned grid
of N x N quads (2 N^2 triangles, 16 bones, 4 influences per vertex) posed between
two frames; prints one JSON line with ms per animate, per-stage algorithmic bytes
and the resulting rates.  Run under `rocprofv3 --kernel-trace --stats` for the
per-kernel split (profiles/r01_anim_*)."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))   # the repo root


def grid(n, bones):
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


def frames(bones, t):
    out = []
    for k in range(bones):
        a = math.radians(5 * math.sin(t + k))
        m = np.eye(4, dtype=np.float32)
        m[0, 0], m[0, 1], m[1, 0], m[1, 1] = math.cos(a), -math.sin(a), math.sin(a), math.cos(a)
        m[1, 3] = 0.2 * math.sin(t * 0.5 + k)
        out.append(m)
    return np.stack(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--bones", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--binary", action="store_true", help="CTL_SCENE_BINARY_BVH: no 4-wide copy to refit")
    ap.add_argument("--shape", action="store_true", help="also report the tree's depth and the nodes one animate rotates")
    a = ap.parse_args()
    import ctypes as C
    import torch
    import cudatracerlib_amd as ctl

    V, N, BI, BW, T, UV = grid(a.n, a.bones)
    t0 = time.perf_counter()
    s = ctl.HostScene()
    s.add_animated_mesh(V, N, BI, BW, T, [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=UV)
    s.add_node(0)
    s.set_camera([0, 8, -20], [0, 0, 0], [0, 1, 0], 50, 64, 64)
    d = s.compile()
    if a.binary:
        d.flags |= ctl.CTL_SCENE_BINARY_BVH
    t_build = time.perf_counter() - t0
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    f0, f1 = frames(a.bones, 0.0), frames(a.bones, 1.0)
    for _ in range(3):
        pt.animate(0, f0, f1, 0.5)
    torch.cuda.synchronize()
    ms = []
    for k in range(a.iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        pt.animate(0, f0, f1, (k + 0.5) / a.iters)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    nv, nt, ne, nn = V.shape[0], T.shape[0], int(d.n_woop_tris), int(d.n_bvh_nodes)
    shape = {}
    if a.shape:
        from cudatracerlib_amd import _abi
        before = pt.read_array(_abi.CTL_ARRAY_BVH_NODES, 0, nn, np.int32, 16)
        pt.animate(0, f0, f1, 0.37)
        after = pt.read_array(_abi.CTL_ARRAY_BVH_NODES, 0, nn, np.int32, 16)
        shape["nodes_with_new_children"] = int(np.any(before[:, 12:14] != after[:, 12:14], axis=1).sum())
        kids = after[:, 12:14]
        depth = np.zeros(nn, np.int64)   # node depth from the root, by the parent words (d.z)
        order = [0]
        for k in order:
            for c in kids[k]:
                if 0 <= c and c != 0x76543210:
                    depth[c >> 2] = depth[k] + 1
                    order.append(int(c >> 2))
        leaf_depth = [depth[k] + 1 for k in range(nn) for c in kids[k] if c < 0]
        shape.update(max_leaf_depth=int(max(leaf_depth)), mean_leaf_depth=round(float(np.mean(leaf_depth)), 2))
    # algorithmic bytes: skin 40 in + 32 out per vertex; tris 12 idx + 32 in/out + 6 x 16 gathers;
    # woop 4 idx + 12 tri + 3 x 16 gathers + 48 out; refit binary 64 in + 64 out per node + leaf
    # gathers (12 + 48 per triangle), wide about half the nodes at 128 B each
    alg = nv * 72 + nt * (12 + 64 + 96) + ne * (4 + 12 + 48 + 48) + nn * 128 + nt * 60 + (nn // 2) * 256
    per = sorted(ms)[len(ms) // 2]
    print(json.dumps({
        "workload": f"skinned grid {a.n}x{a.n} quads: {nv} vertices, {nt} triangles, {a.bones} bones, 4 influences"
                    + (", binary tree only" if a.binary else ""),
        "ms_per_animate_median": round(per, 4), "ms_min": round(min(ms), 4),
        "mtris_per_s": round(nt / per / 1e3, 1),
        "alg_bytes_per_animate": int(alg), "alg_GBps": round(alg / (per * 1e-3) / 1e9, 1),
        "bvh_nodes": nn, "scene_build_s": round(t_build, 2),
        "note": "includes the epsilon readback (one stream sync) and 2 x 1 KB bone uploads",
        **shape,
    }), flush=True)
    pt.close()


if __name__ == "__main__":
    main()

"""Regression fixtures of the oracle itself: SHA-256 digests of small oracle
renders (C1 PrimTracer first_f, C2 PathTracer Direct 1 / 0, WavefrontPathTracer),
each in the reference's binary visit order (mode 0) and in the product's 4-wide
per-ray order (mode 2, tests/helpers.py tie_rule); the node / triangle visits
of a closest-hit and an any-hit batch in each order (culling changes them even
where the hits stay the same); and the occlusion answers of a shadow-ray set
for each shadow form and cull rule (oracle_occluded).  These are NOT reference outputs (the reference
ships none and cannot be built here): they pin the restatement
against unintended changes, and the GPU parity tests pin the HIP path to it.

    python tests/golden/make_oracle_regression.py   # rewrites oracle_regression.json
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import cudatracerlib_amd as ctl  # noqa: E402
import oracle  # noqa: E402
from helpers import tie_rule  # noqa: E402


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def compute():
    orc = oracle.load()
    out = {}
    hs = ctl.HostScene().generate(1, 1.0, 64, 64)
    d = hs.compile(threads=4)
    hs2 = ctl.HostScene().generate(2, 0.05, 64, 48)
    d2 = hs2.compile(threads=4)
    for name, mode in (("", lambda d: 0), ("_wide", tie_rule)):
        p = ctl.PrimParams(ctl._abi.PRIM_DRAW_MODES.index("first_f"), 7, 1.0, 100000.0, 0)
        fb = np.zeros((64 * 64, 7), np.float32)
        depth = np.zeros(64 * 64, np.float32)
        rays = orc.oracle_prim_pass(C.byref(d), C.byref(p), 0, oracle.ptr(fb), oracle.ptr(depth), mode(d), 4)
        out["c1_prim_first_f_64" + name] = {"fb": digest(fb), "depth": digest(depth), "rays": int(rays)}
        for direct in (1, 0):
            pp = ctl.PTParams(direct, 50, 5, 1, 64, 1, 0, 0)
            fb2 = np.zeros((64 * 48, 7), np.float32)
            r2 = sum(orc.oracle_render_pass(C.byref(d2), C.byref(pp), k, oracle.ptr(fb2), mode(d2), 4, 1, None)
                     for k in range(2))
            out[f"c2_path_direct{direct}_64x48x2" + name] = {"fb": digest(fb2), "rays": int(r2)}
        rays = np.zeros((4096, 8), np.float32)
        rng = np.random.default_rng(7)
        lo, hi = np.array(d2.box_min[:]), np.array(d2.box_max[:])
        rays[:, 0:3] = lo + (hi - lo) * rng.random((4096, 3))
        dd = rng.normal(size=(4096, 3))
        rays[:, 4:7] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
        rays[:, 3] = d2.ray_eps
        rays[:, 7] = np.linalg.norm(hi - lo) * rng.random(4096)
        vis = {}
        for bmode, label in ((1, "closest"), (2, "any")):
            t = np.zeros(4096, np.float32)
            u = np.zeros(4096, np.uint32)
            st = np.zeros(4, np.uint64)
            orc.oracle_trace(C.byref(d2), 4096, oracle.ptr(rays), bmode, mode(d2), oracle.ptr(t), oracle.ptr(t),
                             oracle.ptr(t), oracle.ptr(u), oracle.ptr(u), oracle.ptr(st), 4)
            vis[label] = [int(x) for x in st]
        out["c2_batch_visits" + name] = vis
        occ = {}
        for any_hit, cull, label in ((0, 0, "closest"), (1, oracle.CULL_SLAB, "any_slab"),
                                     (1, oracle.CULL_AT_ACCEPT, "any_accept")):
            o = np.zeros(4096, np.uint8)
            orc.oracle_occluded(C.byref(d2), 4096, oracle.ptr(rays), oracle.ptr(o), any_hit, mode(d2), cull, 4)
            occ[label] = digest(o)
        out["c2_occluded" + name] = occ
        fbw = np.zeros((64 * 48, 7), np.float32)
        rw = orc.oracle_wpt_render_pass(C.byref(d2), 1, 50, 5, 1, 1, oracle.ptr(fbw), mode(d2), 4)
        out["c2_wpt_direct1_64x48" + name] = {"fb": digest(fbw), "rays": int(rw)}
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "oracle_regression.json"), "w") as f:
        json.dump(compute(), f, indent=1, sort_keys=True)
    print("wrote oracle_regression.json")

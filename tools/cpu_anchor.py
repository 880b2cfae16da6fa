"""Anchor of the CPU baseline (the restatement's per-core rate
within +-20 % of the reference's): the oracle's binary-order traversal (mode 0,
the reference's TracerayTemplate host branch + Woop leaf loop) timed on the
workload SURVEY.md §6 recorded for the reference's own host traversal in this
container: a 1 M-triangle random soup, SBVH with leaves <= 8, 2 M rays from one
point, every ray hits; 1 and 8 threads.  The reference measured 0.95 Mrays/s on
1 thread and 1.61 on 8.  SURVEY does not record the soup's triangle sizes; its
SBVH build of the soup duplicated 1.6 % of the references, which rules out
large overlapping triangles (vertices uniform in the cube: the spatial splits
explode), so the soups here are small triangles (vertex offsets N(0, edge)
around centres uniform in the unit cube) of three sizes, and the duplicate rate
and the work per ray (inner-node visits, triangle tests) are reported beside
the rates: the per-thread rate compares only at matching work per ray.
Writes profiles/r06_cpu_anchor.json.  Test infrastructure: runs the oracle only."""
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cudatracerlib_amd as ctl  # noqa: E402
import oracle  # noqa: E402

REF = {"1": 0.95, "8": 1.61}   # Mrays/s, SURVEY.md §6
EDGES = [float(x) for x in os.environ.get("CTL_ANCHOR_EDGES", "0.01,0.003,0.001").split(",")]


def soup(edge, n, rng):
    c = rng.random((n, 1, 3))
    e = rng.normal(size=(n, 3, 3)) * edge
    v = (c + e).reshape(-1, 3).astype(np.float32)
    return v, np.arange(n * 3, dtype=np.uint32).reshape(n, 3)


def main():
    rng = np.random.default_rng(0x5EED)
    orc = oracle.load()
    out = {"reference_mrays_s": REF, "cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count(),
           "workloads": {}}
    try:
        out["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    nrays = 2_000_000
    for edge in EDGES:
        kind = f"soup_edge_{edge:g}"
        v, idx = soup(edge, 1_000_000, rng)
        hs = ctl.HostScene()
        hs.set_bvh_builder("sbvh", 1.0e-5).set_bvh_params(0.0, 8, 0, 8)
        hs.add_mesh(v, idx, [ctl.diffuse_material(0.5, 0.5, 0.5)])
        hs.add_node(0)
        hs.set_camera([0.5, 0.5, -2.0], [0.5, 0.5, 0.5], [0, 1, 0], 60, 64, 64)
        t0 = time.perf_counter()
        d = hs.compile(threads=8)
        tb = time.perf_counter() - t0
        dirs = rng.normal(size=(nrays, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        rays = np.zeros((nrays, 8), np.float32)
        rays[:, 0:3] = 0.5
        rays[:, 4:7] = dirs
        rays[:, 7] = 3.0e38
        rec = {"triangles": 1_000_000, "refs": int(d.n_tri_indices), "inner_nodes": int(d.n_bvh_nodes),
               "duplicate_refs_frac": round(int(d.n_tri_indices) / 1_000_000 - 1.0, 4),
               "build_s_8_threads": round(tb, 2), "rays": nrays}
        for th in (1, 8):
            n = nrays if th > 1 else nrays // 4
            t = np.zeros(n, np.float32)
            u = np.zeros(n, np.float32)
            vv = np.zeros(n, np.float32)
            tri = np.zeros(n, np.uint32)
            node = np.zeros(n, np.uint32)
            st = np.zeros(4, np.uint64)
            r = np.ascontiguousarray(rays[:n])
            t0 = time.perf_counter()
            orc.oracle_trace(C.byref(d), n, oracle.ptr(r), 0, 0, oracle.ptr(t), oracle.ptr(u), oracle.ptr(vv),
                             oracle.ptr(tri), oracle.ptr(node), oracle.ptr(st), th)
            dt = time.perf_counter() - t0
            mr = n / dt / 1e6
            rec[f"threads_{th}"] = {"rays_timed": n, "seconds": round(dt, 3), "mrays_s": round(mr, 3),
                                    "hit_fraction": round(float((tri != 0xFFFFFFFF).mean()), 4),
                                    "inner_visits_per_ray": round(float(st[1]) / n, 2),
                                    "tri_tests_per_ray": round(float(st[2]) / n, 2),
                                    "ratio_to_reference": round(mr / REF[str(th)], 3)}
        out["workloads"][kind] = rec
        print(kind, json.dumps(rec), flush=True)
        hs.close()
    path = os.path.join(ROOT, "profiles", "r06_cpu_anchor.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

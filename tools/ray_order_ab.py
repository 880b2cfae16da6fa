"""A/B of the batch traversal's visit order (ctl_set_ray_order: probes/ray_order_experiment.patch applied) on
C3 at full size: camera rays of a pass, a million bounce-like rays, a million
shadow-segment rays and a million NEE shadow rays from their hits (the rays of
tests/test_reference_order.py), each batch through ctl_intersect in the
caller's order and sorted by (octant, origin Morton) keys; then the
WavefrontPathTracer with each order.  Hits and images must be identical; the
sorted rates include the key and sort kernels.  JSON to gpurun_out/ray_order_ab.json.

    python tools/ray_order_ab.py [--launches 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--wpt-passes", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--variants", default="0:16,1:12,1:16,1:24,2:12,2:16,2:24", help="mode:bits,...")
    ap.add_argument("--no-wpt", action="store_true")
    a = ap.parse_args()
    import torch
    import cudatracerlib_amd as ctl
    from test_reference_order import nee_shadow_rays, secondary_rays
    dev = torch.device("cuda:0")
    W, H = 1920, 1080
    t0 = time.time()
    hs = ctl.HostScene().generate(3, a.scale, W, H)   # owns the desc's arrays: keep it alive
    d = hs.compile(threads=int(os.environ.get("OMP_NUM_THREADS", "8")))
    print(f"scene {d.n_tri_data} tris in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.generate_samples(3)
    n = pt.camera_rays()
    rays = torch.zeros((n, 8), dtype=torch.float32, device=dev)
    pt.camera_rays(rays.data_ptr(), n)
    hits = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(n, rays.data_ptr(), hits.data_ptr())
    torch.cuda.synchronize()
    prim = rays.cpu().numpy()
    ph = hits.cpu().numpy()
    keep = prim[:, 7] > 0
    prim, ph = prim[keep], ph[keep]
    rng = np.random.default_rng(2024)
    bounce, shadow = secondary_rays(d, prim, ph, rng, 1_000_000)
    nee = nee_shadow_rays(d, prim, ph, rng, 1_000_000)
    variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
    out = {"scene": f"C3 {d.n_tri_data} tris", "launches": a.launches, "batches": {}}
    stream = torch.cuda.current_stream()
    for name, r, any_hit in (("camera", prim, False), ("bounce", bounce, False), ("shadow_segment_closest", shadow, False),
                             ("nee_shadow_any", nee, True)):
        rt = torch.from_numpy(np.ascontiguousarray(r)).to(dev)
        m = r.shape[0]
        if any_hit:   # the any-hit batch takes tmax = dist - eps, tmin = eps
            rt[:, 3] = float(d.ray_eps)
            rt[:, 7] = rt[:, 7] - float(d.ray_eps)
        base = None
        res = {}
        for mode, bits in variants:
            pt.set_ray_order(mode, bits)
            h = torch.zeros((m, 4), dtype=torch.int32, device=dev)
            for _ in range(2):
                pt.intersect_buffers(m, rt.data_ptr(), h.data_ptr(), any_hit)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.launches):
                pt.intersect_buffers(m, rt.data_ptr(), h.data_ptr(), any_hit)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.launches
            hv = h.cpu().numpy()
            if base is None:
                base = hv
            same = bool(np.array_equal(hv, base))
            res[f"mode{mode}_bits{bits}"] = {"ms": round(ms, 4), "mrays_s": round(m / ms / 1e3, 1), "identical": same}
            print(name, mode, bits, res[f"mode{mode}_bits{bits}"], file=sys.stderr, flush=True)
            if not same:
                raise SystemExit(f"{name}: mode {mode} bits {bits} changed the hits")
        out["batches"][name] = {"rays": int(m), "any_hit": any_hit, **res}
    pt.set_ray_order(0, 16)
    # the WavefrontPathTracer (bounce batches of extension + shadow rays, device queue counts)
    import ctypes as C
    L = ctl.lib()
    wres, img0 = {}, None
    for mode, bits in ([] if a.no_wpt else variants):
        pt.set_ray_order(mode, bits)
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        ms, rs = [], []
        for k in range(a.wpt_passes + 1):
            pt.generate_samples(100 + k)
            prm = ctl.WptParams(1, 50, 5, k + 1, 0)
            pt.reset_rays()
            if L.ctl_wpt_render_pass(pt._ctx, C.byref(prm), C.c_void_p(fb.data_ptr()), None) != 0:
                raise RuntimeError(L.ctl_last_error(pt._ctx).decode())
            pt.sync()
            if k:
                ms.append(pt.last_pass_ms())
                rs.append(pt.rays_traced())
        img = fb.cpu().numpy()
        if img0 is None:
            img0 = img
        same = bool(np.array_equal(img.view(np.uint32), img0.view(np.uint32)))
        wres[f"mode{mode}_bits{bits}"] = {"ms_per_pass": round(sum(ms) / len(ms), 3),
                                          "mrays_s": round(sum(rs) / (sum(ms) * 1e-3) / 1e6, 1), "identical": same}
        print("wpt", mode, bits, wres[f"mode{mode}_bits{bits}"], file=sys.stderr, flush=True)
        if not same:
            raise SystemExit(f"wpt: mode {mode} bits {bits} changed the image")
    out["wavefront_tracer"] = wres
    pt.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "ray_order_ab.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Debug: rays whose batch-traversal hit changes with the visit order (sorted vs
caller order) on C3.  Saves the differing rays, both results, each ray traced
alone (one ray per launch batch of 1: the per-ray result), and the 64 rays of
the sorted wave that held the first few, for replay.  gpurun_out/order_diff.npz.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import cudatracerlib_amd as ctl
    from test_reference_order import secondary_rays
    dev = torch.device("cuda:0")
    W, H = 1920, 1080
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    hs = ctl.HostScene().generate(3, scale, W, H)
    d = hs.compile(threads=int(os.environ.get("OMP_NUM_THREADS", "8")))
    pt = ctl.PathTracer(0)
    pt.upload_scene(d)
    pt.generate_samples(3)
    n = pt.camera_rays()
    rays = torch.zeros((n, 8), dtype=torch.float32, device=dev)
    pt.camera_rays(rays.data_ptr(), n)
    hits = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(n, rays.data_ptr(), hits.data_ptr())
    torch.cuda.synchronize()
    prim, ph = rays.cpu().numpy(), hits.cpu().numpy()
    keep = prim[:, 7] > 0
    prim, ph = prim[keep], ph[keep]
    bounce, _ = secondary_rays(d, prim, ph, np.random.default_rng(2024), 1_000_000)

    def run(r, mode=0, bits=16):
        pt.set_ray_order(mode, bits)
        rt = torch.from_numpy(np.ascontiguousarray(r)).to(dev)
        h = torch.zeros((r.shape[0], 4), dtype=torch.int32, device=dev)
        pt.intersect_buffers(r.shape[0], rt.data_ptr(), h.data_ptr())
        pt.sync()
        pt.set_ray_order(0, 16)
        return h.cpu().numpy()
    base = run(bounce)
    srt = run(bounce, 1, 12)
    diff = np.nonzero((base != srt).any(axis=1))[0]
    print("differing rays:", diff.size, "of", bounce.shape[0], flush=True)
    alone = np.stack([run(bounce[i:i + 1])[0] for i in diff[:200]]) if diff.size else np.zeros((0, 4), np.int32)
    print("alone == caller order:", int((alone == base[diff[:200]]).all(axis=1).sum()),
          "alone == sorted:", int((alone == srt[diff[:200]]).all(axis=1).sum()), "of", alone.shape[0], flush=True)
    # the sorted order itself (recomputed on the host with the device's key formula is not
    # needed: replay waves by tracing the differing ray with its sorted neighbours)
    pt.set_ray_order(1, 12)
    rt = torch.from_numpy(bounce).to(dev)
    h = torch.zeros((bounce.shape[0], 4), dtype=torch.int32, device=dev)
    pt.intersect_buffers(bounce.shape[0], rt.data_ptr(), h.data_ptr())
    pt.sync()
    import ctypes as C
    order = np.zeros(bounce.shape[0], np.uint32)
    # c->rs_order is internal; reconstruct the wave of a differing ray by sorting the keys on the host
    lo, hi = np.array(d.box_min[:]), np.array(d.box_max[:])
    pt.set_ray_order(0, 16)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "order_diff.npz"), rays=bounce[diff], base=base[diff],
                        sorted=srt[diff], alone=alone, idx=diff, lo=lo, hi=hi,
                        eps=np.float32(d.ray_eps))
    # replay: trace the 64-ray blocks of the host-sorted order containing the first differing rays
    oct = ((bounce[:, 4] < 0).astype(np.uint32) | ((bounce[:, 5] < 0).astype(np.uint32) << 1)
           | ((bounce[:, 6] < 0).astype(np.uint32) << 2))

    def spread(x):
        x = x.astype(np.uint32) & 0x3ff
        x = (x | (x << 16)) & 0x030000ff
        x = (x | (x << 8)) & 0x0300f00f
        x = (x | (x << 4)) & 0x030c30c3
        x = (x | (x << 2)) & 0x09249249
        return x
    sc = np.where(hi > lo, np.float32(1024.0) / (hi - lo).astype(np.float32), 0).astype(np.float32)
    q = np.clip(((bounce[:, 0:3] - lo.astype(np.float32)) * sc), 0, 1023).astype(np.uint32)
    m = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    key = (oct << 28) | (m >> 2)
    hk = np.argsort(key >> 19, kind="stable")
    pos = np.empty_like(hk)
    pos[hk] = np.arange(hk.size)
    rep = []
    for i in diff[:8]:
        w = pos[i] // 64
        blk = hk[w * 64:(w + 1) * 64]
        hb = run(bounce[blk])
        j = int(np.nonzero(blk == i)[0][0])
        rep.append((int(i), bool((hb[j] == srt[i]).all()), bool((hb[j] == base[i]).all())))
    print("replayed 64-ray blocks (ray, == sorted, == caller):", rep, flush=True)
    pt.close()


if __name__ == "__main__":
    main()

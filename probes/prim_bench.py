"""GPU probe: PrimTracer passes (ctl_prim_pass) on the C3 scene at 1920x1080 for a
few draw modes; device ms per pass from ctl_last_pass_ms (first two passes warmup)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import cudatracerlib_amd as ctl

W, H = 1920, 1080
cfg = int(os.environ.get("CFG", "3"))
hs = ctl.HostScene().generate(cfg, 1.0, W, H)
d = hs.compile(threads=16)
dev = torch.device("cuda:0")
fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
for mode in ("first_f", "first_f_direct", "first_non_delta_f_direct"):
    pt = ctl.PrimTracer(0, draw_mode=mode)
    pt.upload_scene(d)
    ms, rays = [], []
    for k in range(10):
        pt.reset_rays()
        pt.do_pass(fb.data_ptr(), k)
        pt.sync()
        if k >= 2:
            ms.append(pt.last_pass_ms())
            rays.append(pt.rays_traced())
    pt.close()
    print(f"C{cfg} {mode}: {sum(ms) / len(ms):.4f} ms/pass, {sum(rays) / sum(ms) / 1e3:.1f} Mrays/s", flush=True)

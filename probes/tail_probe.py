import sys, time, os, json
sys.path.insert(0, os.getcwd())
import torch
import cudatracerlib_amd as ctl
hs = ctl.HostScene().generate(3, 1.0, 1920, 1080)
desc = hs.compile(threads=16)
pt = ctl.PathTracer(0, max_path_length=50, rr_start_depth=5, shadow_any_hit=True, tile_size=64)
pt.upload_scene(desc)
fb = torch.zeros((1920 * 1080, 7), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
res = {}
for G in (1, 1, 2, 4, 8):
    torch.cuda.synchronize()
    pt.reset_rays(s)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(0, 16, G):
        if G == 1:
            pt.generate_samples(100 + k, s); pt.render_pass(fb.data_ptr(), s)
        else:
            pt.render_passes(fb.data_ptr(), 100 + k, G, s)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 16
    rays = pt.rays_traced()
    res[G] = (ms, rays / 16 / ms / 1e3)
    print(G, f"{ms:.3f} ms/pass", f"{rays/16/ms/1e3:.1f} Mrays/s", flush=True)

"""GPU probe: 8-rank sharded C3 render vs the 1-rank render of the same passes
(test_full_size_c4_eight_rank_shards), reporting where they differ."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import cudatracerlib_amd as ctl

W, H = 1920, 1080
N, first = int(os.environ.get("NR", "8")), 64
PASSES = int(os.environ.get("NP", "8"))
dev = torch.device("cuda:0")
hs = ctl.HostScene().generate(3, 1.0, W, H)
d = hs.compile(threads=16)
pt = ctl.PathTracer(0)
pt.upload_scene(d)
def render(nr, r, passes=PASSES):
    pt.params = ctl.PTParams(1, 50, 5, 1, 64, nr, r, 0)
    fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
    pt.reset_rays()
    pt.render_passes(fb.data_ptr(), first, passes)
    pt.sync()
    return fb, pt.rays_traced()
one, r1 = render(1, 0)
one2, _ = render(1, 0)
print("one vs one2 mismatching words:", int((one.view(torch.int32) != one2.view(torch.int32)).sum()))
fbs = [render(N, r)[0] for r in range(N)]
total = fbs[0].clone()
for fb in fbs[1:]:
    total += fb
bad = (total.view(torch.int32) != one.view(torch.int32))
print("sum vs one mismatching words:", int(bad.sum()), "per column", bad.sum(0).tolist())
px = bad.any(1).nonzero().flatten()
print("pixels:", px.numel())
for p in px[:10].tolist():
    owners = [r for r in range(N) if fbs[r][p, 6] > 0]
    print(p, (p % W, p // W), "owners", owners, "total", total[p].tolist(), "one", one[p].tolist())
# do single-pass launches per rank equal?

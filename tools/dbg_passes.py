"""Debug: sequential GPU passes vs the oracle for a given first pass (prints differing pixels)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import cudatracerlib_amd as ctl
import oracle
from helpers import oracle_render
orc = oracle.load()
cfg, scale, w, h = 2, 0.25, 200, 136
s = ctl.HostScene().generate(cfg, scale, w, h)
d = s.compile()
pt = ctl.PathTracer(0)
pt.upload_scene(d)
dev = torch.device("cuda:0")
for first, n in [(0, 1), (5, 1), (1, 1), (2, 1), (3, 1), (4, 1)]:
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    pt.params = p
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    for q in range(first, first + n):
        pt.do_pass(fb.data_ptr(), q)
    torch.cuda.synchronize()
    got = fb.cpu().numpy()
    want, _ = oracle_render(orc, d, p, n, w, h, first_pass=first)
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    print("first", first, "bad", bad.size, bad[:8])
    for b in bad[:3]:
        print("  px", b % w, b // w, "want", want[b], "got", got[b])

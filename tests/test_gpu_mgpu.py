"""Multi-GPU path through the C ABI alone: the RCCL PixelData
reduce (ctl_fb_reduce / ctl_fb_reduce_all) and the one-process driver
examples/mgpu_render.cpp.  The box has one GPU, so the communicators here have
one rank; the N-rank image rule itself (tile shards summing to the 1-GPU image
bit for bit) is tested by test_tile_sharding_exact_with_cross_rank_samples and
the gloo test."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "cudatracerlib_amd", "_lib", "mgpu_render")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_fb_reduce_one_rank_communicator(ctl, dev):
    comms = ctl.comm_init_all([0])
    try:
        pt = ctl.PathTracer(0)
        fb = torch.arange(97 * 7, dtype=torch.float32, device=dev).reshape(97, 7)
        want = fb.clone()
        pt.fb_reduce(comms[0], fb.data_ptr(), 97, root=0)
        torch.cuda.synchronize()
        assert torch.equal(fb, want)
        pt.close()
    finally:
        ctl.comm_destroy(comms[0])


def test_mgpu_driver_matches_single_context(ctl, dev, tmp_path):
    """mgpu_render on every visible GPU (one here): the reduced framebuffer equals
    a single context's ctl_render_passes over the same passes, bit for bit."""
    w, h, steps = 320, 180, 2
    out = str(tmp_path / "fb.bin")
    ndev = torch.cuda.device_count()
    r = subprocess.run([DRIVER, "--config", "2", "--scale", "0.25", "--width", str(w), "--height", str(h),
                        "--steps", str(steps), "--out", out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("devices ")]   # RCCL may print its banner too
    assert len(line) == 1, r.stdout
    fields = line[0].split()
    assert int(fields[1]) == ndev and int(fields[5]) > 0
    got = np.fromfile(out, dtype=np.float32).reshape(w * h, 7)
    hs = ctl.HostScene().generate(2, 0.25, w, h)
    desc = hs.compile()
    pt = ctl.PathTracer(0)
    pt.upload_scene(desc)
    fb = torch.zeros((w * h, 7), dtype=torch.float32, device=dev)
    pt.render_passes(fb.data_ptr(), 0, steps * ndev)
    torch.cuda.synchronize()
    want = fb.cpu().numpy()
    pt.close()
    assert want[:, 6].sum() > 0.99 * w * h * steps * ndev
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))

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
    """ctl_fb_reduce reads the rank framebuffer and writes the sum into a separate
    image: reducing after each of two progressive steps leaves the accumulator as
    a single context's and the last image equal to it."""
    comms = ctl.comm_init_all([0])
    try:
        W, H = 96, 64
        hs = ctl.HostScene().generate(2, 0.05, W, H)
        desc = hs.compile()
        pt = ctl.PathTracer(0)
        pt.upload_scene(desc)
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        img = torch.full_like(fb, -1.0)
        for step in range(2):
            pt.render_passes(fb.data_ptr(), 2 * step, 2)
            pt.fb_reduce(comms[0], fb.data_ptr(), img.data_ptr(), W * H, root=0)
        torch.cuda.synchronize()
        ref = ctl.PathTracer(0)
        ref.upload_scene(desc)
        want = torch.zeros_like(fb)
        ref.render_passes(want.data_ptr(), 0, 2)
        ref.render_passes(want.data_ptr(), 2, 2)
        torch.cuda.synchronize()
        assert torch.equal(fb, want) and torch.equal(img, want)
        with pytest.raises(ctl.CTLError):   # the image may not alias the accumulator
            pt.fb_reduce(comms[0], fb.data_ptr(), fb.data_ptr(), W * H, root=0)
        pt.close()
        ref.close()
    finally:
        ctl.comm_destroy(comms[0])


@pytest.mark.parametrize("reduce_every", [0, 1])
def test_mgpu_driver_matches_single_context(ctl, dev, tmp_path, reduce_every):
    """mgpu_render on every visible GPU (one here): the reduced framebuffer equals
    a single context's ctl_render_passes over the same passes, bit for bit, when
    reduced once at the end and when reduced after every step."""
    w, h, steps = 320, 180, 2
    out = str(tmp_path / "fb.bin")
    ndev = torch.cuda.device_count()
    r = subprocess.run([DRIVER, "--config", "2", "--scale", "0.25", "--width", str(w), "--height", str(h),
                        "--steps", str(steps), "--reduce-every", str(reduce_every), "--out", out],
                       capture_output=True, text=True, timeout=300)
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

"""BASELINE configs[2] (C3) and the C5 scene at their full size: ~10M
triangles (a 24.6M-node binary tree, stacks deeper than the 16 LDS entries,
the scratch part of the lane stack), 1920x1080.  One PathTracer pass on the
GPU, the same pass by the oracle over the whole image: every pixel's
PixelData bit-exact, the traversed-ray count equal, no stack overflow
(ctl_sync), the scene's worst-case stack within the device stack."""
import numpy as np
import pytest

from helpers import binary_bvh, oracle_render

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

torch = pytest.importorskip("torch")

W, H = 1920, 1080
ORACLE_THREADS = 16   # the GPU box's CPU share


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def full_pass(ctl, orc, d, dev, params, pass_index=0):
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        bound = pt.stack_bound()
        assert 0 < bound <= 128
        pt.params = params
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        pt.do_pass(fb.data_ptr(), pass_index)
        pt.sync()                       # raises CTLError on a stack overflow
        got, grays = fb.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()
    want, wrays = oracle_render(orc, d, params, 1, W, H, threads=ORACLE_THREADS, first_pass=pass_index)
    return got, grays, want, wrays, bound


def check(got, grays, want, wrays):
    assert grays == wrays
    assert np.isfinite(got).all()
    assert (want[:, 6] > 0).mean() > 0.999      # AddSample keeps nearly every sample
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad.size, bad[:10], want[bad[:3]], got[bad[:3]])


@pytest.fixture(scope="module")
def c3(ctl):
    hs = ctl.HostScene().generate(3, 1.0, W, H)
    d = hs.compile()
    assert d.n_tri_data > 9_900_000 and d.n_bvh_nodes > 10_000_000   # SBVH (leaf <= 2): 15.3M inner nodes
    yield hs, d
    hs.close()


@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_full_size_c3_pass_bit_exact(ctl, orc, dev, c3, bvh):
    _, d = c3
    d = binary_bvh(d) if bvh == "binary" else d
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    got, grays, want, wrays, bound = full_pass(ctl, orc, d, dev, p, pass_index=3)
    assert bound > 16                  # deeper than the LDS part of the lane stack
    assert grays > 2 * W * H
    check(got, grays, want, wrays)


def test_full_size_c3_closest_hit_shadows(ctl, orc, dev, c3):
    """The reference's own Occluded (closest hit tested against the light
    distance, KernelDynamicScene.cu:70-80) instead of the any-hit shadow rays."""
    _, d = c3
    p = ctl.PTParams(1, 50, 5, 0, 64, 1, 0, 0)
    check(*full_pass(ctl, orc, d, dev, p)[:4])


def test_full_size_c3_batched_passes_equal_sequential(ctl, dev, c3):
    """The bench's launch shape: 8 passes in one ctl_render_passes launch give
    the framebuffer and ray count of 8 ctl_render_pass calls, bit for bit."""
    _, d = c3
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        seq = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        for k in range(8):
            pt.do_pass(seq.data_ptr(), 20 + k)
        pt.sync()
        seq_rays = pt.rays_traced()
        bat = torch.zeros_like(seq)
        pt.reset_rays()
        pt.render_passes(bat.data_ptr(), 20, 8)
        pt.sync()
        assert pt.rays_traced() == seq_rays > 8 * 2 * W * H
        assert torch.equal(seq.view(torch.int32), bat.view(torch.int32))
    finally:
        pt.close()


def test_full_size_c5_pass_bit_exact(ctl, orc, dev, c3):
    c3[0].close()                      # free the C3 host arrays first
    hs = ctl.HostScene().generate(5, 1.0, W, H)
    try:
        d = hs.compile()
        assert d.n_tri_data > 9_900_000 and d.n_textures >= 2
        p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
        check(*full_pass(ctl, orc, d, dev, p)[:4])
    finally:
        hs.close()

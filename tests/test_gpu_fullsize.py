"""BASELINE configs[2] (C3) and the C5 scene at their full size: ~10M
triangles (a 24.6M-node binary tree, stacks deeper than the 16 LDS entries,
the scratch part of the lane stack), 1920x1080.  One PathTracer pass on the
GPU, the same pass by the oracle over the whole image: every pixel's
PixelData bit-exact, the traversed-ray count equal, no stack overflow
(ctl_sync), the scene's worst-case stack within the device stack."""
import ctypes as C
import time

import numpy as np
import pytest

from helpers import binary_bvh, oracle_render, tie_rule

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


def test_full_size_c3_reference_dopass_loop(ctl, dev, c3):
    """The reference's pass loop as a drop-in would drive it: Tracer::DoPass calls
    UpdateKernel, then renders (Kernel/Tracer.h:209-248).  The first of ten
    rounds uploads the scene (ctl_scene_upload); rounds 2..10 call
    ctl_scene_update on the unchanged desc, which must take under 1 ms each (no
    copy, no device sync) and leave the image of ten plain passes."""
    _, d = c3
    pt = ctl.PathTracer(0)
    try:
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        up = []
        pt.reset_rays()
        for k in range(10):
            t0 = time.perf_counter()
            if k == 0:
                pt.upload_scene(d)
            else:
                pt.update_scene(d, 0)
            up.append(time.perf_counter() - t0)
            pt.do_pass(fb.data_ptr(), 40 + k)
        pt.sync()
        loop_rays = pt.rays_traced()
        ref = torch.zeros_like(fb)
        pt.reset_rays()
        pt.render_passes(ref.data_ptr(), 40, 10)
        pt.sync()
        assert pt.rays_traced() == loop_rays
        assert torch.equal(fb.view(torch.int32), ref.view(torch.int32))
    finally:
        pt.close()
    assert up[0] > 0.1                       # the upload copies ~3.5 GB and collapses the trees
    assert max(up[1:]) < 1e-3, up


def eight_rank_shards(ctl, orc, d, dev, first):
    """The scene at 1080p sharded over 8 ranks (tile % 8 == rank,
    IBlockSampler.h:100-108), each rank's 8 passes in one ctl_render_passes
    launch (the bench's N = 8 step): the 8 rank framebuffers sum bit for bit to
    the 1-rank framebuffer of the same passes (every pixel has one owner,
    Image.cu:22-44 adds in the 1-GPU order); rank 0's framebuffer equals the
    oracle's rank-0 render on every 97th pixel; the ranks' rays add up to the
    1-rank count plus the few apron paths a rank traces for its neighbours; no
    stack overflow (ctl_sync)."""
    N = 8
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(d)
        fbs, rays = [], []
        for r in range(N):
            pt.params = ctl.PTParams(1, 50, 5, 1, 64, N, r, 0)
            fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
            pt.reset_rays()
            pt.render_passes(fb.data_ptr(), first, N)
            pt.sync()
            rays.append(pt.rays_traced())
            fbs.append(fb)
        total = fbs[0].clone()
        for fb in fbs[1:]:
            total += fb
        pt.params = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
        one = torch.zeros_like(total)
        pt.reset_rays()
        pt.render_passes(one.data_ptr(), first, N)
        pt.sync()
        one_rays = pt.rays_traced()
        assert torch.equal(total.view(torch.int32), one.view(torch.int32))
        # each pixel is written by exactly one rank
        nz = torch.stack([(fb[:, 6] > 0) for fb in fbs]).sum(0)
        assert int(nz.max()) == 1 and float((nz == 1).float().mean()) > 0.999
        rank0 = fbs[0].cpu().numpy()
    finally:
        pt.close()
    assert one_rays <= sum(rays) <= one_rays * 1.001, (one_rays, sum(rays))
    # rank 0 against the oracle's rank mode, every 97th pixel (sources), on the
    # pixels that received exactly their own sample in every pass
    import oracle
    from helpers import jitter_landing
    want = np.zeros((W * H, 7), np.float32)
    p0 = ctl.PTParams(1, 50, 5, 1, 64, N, 0, 0)
    for p in range(first, first + N):
        orc.oracle_render_pass(C.byref(d), C.byref(p0), p, oracle.ptr(want), tie_rule(d), ORACLE_THREADS, 97, None)
    lin = np.arange(W * H)
    ok = lin % 97 == 0
    for p in range(first, first + N):
        lx, ly = jitter_landing(orc, p, W, H)
        self_land = (lx == lin % W) & (ly == lin // W)
        ok &= self_land
        # no neighbour's sample lands on a checked pixel
        for dx, dy in ((1, 0), (0, 1), (1, 1)):
            src = lin - dx - dy * W
            valid = (src >= 0) & (lin % W >= dx)
            s = np.clip(src, 0, W * H - 1)
            ok &= ~(valid & (lx[s] == lin % W) & (ly[s] == lin // W))
    tiles_x = -(-W // 64)
    owned = (((lin // W) // 64) * tiles_x + (lin % W) // 64) % N == 0
    ok &= owned
    assert ok.sum() > 2000
    assert np.array_equal(rank0[ok].view(np.uint32), want[ok].view(np.uint32))


def test_full_size_c4_eight_rank_shards(ctl, orc, dev, c3):
    """BASELINE configs[3] (C4) on one GPU: the 10M-triangle C3 scene, 8 ranks."""
    eight_rank_shards(ctl, orc, c3[1], dev, 64)


@pytest.fixture(scope="module")
def c5(ctl, c3):
    c3[0].close()                      # free the C3 host arrays first
    hs = ctl.HostScene().generate(5, 1.0, W, H)
    d = hs.compile()
    assert d.n_tri_data > 9_900_000 and d.n_textures >= 2
    yield hs, d
    hs.close()


def test_full_size_c5_pass_bit_exact(ctl, orc, dev, c5):
    p = ctl.PTParams(1, 50, 5, 1, 64, 1, 0, 0)
    check(*full_pass(ctl, orc, c5[1], dev, p)[:4])


def test_full_size_c5_eight_rank_shards(ctl, orc, dev, c5):
    """BASELINE configs[4] (C5: roughdielectric + MIP-mapped textures, 10 M
    triangles, 1080p, 8 GPUs) in its multi-GPU form on one GPU: the full-shading
    path kernel (path_kernel_persistent FULL) renders each rank's 8 passes in one
    launch; the rank images sum bit for bit to the 1-rank image, rank 0 equals the
    oracle's rank render, ray counts add up."""
    eight_rank_shards(ctl, orc, c5[1], dev, 72)

"""PrimTracer (BASELINE configs[0], C1: Cornell box, 256x256, 1 spp, first_f;
Integrators/PrimTracer.cu:19-106, 181-233) through ctl_prim_pass, bit-exact
against the oracle's restatement: PixelData, depth image and ray count, for
every draw mode, on the one-instance and the two-level traversal, plain and
C5 (textured / roughdielectric) shading."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import binary_bvh, tie_rule

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


SCENES = {}


def scene(ctl, config, scale, w, h):
    key = (config, scale, w, h)
    if key not in SCENES:
        s = ctl.HostScene().generate(config, scale, w, h)
        SCENES[key] = (s, s.compile())
    return SCENES[key][1]


def prim_gpu(ctl, d, mode, pass_index, dev, near=1.0, far=100000.0):
    w, h = d.camera.width, d.camera.height
    pt = ctl.PrimTracer(0, draw_mode=mode, near=near, far=far)
    try:
        pt.upload_scene(d)
        fb = torch.full((w * h, 7), 7.0, dtype=torch.float32, device=dev)   # DoPass clears it
        depth = torch.zeros(w * h, dtype=torch.float32, device=dev)
        pt.reset_rays()
        pt.do_pass(fb.data_ptr(), pass_index, depth.data_ptr())
        pt.sync()
        return fb.cpu().numpy(), depth.cpu().numpy(), pt.rays_traced()
    finally:
        pt.close()


def prim_oracle(ctl, orc, d, mode, pass_index, near=1.0, far=100000.0):
    w, h = d.camera.width, d.camera.height
    p = ctl.PrimParams(mode if isinstance(mode, int) else ctl._abi.PRIM_DRAW_MODES.index(mode), 7, near, far, 0)
    fb = np.zeros((w * h, 7), np.float32)
    depth = np.zeros(w * h, np.float32)
    rays = orc.oracle_prim_pass(C.byref(d), C.byref(p), pass_index, oracle.ptr(fb), oracle.ptr(depth), tie_rule(d), 0)
    return fb, depth, rays


def same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("bvh", ["wide", "binary"])
def test_c1_first_f_bit_exact(ctl, orc, dev, bvh):
    """configs[0] as BASELINE names it: Cornell box, 256x256, 1 spp, first_f."""
    d = scene(ctl, 1, 1.0, 256, 256)
    d = binary_bvh(d) if bvh == "binary" else d
    assert d.n_nodes == 8 and d.scene_start_node >= 0   # two-level (one node per shape)
    got, gdep, grays = prim_gpu(ctl, d, "first_f", 0, dev)
    want, wdep, wrays = prim_oracle(ctl, orc, d, "first_f", 0)
    assert grays == wrays == 256 * 256
    assert np.all(want[:, 6] == 1.0)            # every pixel got its sample
    assert want[:, :3].max() > 0.05
    assert same(want, got) and same(wdep, gdep)


@pytest.mark.parametrize("mode", list(range(15)))
@pytest.mark.parametrize("config,scale,w,h", [(1, 1.0, 96, 64), (2, 0.25, 96, 64), (5, 0.003, 96, 64)])
def test_all_draw_modes_bit_exact(ctl, orc, dev, mode, config, scale, w, h):
    d = scene(ctl, config, scale, w, h)
    got, gdep, grays = prim_gpu(ctl, d, mode, 5, dev, near=0.5, far=500.0)
    want, wdep, wrays = prim_oracle(ctl, orc, d, mode, 5, near=0.5, far=500.0)
    assert grays == wrays
    bad = np.nonzero((want.view(np.uint32) != got.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], want[bad[:3]], got[bad[:3]])
    assert same(wdep, gdep)
    if mode in (11, 14):
        assert grays > w * h                   # first_f_direct traces shadow rays


def test_prim_pass_rate(ctl, dev):
    """The C1 pass through the persistent fetch loop, timed (plumbing config)."""
    d = scene(ctl, 1, 1.0, 256, 256)
    pt = ctl.PrimTracer(0)
    pt.upload_scene(d)
    fb = torch.zeros((256 * 256, 7), dtype=torch.float32, device=dev)
    for k in range(3):
        pt.do_pass(fb.data_ptr(), k)
    ms = pt.last_pass_ms()
    pt.close()
    assert 0.0 < ms < 100.0

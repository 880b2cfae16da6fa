"""PrimTracer restatement in the oracle (test infrastructure; CPU): range
properties of the draw modes on the Cornell box (BASELINE configs[0])."""
import ctypes as C

import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def c1(ctl):
    hs = ctl.HostScene().generate(1, 1.0, 128, 128)
    d = hs.compile()
    yield d
    hs.close()


def run(ctl, orc, d, mode, near=1.0, far=100000.0):
    w, h = d.camera.width, d.camera.height
    fb = np.zeros((w * h, 7), np.float32)
    dep = np.zeros(w * h, np.float32)
    p = ctl.PrimParams(ctl._abi.PRIM_DRAW_MODES.index(mode), 7, near, far, 0)
    rays = orc.oracle_prim_pass(C.byref(d), C.byref(p), 0, oracle.ptr(fb), oracle.ptr(dep), 1, 4)
    return fb, dep, rays


def test_first_f_is_albedo_over_pi(ctl, orc, c1):
    fb, dep, rays = run(ctl, orc, c1, "first_f")
    assert rays == 128 * 128 and np.all(fb[:, 6] == 1.0)
    # diffuse f(wi, wo=(0,0,1)) = R / pi on the front side
    assert fb[:, :3].max() <= 1.0 / np.pi + 1e-6 and fb[:, :3].max() > 0.1
    assert np.all((dep > 0) & (dep <= 1.0))


@pytest.mark.parametrize("mode,lo,hi", [("v_absdot_n_geo", 0, 1), ("n_geo_colored", 0, 1), ("n_shade_colored", 0, 1),
                                        ("bary_coords", 0, 1), ("D3D_depth", 0, 1)])
def test_mode_ranges(ctl, orc, c1, mode, lo, hi):
    fb, _, _ = run(ctl, orc, c1, mode)
    assert fb[:, :3].min() >= lo - 1e-6 and fb[:, :3].max() <= hi + 1e-6
    assert fb[:, :3].max() > 0.0


def test_first_f_direct_traces_shadow_rays(ctl, orc, c1):
    fb, _, rays = run(ctl, orc, c1, "first_f_direct")
    assert rays > 128 * 128
    f, _, _ = run(ctl, orc, c1, "first_f")
    assert np.all(fb[:, :3] >= 0.5 * f[:, :3] - 1e-7)   # Le + direct + f/2 >= f/2

"""CTL_PT_RENDER_AHEAD: Tracer::DoPass's host loop (Kernel/Tracer.h:209-248:
UpdateKernel -> sampler tables -> one pass per call) through ctl_render_pass,
rendering the next passes ahead in one launch once the loop is steady.  The
framebuffer after every call equals the one-pass-per-call framebuffer bit for
bit, also when the loop leaves a window early: a scene change, a parameter
change, a pass index that is not the next one, another framebuffer, or another
use of the sample slots drops the pending passes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

W, H = 320, 200


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def scenes(ctl):
    a = ctl.HostScene().generate(2, 0.25, W, H)
    da = a.compile()
    b = ctl.HostScene().generate(2, 0.25, W, H)
    b.set_camera([0.0, 2.5, -9.0], [0.5, 1.0, 0.0], [0, 1, 0], 50.0, W, H)
    db = b.compile()
    yield da, db
    a.close()
    b.close()


def run(ctl, dev, scenes, script, ahead):
    """Executes `script` (a list of (op, arg)) on a fresh tracer; returns the
    framebuffer after every render call and the rays traced."""
    da, db = scenes
    pt = ctl.PathTracer(0)
    fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
    fb2 = torch.zeros_like(fb)
    out = []
    try:
        pt.upload_scene(da)
        base = pt.params.flags
        if ahead:
            pt.params.flags = base | ctl.CTL_PT_RENDER_AHEAD
        pt.reset_rays()
        for op, arg in script:
            if op == "pass":          # DoPass: UpdateKernel (dirty 0) + tables + one pass
                pt.update_scene(da if not getattr(pt, "_b", False) else db, 0)
                pt.do_pass(fb.data_ptr(), arg)
                torch.cuda.synchronize()
                out.append(fb.clone())
            elif op == "camera":      # a new camera in the desc: UpdateKernel copies it
                pt._b = True
            elif op == "shadow":
                pt.params.shadow_any_hit = arg
            elif op == "other_fb":
                pt.do_pass(fb2.data_ptr(), arg)
            elif op == "passes":
                pt.render_passes(fb.data_ptr(), arg, 2)
                torch.cuda.synchronize()
                out.append(fb.clone())
        pt.sync()
        rays = pt.rays_traced()
    finally:
        pt.close()
    return out, rays


def same(ctl, dev, scenes, script):
    plain, rays_plain = run(ctl, dev, scenes, script, False)
    ahead, rays_ahead = run(ctl, dev, scenes, script, True)
    assert len(plain) == len(ahead)
    for k, (a, b) in enumerate(zip(plain, ahead)):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), f"call {k} differs"
    assert rays_ahead >= rays_plain
    return rays_plain, rays_ahead


def test_render_ahead_steady_loop(ctl, dev, scenes):
    """24 DoPass calls: windows of 1, 2, 4, 8, 8 passes, then one of 8 ahead by 1."""
    rays_plain, rays_ahead = same(ctl, dev, scenes, [("pass", p) for p in range(24)])
    assert rays_ahead > rays_plain           # the last window rendered passes 24 .. 29 ahead


@pytest.mark.parametrize("case", ["camera", "shadow", "skip", "other_fb", "slots"])
def test_render_ahead_drops_pending_passes(ctl, dev, scenes, case):
    """Inside the 8-pass window (passes 7 .. 14), the loop changes something at
    pass 9: the pending passes are dropped and every framebuffer still equals
    one pass per call."""
    script = [("pass", p) for p in range(9)]
    if case == "camera":
        script += [("camera", None)] + [("pass", p) for p in range(9, 16)]
    elif case == "shadow":
        script += [("shadow", 0)] + [("pass", p) for p in range(9, 16)]
    elif case == "skip":
        script += [("pass", p) for p in range(12, 19)]
    elif case == "other_fb":
        script += [("other_fb", 9)] + [("pass", p) for p in range(10, 16)]
    elif case == "slots":
        script += [("passes", 40)] + [("pass", p) for p in range(9, 16)]
    same(ctl, dev, scenes, script)


def test_render_ahead_exact_at_window_ends(ctl, dev, scenes):
    """A loop that ends with its last window: the rays equal one pass per call's
    and ctl_render_passes' over the same passes (1 + 2 + 4 + 8 = 15 passes)."""
    da, _ = scenes
    rays_plain, rays_ahead = same(ctl, dev, scenes, [("pass", p) for p in range(15)])
    assert rays_ahead == rays_plain
    pt = ctl.PathTracer(0)
    try:
        pt.upload_scene(da)
        fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
        pt.reset_rays()
        pt.render_passes(fb.data_ptr(), 0, 15)
        pt.sync()
        assert pt.rays_traced() == rays_plain
    finally:
        pt.close()

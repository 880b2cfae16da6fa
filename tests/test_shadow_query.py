"""The NEE shadow query as any-hit gives the image of the reference's
closest-hit `Occluded` (KernelDynamicScene.cu:70-80, PathTracer.cu:40-47).

Closest-hit: occluded iff the nearest hit t satisfies eps < t < dist - eps.
Every triangle test accepts only t > eps (TraceHelper.cu:121 with tmin = eps),
so the nearest hit exists below dist - eps exactly when some hit does, which is
what the any-hit query with t_max = dist - eps answers.  The traversal culls a
box only beyond the current t_max, so neither query can miss an accepted hit.
Checked here on the oracle (the GPU suite checks each mode against it bit for
bit): framebuffers of both modes are identical, so a drop-in user sets
shadow_any_hit = 1 and gets the headline rate."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import oracle_render


@pytest.mark.parametrize("config,scale,w,h", [(1, 1.0, 96, 64), (2, 0.02, 96, 64), (5, 0.002, 96, 64)])
def test_any_hit_shadow_query_equals_closest_hit(ctl, config, scale, w, h):
    orc = oracle.load()
    hs = ctl.HostScene().generate(config, scale, w, h)
    d = hs.compile(threads=4)
    fbs = []
    for any_hit in (1, 0):
        p = ctl.PTParams(1, 50, 5, any_hit, 64, 1, 0, 0)
        fb, _ = oracle_render(orc, d, p, 2, w, h, threads=4)
        fbs.append(fb)
    assert fbs[0][:, 6].sum() > 0
    assert np.array_equal(fbs[0].view(np.uint32), fbs[1].view(np.uint32))

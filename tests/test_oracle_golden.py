"""The oracle (CPU restatement of the reference) against the reference's own
recorded outputs and against BVH-independent truths.  CPU only."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle
from helpers import random_rays, oracle_trace

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_cudarng_matches_reference_recorded_values(orc):
    g = json.load(open(os.path.join(GOLDEN, "sampler_reference_values.json")))
    f = np.zeros(3, np.float32)
    orc.oracle_xorwow_uniforms(7539414, 0, 3, oracle.ptr(f))
    np.testing.assert_allclose(f, g["cudarng_7539414_first_uniforms"], rtol=0, atol=2e-8)


def test_sequence_sampler_pixel0_matches_reference(orc):
    g = json.load(open(os.path.join(GOLDEN, "sampler_reference_values.json")))
    nseq, ln = 4096, 30
    s1 = np.zeros(nseq * ln, np.float32)
    s2 = np.zeros(nseq * ln * 2, np.float32)
    orc.oracle_sampler_tables(0, nseq, ln, oracle.ptr(s1), oracle.ptr(s2))
    o1 = np.zeros(1, np.float32)
    o2 = np.zeros(4, np.float32)
    orc.oracle_sampler_draws(oracle.ptr(s1), oracle.ptr(s2), nseq, ln, 0, 1, oracle.ptr(o1), 2, oracle.ptr(o2))
    np.testing.assert_allclose(o1, g["pass0_pixel0"]["randomFloat"], rtol=0, atol=2e-8)
    np.testing.assert_allclose(o2.reshape(2, 2), g["pass0_pixel0"]["randomFloat2"], rtol=0, atol=2e-8)


def test_xorwow_jump_equals_stepping(orc):
    # offset-jump through GF(2) powers == plain stepping of the same stream
    a = np.zeros(64, np.uint32)
    b = np.zeros(16, np.uint32)
    orc.oracle_xorwow_raw(1234, 7539414, 0, 64, oracle.ptr(a))
    orc.oracle_xorwow_raw(1234, 7539414, 48, 16, oracle.ptr(b))
    assert np.array_equal(a[48:], b)
    # subsequence s+1 == offset 2^67 from s: check via two different subsequences differing
    c = np.zeros(8, np.uint32)
    orc.oracle_xorwow_raw(1234, 7539415, 0, 8, oracle.ptr(c))
    assert not np.array_equal(a[:8], c)


def test_passes_continue_one_stream(orc):
    # pass p+1's first draw is the draw right after pass p's last one (Sampler.h:36-55)
    nseq, ln = 16, 3
    per = nseq * ln * 3
    s1 = np.zeros(nseq * ln, np.float32)
    s2 = np.zeros(nseq * ln * 2, np.float32)
    orc.oracle_sampler_tables(1, nseq, ln, oracle.ptr(s1), oracle.ptr(s2))
    u = np.zeros(2 * per, np.float32)
    orc.oracle_xorwow_uniforms(7539414, 0, 2 * per, oracle.ptr(u))
    # pass 1, sequence 0: first ln draws are the 1-D elements k=0..ln-1 of sequence 0
    assert np.array_equal(s1.reshape(ln, nseq)[:, 0], u[per:per + ln])
    xy = s2.reshape(ln, nseq, 2)[:, 0, :].ravel()
    assert np.array_equal(xy, u[per + ln:per + 3 * ln])


def test_woop_roundtrip(orc):
    rng = np.random.default_rng(3)
    for _ in range(200):
        v = rng.normal(size=(3, 3)).astype(np.float32) * 10
        w = np.zeros(12, np.float32)
        orc.oracle_woop_set(oracle.ptr(v[0]), oracle.ptr(v[1]), oracle.ptr(v[2]), oracle.ptr(w))
        a, b, c = (np.zeros(3, np.float32) for _ in range(3))
        orc.oracle_woop_get(oracle.ptr(w), oracle.ptr(a), oracle.ptr(b), oracle.ptr(c))
        np.testing.assert_allclose(np.stack([a, b, c]), v, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.2), (3, 0.003)])
def test_bvh_traversal_equals_brute_force(ctl, orc, config, scale):
    """The closest hit is a property of the triangle set, not of the BVH:
    oracle traversal over the product's BVH == exhaustive Woop scan."""
    s = ctl.HostScene().generate(config, scale, 64, 64)
    d = s.compile()
    rays = random_rays(d, 20000, seed=config)
    t, u, v, tri, node, st = oracle_trace(orc, d, rays, mode=0)
    n = rays.shape[0]
    bt = np.zeros(n, np.float32)
    btri = np.zeros(n, np.uint32)
    orc.oracle_brute_force(C.byref(d), n, oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
    assert (tri != 0xFFFFFFFF).sum() > n // 10
    assert np.array_equal(t, bt)
    assert np.array_equal(tri, btri)


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.2), (3, 0.003)])
@pytest.mark.parametrize("max_leaf", [8, 2])
def test_sbvh_traversal_equals_brute_force(ctl, orc, config, scale, max_leaf):
    """The SBVH builder (the reference's SplitBVHBuilder: spatial splits with
    clipped references, unsplitting) yields a valid tree over the same
    triangles: traversal == exhaustive Woop scan; references were split."""
    s = ctl.HostScene().generate(config, scale, 64, 64)
    s.set_bvh_builder("sbvh", 1.0e-5).set_bvh_params(0.0, 8, 0, max_leaf)
    d = s.compile()
    rays = random_rays(d, 20000, seed=config + 7)
    t, u, v, tri, node, st = oracle_trace(orc, d, rays, mode=0)
    n = rays.shape[0]
    bt = np.zeros(n, np.float32)
    btri = np.zeros(n, np.uint32)
    orc.oracle_brute_force(C.byref(d), n, oracle.ptr(rays), oracle.ptr(bt), oracle.ptr(btri), 0)
    assert (tri != 0xFFFFFFFF).sum() > n // 10
    assert np.array_equal(t, bt)
    assert np.array_equal(tri, btri)
    if config != 1:
        assert d.n_woop_tris > d.n_tri_data   # spatial splits duplicated references


def test_image_resolve_oracle_matches_numpy(orc):
    """copySamplesToOutput: weight-normalised RGB (+ splat), sRGB curve, clamp,
    truncation to 8 bit (ImagePipeline.cu:8-21, Spectrum.cu:229-234,
    Spectrum.h:521-526) - the oracle against an independent numpy restatement."""
    rng = np.random.default_rng(7)
    n = 5000
    fb = np.zeros((n, 7), np.float32)
    fb[:, 0:3] = rng.random((n, 3), dtype=np.float32) * 3
    fb[:, 3:6] = rng.random((n, 3), dtype=np.float32) * 0.1
    fb[:, 6] = rng.integers(0, 5, n).astype(np.float32)
    out = np.zeros(n, np.uint32)
    orc.oracle_image_resolve(oracle.ptr(fb), n, 1, np.float32(0.25), oracle.ptr(out))
    w = np.where(fb[:, 6] != 0, fb[:, 6], np.float32(1)).astype(np.float32)
    s = fb[:, 0:3] * (np.float32(1) / w)[:, None] + fb[:, 3:6] * np.float32(0.25)
    lin = s <= np.float32(0.0031308)
    srgb = np.where(lin, np.float32(12.92) * s,
                    np.float32(1.055) * np.power(s.astype(np.float64), 1 / 2.4).astype(np.float32) - np.float32(0.055))
    c = (np.clip(srgb, 0, 1).astype(np.float32) * np.float32(255)).astype(np.uint32)
    want = c[:, 0] | (c[:, 1] << 8) | (c[:, 2] << 16) | (255 << 24)
    assert np.array_equal(out, want.astype(np.uint32))


def test_oracle_regression_fixtures():
    """The oracle's own outputs against committed digests (tests/golden/
    make_oracle_regression.py): a regression guard on the restatement, not a
    reference fixture."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_oracle_regression",
                                                  os.path.join(GOLDEN, "make_oracle_regression.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    want = json.load(open(os.path.join(GOLDEN, "oracle_regression.json")))
    assert mod.compute() == want

"""Edge cases of the render loop (camera.go:90-341) on the GPU against the oracle:
degenerate image sizes, non-square spp (camera.go:211-213 truncates to
floor(sqrt)^2), shallow depth limits, ragged row shards, an empty world and a
world without lights.  Tolerances as in test_parity_gpu.py; the small images
make the 8-bit statistics coarse, so the linear-RGB bound carries the check."""
import numpy as np
import pytest

from tests.parity import compare

pytestmark = pytest.mark.gpu


def _render_both(rt, oracle, t, w, l, cam, seed=9, **kw):
    with rt.Scene(t, w, l) as sc:
        img, st = sc.render(cam, seed=seed, **kw)
    ref, ost = oracle.render(t, w, l, cam, seed=seed, threads=8)
    return img, st, ref, ost


@pytest.mark.parametrize("mode", ["fused", "wavefront"])
@pytest.mark.parametrize("width,spp,depth", [
    (1, 1, 0),      # a 1x1 image, one sample
    (7, 10, 0),     # spp 10 -> 3x3 strata, width not a multiple of anything
    (33, 2, 1),     # spp 2 -> 1 sample; MaxDepth 1: one bounce then black
    (20, 16, 2),
    (65, 5, 3),     # a wave of 64 lanes plus one
])
def test_degenerate_sizes(rt, oracle, gpu, width, spp, depth, mode):
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = width, spp
    if depth:
        cam.MaxDepth = depth
    img, st, ref, ost = _render_both(rt, oracle, t, w, l, cam, mode=mode)
    d = cam.derived()
    assert img.shape == ref.shape == (d.height, d.width, 3)
    assert st["samples"] == ost["samples"] == d.width * d.height * d.spp_sqrt ** 2
    assert abs(st["segments"] - ost["segments"]) <= 0.02 * ost["segments"] + 10
    m = compare(img, ref)
    assert m["frac_close"] >= 0.97, m


def test_ragged_row_shards_are_bitwise(rt, gpu):
    """Heights not divisible by the rank count (row r -> rank r % N): the shards
    reassemble to the single-GPU image exactly."""
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel, cam.AspectRatio = 37, 9, 1.3  # H = 28
    H = cam.derived().height
    with rt.Scene(t, w, l) as sc:
        full, _ = sc.render(cam, seed=2)
        for n in (3, 5, 29, 40):  # more ranks than rows: some shards are empty
            rows = 0
            for r in range(n):
                part, st = sc.render(cam, seed=2, rank=r, nranks=n)
                assert np.array_equal(part, full[r::n]), (n, r)
                rows += part.shape[0]
            assert rows == H


def test_empty_world_is_background(rt, oracle, gpu):
    """world.Hit never succeeds: every sample returns the Background (camera.go:300-302)."""
    t = rt.Tree(1)
    world = t.list()
    cam = rt.Camera(Width=16, SamplesPerPixel=4, Background=(0.7, 0.8, 1.0))
    with rt.Scene(t, world, -1) as sc:
        img, st = sc.render(cam, seed=1)
    assert st["segments"] == st["samples"]
    assert np.allclose(img, np.array([0.7, 0.8, 1.0], np.float32), rtol=0, atol=1e-6)
    ref, _ = oracle.render(t, world, -1, cam, seed=1, threads=4)
    assert np.allclose(img, ref, rtol=0, atol=1e-6)


def test_small_negative_samples_in_fixed_point(rt, gpu):
    """Pixel sums take each sample as floor(v * 2^32) in int64 (rt_path.h to_fixed).
    Negative samples work like positive ones; the one corner is (-2^-24, 0), where
    v - floor(v) rounds to 1.0f in fp32: those samples are taken as -2^-24 (a defined
    conversion, error below 2^-24), never as an out-of-range float-to-int cast."""
    t = rt.Tree(1)
    world = t.list()
    bg = (-1e-30, -3e-9, -0.25)
    cam = rt.Camera(Width=8, SamplesPerPixel=9, Background=bg)
    with rt.Scene(t, world, -1) as sc:
        img, st = sc.render(cam, seed=1)
    assert st["overflow_samples"] == 0
    assert np.isfinite(img).all()
    ulp24 = 2.0 ** -24
    assert np.all(np.abs(img[..., 0].astype(np.float64) - bg[0]) <= ulp24)
    assert np.all(np.abs(img[..., 1].astype(np.float64) - bg[1]) <= ulp24)
    assert np.all(img[..., 0] <= 0) and np.all(img[..., 1] <= 0)
    assert np.all(img[..., 2] == np.float32(-0.25))  # exact in fixed point


def test_world_without_lights_list(rt, oracle, gpu):
    """lights = nil-equivalent (-1): the mixture pdf's light half follows the
    reference's empty-list rules (hittable.go:89-103)."""
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 24, 9
    img, st, ref, ost = _render_both(rt, oracle, t, w, t.list(), cam)
    m = compare(img, ref)
    assert m["frac_close"] >= 0.97, m

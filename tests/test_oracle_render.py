"""Oracle self-consistency (CPU): determinism, rank interleaving, and the fp32
twin against the fp64 restatement (statistical)."""
import numpy as np
import pytest

from tests import scenes


def small(rt, name, width=24, spp=9):
    t, cam, w, l = rt.demo_scene(name)
    cam.Width = width
    cam.SamplesPerPixel = spp
    return t, cam, w, l


def test_deterministic(rt, oracle):
    t, cam, w, l = small(rt, "cornell")
    a, _ = oracle.render(t, w, l, cam, seed=5, threads=4)
    b, _ = oracle.render(t, w, l, cam, seed=5, threads=2)
    assert np.array_equal(a, b)
    c, _ = oracle.render(t, w, l, cam, seed=6, threads=4)
    assert not np.array_equal(a, c)


def test_rank_interleave_is_bitwise(rt, oracle):
    t, cam, w, l = small(rt, "book1")
    full, _ = oracle.render(t, w, l, cam, seed=2, threads=4)
    for n in (2, 3):
        for r in range(n):
            part, _ = oracle.render(t, w, l, cam, seed=2, threads=4, rank=r, nranks=n)
            assert np.array_equal(part, full[r::n])


# The naive fp32 twin (reference algorithm, every op in fp32) drifts at Cornell's
# ~555-unit coordinates (+6.7 % segments, -3 % mean: flat boxes and self-hits);
# the HIP path's robustness measures keep it within 0.01 % of fp64 there
# (tests/test_parity_gpu.py).  The twin is checked on small-coordinate scenes.
@pytest.mark.parametrize("name", ["quads", "simple_light"])
def test_fp32_twin_statistics(rt, oracle, name):
    t, cam, w, l = small(rt, name, width=32, spp=16)
    a, sa = oracle.render(t, w, l, cam, seed=3, threads=8, precision=64)
    b, sb = oracle.render(t, w, l, cam, seed=3, threads=8, precision=32)
    assert abs(sa["segments"] - sb["segments"]) <= 0.01 * sa["segments"]
    ma, mb = np.nanmean(a), np.nanmean(b)
    assert abs(ma - mb) <= 0.01 * max(ma, 1e-3)


def clamp_scene(rt, spp=4, maxc=1.5):
    """A diffuse wall filling the view, lit by a very bright quad behind the camera:
    every camera ray's first vertex is a Lambertian clamp vertex (camera.go:328-330),
    so EVERY sample -- and so every pixel mean -- has r+g+b <= MaxContribution, and
    samples whose scattered ray reaches the light are clamped to exactly M."""
    t = rt.Tree(1)
    world = t.list()
    wall = t.lambertian((0.8, 0.6, 0.4))
    t.add(world, t.quad((-50, -50, -5), (100, 0, 0), (0, 100, 0), wall))
    light = t.quad((-20, -20, 10), (0, 40, 0), (40, 0, 0), t.light((1000.0, 900.0, 800.0)))  # faces -z
    t.add(world, light)
    lights = t.list(light)
    cam = rt.Camera(Width=24, SamplesPerPixel=spp, MaxContribution=maxc, VerticalFOV=30)
    cam.PositionCamera((0, 0, 5), (0, 0, -5))
    return t, cam, world, lights


def test_maxcontribution_clamp(rt, oracle):
    t, cam, w, l = clamp_scene(rt)
    img, _ = oracle.render(t, w, l, cam, seed=1, threads=4)
    s = img.astype(np.float64).sum(axis=2)
    assert (s <= 1.5 * (1 + 1e-6)).all(), s.max()
    # the clamp is active: a good share of pixels reach M (every sample clamped there)
    assert (np.abs(s - 1.5) < 1e-5).mean() > 0.05


def test_obj_fixture_is_well_conditioned(rt, oracle):
    """The OBJ feature scene must not decide hits by rounding (coplanar overlapping
    faces would make fp32-vs-fp64 parity meaningless): the fp32 twin agrees."""
    import os
    t, cam, w, l = scenes.build(rt, "obj_mixed",
                                os.path.join(os.path.dirname(scenes.__file__), "..", "assets"))
    a, sa = oracle.render(t, w, l, cam, seed=11, threads=8, precision=64)
    b, sb = oracle.render(t, w, l, cam, seed=11, threads=8, precision=32)
    assert sa["segments"] == sb["segments"]
    close = np.abs(a - b) <= 1e-3 * np.maximum(1.0, np.abs(a))
    assert close.mean() >= 0.999

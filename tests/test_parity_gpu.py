"""GPU (HIP, fp32) vs CPU oracle (fp64 restatement) on the same counter-RNG stream.

Contract, with the tolerance written here:
  * linear RGB: |gpu - oracle| <= 2^-10 * max(1, |oracle|) for >= 99.5 % of channels
  * 8-bit output (PrintColor): equal for >= 99.5 % of channels, within 2 LSB >= 99.9 %
    (P1's "all within 2 LSB" cannot hold at these spp: one forked sample of 9 moves a
    pixel by far more; measured worst 99.96 %, gpurun_out parity logs / DESIGN.md §6)
  * image mean within 0.5 %
Residual mismatches are whole-sample path forks caused by fp32-vs-fp64 rounding
at discrete decisions (dielectric coin, edge hits), each worth 1/spp of a pixel.
"""
import numpy as np
import pytest

from tests.parity import compare

pytestmark = pytest.mark.gpu

CASES = [
    # scene, width, spp, max_depth override (0 = scene default)
    ("cornell", 64, 16, 0),
    ("quads", 48, 9, 0),
    ("book1", 64, 9, 0),
    ("simple_light", 64, 9, 0),
    ("book3", 48, 9, 0),
    ("book2", 48, 9, 0),
    ("cornell_smoke", 48, 9, 0),
    ("model:64x16", 64, 9, 0),
    ("model:384x96", 40, 4, 0),  # 74K triangles: deep BVH, exercises the HBM stack overflow
]


@pytest.mark.parametrize("mode", ["fused", "wavefront"])
@pytest.mark.parametrize("scene,width,spp,depth", CASES)
def test_scene_parity(rt, oracle, gpu, scene, width, spp, depth, mode):
    t, cam, w, l = rt.demo_scene(scene)
    cam.Width = width
    cam.SamplesPerPixel = spp
    if depth:
        cam.MaxDepth = depth
    with rt.Scene(t, w, l) as sc:
        img, st = sc.render(cam, seed=7, mode=mode)
    ref, ost = oracle.render(t, w, l, cam, seed=7, threads=8)
    m = compare(img, ref)
    print(scene, mode, m, st["segments"], ost["segments"])
    assert st["samples"] == ost["samples"]
    assert abs(st["segments"] - ost["segments"]) <= 0.01 * ost["segments"] + 10
    assert m["frac_close"] >= 0.995, m
    assert m["q_equal"] >= 0.995, m
    assert m["q_within2"] >= 0.999, m
    assert abs(m["mean_gpu"] - m["mean_ref"]) <= 5e-3 * max(1.0, abs(m["mean_ref"])), m

"""The device BVH builder (rt_build.hip, PLOC) against the host binned-SAH builder
(host_bvh.cpp).  The closest hit does not depend on the tree (bvh.go:69-82 visits
everything that may hold it), so both trees must give the same segments and, up
to exact ties between coincident surfaces, the same image."""
import numpy as np
import pytest

from tests.parity import compare
from tests.test_scene import bvh_invariants

pytestmark = pytest.mark.gpu


def _scene(rt, tune, builder, name="model:256x32"):
    tune("RT_BVH_BUILDER", builder)
    t, cam, w, l = rt.demo_scene(name)
    return t, cam, w, l, rt.Scene(t, w, l)


@pytest.mark.parametrize("name", ["model:96x24", "book2", "book1"])
def test_device_tree_invariants(rt, gpu, tune, name):
    t, cam, w, l, sc = _scene(rt, tune, "device", name)
    with sc:
        assert sc.info()["bvh_builder"] == 1
        nodes, refs, _ = bvh_invariants(sc)
        again = rt.Scene(t, w, l)
        n2, r2, _, _ = again.export_bvh()
        again.close()
    assert np.array_equal(nodes, n2) and np.array_equal(refs, r2), "device build is deterministic"


@pytest.mark.parametrize("name,width,spp", [("model:256x32", 96, 16), ("book2", 64, 16)])
def test_device_tree_renders_like_host_tree(rt, gpu, tune, name, width, spp):
    imgs, stats = [], []
    for builder in ("host", "device"):
        t, cam, w, l, sc = _scene(rt, tune, builder, name)
        cam.Width, cam.SamplesPerPixel = width, spp
        with sc:
            img, st = sc.render(cam, seed=5)
            assert sc.info()["bvh_builder"] == (builder == "device")
        imgs.append(img)
        stats.append(st)
    m = compare(imgs[1], imgs[0])
    print(name, m, stats[0]["segments"], stats[1]["segments"])
    assert m["frac_close"] >= 0.9999 and m["q_equal"] >= 0.9999, m
    assert abs(stats[0]["segments"] - stats[1]["segments"]) <= 1e-5 * stats[0]["segments"] + 2


def test_auto_builder_threshold(rt, gpu, tune):
    tune("RT_BVH_DEVICE_MIN", "4096")
    t, cam, w, l = rt.demo_scene("model:96x24")  # 4.6k triangles + 2 spheres
    with rt.Scene(t, w, l) as sc:
        assert sc.info()["bvh_builder"] == 1
    tune("RT_BVH_DEVICE_MIN", "100000")
    with rt.Scene(t, w, l) as sc:
        assert sc.info()["bvh_builder"] == 0


@pytest.mark.parametrize("name,width,spp", [("model:256x32", 96, 16), ("book2", 64, 16)])
def test_bvh8_renders_like_bvh4(rt, gpu, tune, name, width, spp):
    """The opt-in BVH8 (RT_BVH8=1, host_bvh8.cpp, 16-bit planes) tests the same leaves
    as the BVH4: the closest hit does not depend on the tree, so the image is the same
    bits (conservative quantisation; ties between coincident surfaces aside).  The BVH8
    kernels are compiled only into A/B builds (-DRT_BVH8_KERNELS): the default
    library keeps rendering the (compressed) BVH4, with the same image, when the BVH8 is built."""
    imgs, widths = [], []
    for v in ("0", "1"):
        tune("RT_BVH8", v)
        t, cam, w, l = rt.demo_scene(name)
        cam.Width, cam.SamplesPerPixel = width, spp
        with rt.Scene(t, w, l) as sc:
            img, st = sc.render(cam, seed=5, mode="fused")
            widths.append(st["tree_width"])
        imgs.append(img)
    # (5: the default library traverses the compressed BVH4 of host_qbvh.cpp)
    assert widths[0] == 5 and widths[1] in (5, 8), widths
    assert np.array_equal(imgs[0], imgs[1], equal_nan=True)

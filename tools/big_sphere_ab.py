"""Dev tool: which change made test_big_spheres_outside_the_bvh_same_image
non-bitwise?  book1 at 64 px, 16 spp (the test's render) with the ground sphere before the
BVH (RT_BIG_SPHERE_R 256) or in it (1e30), on the compressed BVH4 and on the 128-B nodes
(RT_QBVH 1 / 0): differing pixels between each pair, one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402

imgs = {}
for q in ("1", "0"):
    for r in ("256", "1e30"):
        with rt.tuning(RT_BIG_SPHERE_R=r, RT_QBVH=q):
            t, cam, w, l = rt.demo_scene("book1")
            cam.Width, cam.SamplesPerPixel = 64, 16
            with rt.Scene(t, w, l) as sc:
                img, st = sc.render(cam, seed=8)
        imgs[(q, r)] = img
        print(json.dumps({"qbvh": q, "big_r": r, "tree_width": st["tree_width"],
                          "segments": st["segments"]}), flush=True)
def ndiff(a, b):
    return int(np.any(imgs[a] != imgs[b], axis=2).sum())
print(json.dumps({"pixels": int(imgs[("1", "256")].shape[0] * imgs[("1", "256")].shape[1]),
                  "qbvh1_256_vs_1e30": ndiff(("1", "256"), ("1", "1e30")),
                  "qbvh0_256_vs_1e30": ndiff(("0", "256"), ("0", "1e30")),
                  "256_qbvh1_vs_qbvh0": ndiff(("1", "256"), ("0", "256")),
                  "1e30_qbvh1_vs_qbvh0": ndiff(("1", "1e30"), ("0", "1e30"))}), flush=True)

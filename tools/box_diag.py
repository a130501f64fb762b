"""Dev probe: one-launch vs sliced renders of cornell with and without the record loop's box
slab test (RT_BRUTE_BOX): differing channels, overflow samples, non-finite channels."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

W, SPP = int(sys.argv[1]), int(sys.argv[2])
for flag in ("0", "1"):
    rt.tune("RT_BRUTE_BOX", flag)
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = W, SPP
    with rt.Scene(t, w, l) as sc:
        a, sa = sc.render(cam, seed=1)
        b, sb = sc.render(cam, seed=1, progress_slices=16)
        c, sc2 = sc.render(cam, seed=1)
    diff = np.argwhere(a != b)
    print(json.dumps({"box": flag, "differ_ab": int((a != b).sum()), "differ_ac": int((a != c).sum()),
                      "overflow": [sa["overflow_samples"], sb["overflow_samples"]],
                      "nonfinite": int((~np.isfinite(a)).sum()), "max": float(np.nanmax(a)),
                      "first_diffs": diff[:5].tolist(),
                      "vals": [[float(a[tuple(x)]), float(b[tuple(x)])] for x in diff[:5]]}), flush=True)

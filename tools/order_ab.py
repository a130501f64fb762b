#!/usr/bin/env python3
"""A/B of the chunk-group sweep order (dev tool, RT_SWEEP): renders SCENE's rank-0 share of N
rows with each listed order, alternated, and checks every image is bit-identical to the first.
usage: python3 tools/order_ab.py scene width spp nranks forward,reverse [reps]
(round 6 also measured `auto` and `costliest`, a one-sample probe launch's per-group costs,
since removed: profiles/r6_sweep_order_ab.jsonl)
-> one JSON line"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402

scene, width, spp, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
modes = sys.argv[5].split(",")
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1":
    cam.AspectRatio = 1.5
res = {m: [] for m in modes}
ref, same = None, True
with rt.Scene(t, w, l) as sc:
    sc.render(cam, seed=1, nranks=n)
    for _ in range(reps):
        for m in modes:
            with rt.tuning(RT_SWEEP=m):
                img, st = sc.render(cam, seed=1, nranks=n, profile=True)
            res[m].append(round(st["ms_total"], 3))
            if ref is None:
                ref = img
            same = same and bool(np.array_equal(ref.view(np.uint32), img.view(np.uint32)))
base = np.median(res[modes[0]])
print(json.dumps({"scene": scene, "width": width, "spp": spp, "nranks": n, "ms_total": res,
                  "ratio_to_first": {m: round(float(np.median(v) / base), 4) for m, v in res.items()},
                  "bitwise_same": same}), flush=True)

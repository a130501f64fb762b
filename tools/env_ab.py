"""Env-switch A/B (dev tool): one upload-time switch (e.g. RT_BRUTE_VERT) off vs on —
bitwise image comparison at small size for a few scenes, then alternated full-size timings.
usage: env_ab.py VAR[=OFF,ON] OUT.jsonl scene:width:spp [...]   (the first scene is also the
timed one; OFF, ON default to 0, 1)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

var, out_path, specs = sys.argv[1], sys.argv[2], sys.argv[3:]
vals = (0, 1)
if "=" in var:
    var, v = var.split("=")
    vals = tuple(v.split(","))


def render(scene, width, spp, val, seed=3):
    rt.tune(var, val)
    t, cam, w, l = rt.demo_scene(scene)
    cam.Width = width
    with rt.Scene(t, w, l) as sc:
        cam.SamplesPerPixel = 1
        sc.render(cam, seed=seed)
        cam.SamplesPerPixel = spp
        t0 = time.time()
        img, st = sc.render(cam, seed=seed, profile=True)
        return img, st, time.time() - t0


out = open(out_path, "a")
for spec in specs:
    scene = spec.split(":")[0]
    a, _, _ = render(scene, 160, 64, vals[0])
    b, _, _ = render(scene, 160, 64, vals[1])
    rec = {"var": var, "check": "bitwise", "scene": scene,
           "identical": bool(np.array_equal(a, b, equal_nan=True)), "channels_differ": int((a != b).sum())}
    print(json.dumps(rec), flush=True)
    out.write(json.dumps(rec) + "\n")
scene, width, spp = specs[0].split(":")
for rep in range(3):
    for val in vals:
        _, st, dt = render(scene, int(width), int(spp), val)
        rec = {"var": var, "val": val, "scene": scene, "W": int(width), "spp": int(spp),
               "ms_fused": st["ms_fused"], "Msamples_s": round(st["samples"] / dt / 1e6, 2)}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")

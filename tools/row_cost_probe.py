#!/usr/bin/env python3
"""Per-row path cost of a scene (dev tool): renders single rows (rank = row, nranks = height) at
a low spp and prints segments per sample for every STEP-th row -> one JSON line per scene.
Which end of the image is cheap decides how long the render's tail is (the chunks in flight
when the pool empties are the sweep's last rows).
usage: python3 tools/row_cost_probe.py scene width spp step"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402

scene, width, spp, step = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1":
    cam.AspectRatio = 1.5
h = cam.derived().height
segs, ms = [], []
with rt.Scene(t, w, l) as sc:
    for r in range(0, h, step):
        _, st = sc.render(cam, seed=1, rank=r, nranks=h, profile=True)
        segs.append(round(st["segments"] / st["samples"], 3))
        ms.append(round(st["ms_fused"], 3))
print(json.dumps({"scene": scene, "width": width, "height": h, "spp": spp, "step": step,
                  "segments_per_sample": segs, "ms": ms}), flush=True)

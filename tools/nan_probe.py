"""Dev probe: the path trace of one sample of cornell (GPU and oracle), e.g. a sample whose
contribution was NaN (found with a -DRT_NAN_DEBUG build: tools/build_variant.sh nan).
usage: nan_probe.py W SPP GPIX SAMPLE"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

np.set_printoptions(linewidth=220, precision=7, suppress=False)
W, SPP, PIX, S = (int(a) for a in sys.argv[1:5])
t, cam, w, l = rt.demo_scene("cornell")
cam.Width, cam.SamplesPerPixel = W, SPP
with rt.Scene(t, w, l) as sc:
    _, st = sc.render(cam, seed=1, trace=(PIX, S))
g = st["trace"]
for row in g:
    print("o", row[0:3], "d", row[4:7], "k", int(row[7]), "t", row[8], "uv", row[9:11],
          "ref", hex(row[11:12].view(np.uint32)[0]))

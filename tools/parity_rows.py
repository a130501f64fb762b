"""Dev tool: full-size parity of one config on a row subsample, GPU library vs the fp64 oracle
(tests/test_render_gpu.py::test_full_size_parity_on_row_subsample's comparison, for A/B of
libraries and row sets).  The oracle's rows are cached in a .npy so several libraries
(RT_AMD_LIB=...) can be compared against one oracle render.

python3 tools/parity_rows.py SCENE WIDTH SPP STRIDE OFFSET [ASPECT] [CACHE.npy]  -> one JSON line
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import go_raytracer_amd as rt  # noqa: E402
from oracle import pyoracle  # noqa: E402  (dev tool: the checker)
from tests.parity import compare  # noqa: E402

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
scene, width, spp, stride, offset = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
aspect = float(sys.argv[6]) if len(sys.argv) > 6 and sys.argv[6] != "-" else None
cache = sys.argv[7] if len(sys.argv) > 7 else None
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if aspect:
    cam.AspectRatio = aspect
with rt.Scene(t, w, l) as sc:
    img, st = sc.render(cam, seed=1, rank=offset, nranks=stride)
if cache and os.path.exists(cache):
    ref = np.load(cache)
else:
    ref, _ = pyoracle.render(t, w, l, cam, seed=1, threads=16, rank=offset, nranks=stride)
    if cache:
        np.save(cache, ref)
m = compare(img, ref)
print(json.dumps({"scene": scene, "width": width, "spp": spp, "rows": f"{offset}::{stride}",
                  "lib": os.environ.get("RT_AMD_LIB", "in-tree"), "segments": st["segments"], **m}),
      flush=True)

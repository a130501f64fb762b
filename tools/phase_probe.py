#!/usr/bin/env python3
"""Where the fused kernel's waves spend their cycles (dev tool).  Needs a library
built with -DRT_PHASES (tools/build_variant.sh phases -DRT_PHASES; run with
RT_AMD_LIB=go_raytracer_amd/build_abl/phases/librt_amd.so).
usage: phase_probe.py scene width spp  -> one JSON line: phase shares of the loop's
cycles, traversal/shading lane utilisation.  CHUNK=K fixes the chunk size, NRANKS=N renders
rank 0's row share of N"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

NAMES = ["grab", "trav", "media", "shade", "tex", "light", "term", "loop",
         "trav_lanes", "trav_rounds", "shade_lanes", "shade_rounds", "step_lanes", "step_wave",
         "qnode_lanes", "qleaf_lanes", "qmixed", "qiters", "qsame", "quniq", "qtop", "qmid"]
scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
t, cam, w, l = rt.demo_scene(scene)
cam.Width = width
if scene == "book1":
    cam.AspectRatio = 1.5
path = "/tmp/phase_times.bin"
with rt.Scene(t, w, l) as sc:
    cam.SamplesPerPixel = 1
    sc.render(cam)
    cam.SamplesPerPixel = spp
    rt.tune("RT_WAVE_TIMES", path)
    kw = {"chunk": int(os.environ["CHUNK"])} if "CHUNK" in os.environ else {}
    img, st = sc.render(cam, profile=True, nranks=int(os.environ.get("NRANKS", "1")), **kw)
    rt.untune("RT_WAVE_TIMES")
a = np.fromfile(path, dtype=np.uint64).reshape(-1, 4 + len(NAMES)).astype(np.float64)
ph = a[:, 4:].sum(axis=0)
loop = ph[7]
out = {"scene": scene, "W": width, "spp": spp, "ms": round(st["ms_fused"], 2),
       "chunk": st.get("chunk_samples"), "nranks": int(os.environ.get("NRANKS", "1")),
       "segments": st["segments"], "waves": len(a)}
for i in range(7):
    out[NAMES[i]] = round(ph[i] / loop, 4)
out["other"] = round(1 - (ph[0] + ph[1] + ph[2] + ph[3]) / loop, 4)
out["trav_lane_util"] = round(ph[8] / max(ph[9], 1) / 64, 4)
out["shade_lane_util"] = round(ph[10] / max(ph[11], 1) / 64, 4)
out["trav_rounds_per_seg"] = round(ph[9] * 64 / max(st["segments"], 1), 3)
out["steps_per_seg"] = round(ph[12] / max(st["segments"], 1), 2)
out["step_simd_eff"] = round(ph[12] / max(ph[13], 1) / 64, 4)
out["cycles_per_seg_wave"] = round(loop / max(st["segments"], 1), 1)
if ph[17] > 0:  # compressed-BVH kernels: node / leaf lanes per iteration, mixed iterations
    out["q_node_lanes_per_iter"] = round(ph[14] / ph[17], 2)
    out["q_leaf_lanes_per_iter"] = round(ph[15] / ph[17], 2)
    out["q_mixed_iter_frac"] = round(ph[16] / ph[17], 4)
    lanes = ph[14] + ph[15]
    out["q_lanes_on_first_item"] = round(ph[18] / lanes, 4)  # scalar-fetch candidates
    out["q_distinct_items_per_iter"] = round(ph[19] / ph[17], 2)
    out["q_lanes_levels_0_3"] = round(ph[20] / lanes, 4)
    out["q_lanes_levels_4_5"] = round(ph[21] / lanes, 4)
print(json.dumps(out), flush=True)

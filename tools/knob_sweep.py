"""Sweep one tuning knob on one scene, values alternated over reps (dev tool):
python3 tools/knob_sweep.py scene width spp KNOB v1,v2,... [reps]
One JSON line per render (kernel time from the HIP events of the fused launch, and the image
mean, which scheduling knobs must not change).  NRANKS=N renders rank 0's row share of N."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import go_raytracer_amd as rt  # noqa: E402

rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

scene, width, spp, knob = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
values = sys.argv[5].split(",")
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 2
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1":
    cam.AspectRatio = 1.5
nr = int(os.environ.get("NRANKS", "1"))
with rt.Scene(t, w, l) as sc:
    sc.render(cam, seed=1, mode="fused", nranks=nr)
    for _ in range(reps):
        for v in values:
            rt.tune(knob, v)
            img, st = sc.render(cam, seed=1, mode="fused", profile=True, nranks=nr)
            print(json.dumps({"scene": scene, "knob": knob, "value": v, "nranks": nr,
                              "ms_fused": round(st["ms_fused"], 3), "chunk": st["chunk_samples"],
                              "mean": float(img.mean())}), flush=True)
    rt.untune(knob)

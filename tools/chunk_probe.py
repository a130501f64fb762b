"""Kernel ms per fixed chunk size K (opts.chunk) on one config and row share (dev tool):
usage chunk_probe.py scene width spp [nranks]"""
import json, os, sys
sys.path.insert(0, os.getcwd())
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)
scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1": cam.AspectRatio = 1.5
with rt.Scene(t, w, l) as sc:
    sc.render(cam, nranks=n)
    for k in [int(x) for x in os.environ.get("KS", "8,16,32").split(",")]:
        ms = []
        for _ in range(2):
            _, st = sc.render(cam, nranks=n, chunk=k, profile=True)
            ms.append(st["ms_fused"])
        print(json.dumps({"scene": scene, "nranks": n, "chunk": k, "ms": round(min(ms), 2)}), flush=True)

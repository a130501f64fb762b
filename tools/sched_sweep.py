"""Sweep the fused kernel's scheduling knobs (dev tool):
python3 tools/sched_sweep.py scene width spp  budget1,budget2 shade1,shade2"""
import json, os, sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import go_raytracer_amd as rt
rt.tune_from_env()  # dev tool: RT_* knobs from the environment (rt_tune_set)

scene, width, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
budgets = [int(x) for x in sys.argv[4].split(",")]
shades = [int(x) for x in sys.argv[5].split(",")]
t, cam, w, l = rt.demo_scene(scene)
cam.Width, cam.SamplesPerPixel = width, spp
if scene == "book1":
    cam.AspectRatio = 1.5
with rt.Scene(t, w, l) as sc:
    sc.render(cam, seed=1, mode="fused")
    for b in budgets:
        for m in shades:
            rt.tune("RT_STEP_BUDGET", b), rt.tune("RT_SHADE_MIN", m)
            t0 = time.time()
            img, st = sc.render(cam, seed=1, mode="fused")
            dt = time.time() - t0
            print(json.dumps({"scene": scene, "budget": b, "shade_min": m,
                              "Msamples_s": round(st["samples"] / dt / 1e6, 1),
                              "mean": float(img.mean())}), flush=True)
